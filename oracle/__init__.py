"""ORACLE -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package, and only as the checker / the timed CPU baseline.  The product (rlgpu) never
imports, links or executes anything here.  Built by oracle/Makefile into
oracle/build/liboracle.so (plain gcc/g++, strict IEEE float).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
# variant "libm": the same restatement with the host libm in place of the deterministic sin / cos / atan /
# atan2 / asin kernels (include/rlgpu_detmath.h RLGPU_DETMATH_LIBM), for tests/test_detmath_bound.py only
LIB_PATHS = {"": LIB_PATH, "libm": os.path.join(_HERE, "build", "liboracle_libm.so")}
_libs = {}


def lib(variant=""):
    if variant not in _libs:
        path = LIB_PATHS[variant]
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle`")
        _libs[variant] = ctypes.CDLL(path)
    return _libs[variant]


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def gae_flat(rews, terms, vals, trunc_vals, gamma, lam, return_std, clip_range):
    """oracle_gae_flat: GAE.cpp:7-208. Returns (adv, target, ret, clip_portion, status)."""
    rews = np.ascontiguousarray(rews, np.float32)
    terms = np.ascontiguousarray(terms, np.int8)
    vals = np.ascontiguousarray(vals, np.float32)
    tv = None if trunc_vals is None else np.ascontiguousarray(trunc_vals, np.float32)
    n = rews.size
    nt = 0 if tv is None else tv.size
    adv = np.empty(n, np.float32)
    tgt = np.empty(n, np.float32)
    ret = np.empty(n, np.float32)
    clip = ctypes.c_float(0)
    f = lib().oracle_gae_flat
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64] * 2 + [ctypes.c_float] * 4 + \
        [ctypes.c_void_p] * 3 + [ctypes.POINTER(ctypes.c_float)]
    st = f(_p(rews), _p(terms), _p(vals), _p(tv), n, nt, gamma, lam, return_std, clip_range,
           _p(adv), _p(tgt), _p(ret), ctypes.byref(clip))
    return adv, tgt, ret, clip.value, st


def gae_rollout(rews, terms, vals, trunc_vals, boot_vals, gamma, lam, return_std, clip_range):
    rews = np.ascontiguousarray(rews, np.float32)
    T, N = rews.shape
    terms = np.ascontiguousarray(terms, np.int8)
    vals = np.ascontiguousarray(vals, np.float32)
    tv = None if trunc_vals is None else np.ascontiguousarray(trunc_vals, np.float32)
    bv = None if boot_vals is None else np.ascontiguousarray(boot_vals, np.float32)
    adv = np.empty((T, N), np.float32)
    tgt = np.empty((T, N), np.float32)
    ret = np.empty((T, N), np.float32)
    f = lib().oracle_gae_rollout
    f.restype = None
    f.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int32] * 2 + [ctypes.c_float] * 4 + [ctypes.c_void_p] * 3
    f(_p(rews), _p(terms), _p(vals), _p(tv), _p(bv), T, N, gamma, lam, return_std, clip_range,
      _p(adv), _p(tgt), _p(ret))
    return adv, tgt, ret


# ------------------------------------------------------------------ env (rsim_ref.cpp + env_ref.cpp)
OBS, ACTIONS, REWARDS, PADS, MAX_REWARDS = 167, 90, 13, 34, 32


def arena_state_size():
    return lib().oracle_arena_state_size()


class EnvSet:
    """CPU restatement of RLGC::EnvSet with the ExampleMain plugin set (2v2, tickSkip 8, actionDelay 7)."""

    def __init__(self, num_arenas, seed=1234, tick_skip=8, action_delay=7, threads=1, max_episode_steps=0,
                 mesh=None, rewards=None, terminals=None, arith=0, arena_offset=0, state_setter=0, variant=""):
        """mesh: (tris [N, 9] float32 bullet units, object_ntris int32 [K]) or an object with
        .tris / .object_ntris (rlgpu.mesh.ArenaMesh); None = the built-in synthetic mesh.
        rewards / terminals: structured arrays of rlgpu_reward_spec / rlgpu_terminal_spec records
        (include/rlgpu_env.h), None = ExampleMain's lists (the oracle restates them itself).
        arith: the reference build's Bullet arithmetic (include/rlgpu_arith.h: 0 MSVC x64, 1 GCC x86-64,
        2 scalar).  arena_offset: global index of arena 0 (rlgpu_envset_config.arena_offset).
        state_setter: 0 KickoffState, 1 FuzzedKickoffState (rlgpu_envset_config.state_setter).
        variant: "" the oracle, "libm" its host-libm twin (lib())."""
        L = lib(variant)
        L.oracle_env_create.restype = ctypes.c_void_p
        L.oracle_env_create.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int]
        for n in ("oracle_env_destroy", "oracle_env_step_first_half", "oracle_env_reset", "oracle_env_build_obs"):
            getattr(L, n).argtypes = [ctypes.c_void_p]
        L.oracle_env_step_second_half.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_env_step.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.oracle_env_reset_arenas.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_env_get_arenas.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.oracle_env_set_arenas.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.oracle_env_read.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 6
        self.L = L
        self.n = num_arenas
        self.h = L.oracle_env_create(num_arenas, seed, tick_skip, action_delay, threads, arena_offset, int(state_setter))
        L.oracle_env_set_max_episode_steps.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.oracle_env_read_traj_terms.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_env_set_max_episode_steps(self.h, max_episode_steps)
        L.oracle_env_set_arith.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.oracle_env_set_arith(self.h, int(arith))
        if mesh is not None:
            tris, objs = (mesh.tris, mesh.object_ntris) if hasattr(mesh, "tris") else mesh
            self._mesh = (np.ascontiguousarray(tris, np.float32).reshape(-1, 9), np.ascontiguousarray(objs, np.int32))
            L.oracle_env_set_mesh.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
            L.oracle_env_set_mesh(self.h, _p(self._mesh[0]), len(self._mesh[0]), _p(self._mesh[1]), len(self._mesh[1]))
        self.num_rewards = REWARDS
        if rewards is not None or terminals is not None:
            L.oracle_env_set_plugins.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
            self._rw = None if rewards is None else np.ascontiguousarray(rewards)
            self._tc = None if terminals is None else np.ascontiguousarray(terminals)
            nr = 0 if self._rw is None else self._rw.size
            nt = 0 if self._tc is None else self._tc.size
            L.oracle_env_set_plugins(self.h, None if self._rw is None else self._rw.ctypes.data, nr,
                                     None if self._tc is None else self._tc.ctypes.data, nt)
            if self._rw is not None:
                self.num_rewards = nr
        self.traj_terms = np.zeros(4 * num_arenas, np.int8)
        P = 4 * num_arenas
        self.obs = np.zeros((P, OBS), np.float32)
        self.masks = np.zeros((P, ACTIONS), np.uint8)
        self.rewards = np.zeros(P, np.float32)
        self.terminals = np.zeros(num_arenas, np.uint8)
        self.trunc_obs = np.zeros((P, OBS), np.float32)
        self._last_rewards = np.zeros((num_arenas, MAX_REWARDS), np.float32)
        self.read()

    def __del__(self):
        if getattr(self, "h", None):
            self.L.oracle_env_destroy(self.h)
            self.h = None

    def read(self):
        if hasattr(self, "traj_terms"):
            self.L.oracle_env_read_traj_terms(self.h, _p(self.traj_terms))
        self.L.oracle_env_read(self.h, _p(self.obs), _p(self.masks), _p(self.rewards), _p(self.terminals),
                               _p(self.trunc_obs), _p(self._last_rewards))
        self.last_rewards = self._last_rewards[:, :self.num_rewards]

    def step_first_half(self):
        self.L.oracle_env_step_first_half(self.h)

    def step_second_half(self, actions):
        a = np.ascontiguousarray(actions, np.int32)
        self.L.oracle_env_step_second_half(self.h, _p(a))
        self.read()

    def step(self, actions, reset_terminated=True):
        a = np.ascontiguousarray(actions, np.int32)
        self.L.oracle_env_step(self.h, _p(a), int(reset_terminated))
        self.read()

    def reset(self):
        self.L.oracle_env_reset(self.h)
        self.read()

    def reset_arenas(self, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        self.L.oracle_env_reset_arenas(self.h, _p(m))
        self.read()

    def build_obs(self):
        self.L.oracle_env_build_obs(self.h)
        self.read()

    def get_arenas(self, first=0, count=None):
        count = self.n - first if count is None else count
        buf = np.zeros(count * arena_state_size(), np.uint8)
        self.L.oracle_env_get_arenas(self.h, first, count, _p(buf))
        return buf

    def set_arenas(self, buf, first=0):
        buf = np.ascontiguousarray(buf, np.uint8)
        count = buf.size // arena_state_size()
        self.L.oracle_env_set_arenas(self.h, first, count, _p(buf))


def action_table():
    t = np.zeros((ACTIONS, 8), np.float32)
    m = np.zeros((4, ACTIONS), np.uint8)
    lib().oracle_action_table(_p(t), _p(m))
    return t, m


def pad_map():
    m = np.zeros(PADS, np.int32)
    lib().oracle_pad_map(_p(m))
    return m


# ------------------------------------------------------------------ action sampler (sampler_ref.c)
def sample_actions(logits16, masks, deterministic, seed, step, row0=0, f16=False, with_logp=True):
    """oracle_sample_actions: PPOLearner.cpp:78-184 in the GPU sampler's operation order.
    logits16: uint16 [n, A] bf16 (or fp16) bit patterns, or float32 [n, A] logits (the fp32 inference of
    useHalfPrecision = false).  Returns (actions int32 [n], logp f32 [n])."""
    kind = 2 if np.asarray(logits16).dtype == np.float32 else int(f16)
    lg = np.ascontiguousarray(logits16, np.float32 if kind == 2 else np.uint16)
    mk = np.ascontiguousarray(masks, np.uint8)
    n, A = lg.shape
    act = np.empty(n, np.int32)
    lp = np.empty(n, np.float32) if with_logp else None
    f = lib().oracle_sample_actions
    f.restype = None
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                  ctypes.c_uint64, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    f(_p(lg), _p(mk), n, A, int(deterministic), seed, step, row0, kind, _p(act), _p(lp))
    return act, lp


def sampler_probs(logits16, masks, seed, step, row0=0, f16=False):
    """The clamped probs [n, A] the sampler draws from and each row's uniform r [n] (oracle_sampler_probs);
    float32 logits as in sample_actions."""
    kind = 2 if np.asarray(logits16).dtype == np.float32 else int(f16)
    lg = np.ascontiguousarray(logits16, np.float32 if kind == 2 else np.uint16)
    mk = np.ascontiguousarray(masks, np.uint8)
    n, A = lg.shape
    pr = np.empty((n, A), np.float32)
    r = np.empty(n, np.float32)
    f = lib().oracle_sampler_probs
    f.restype = None
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                  ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    f(_p(lg), _p(mk), n, A, seed, step, row0, kind, _p(pr), _p(r))
    return pr, r


TRIG_OPS = {"sin": 0, "cos": 1, "atan2": 2, "asin": 3, "atan": 4}


def detmath_trig(op, x, y=None, variant=""):
    """rs_sinf / rs_cosf / rs_atan2f(y, x) / rs_asinf / rs_atanf (include/rlgpu_detmath.h) over an array;
    variant "libm" gives the host libm's sinf / cosf / atan2f / asinf / atanf instead."""
    x = np.ascontiguousarray(x, np.float32)
    yy = np.ascontiguousarray(x if y is None else y, np.float32)
    out = np.empty_like(x)
    f = lib(variant).oracle_detmath_trig
    f.restype = None
    f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    f(TRIG_OPS[op], _p(x), _p(yy), x.size, _p(out))
    return out


def set_libm_sites(mask):
    """Which call sites (include/rlgpu_detmath.h RS_SITE_* bits, -1 = all) the "libm" variant swaps libm in at."""
    f = lib("libm").oracle_set_libm_sites
    f.restype = None
    f.argtypes = [ctypes.c_int]
    f(int(mask) & 0x7FFFFFFF if mask != -1 else 0x7FFFFFFF)


def detmath_exp_log(x):
    """rs_expf / rs_logf (include/rlgpu_detmath.h) over an array."""
    x = np.ascontiguousarray(x, np.float32)
    ex, lg = np.empty_like(x), np.empty_like(x)
    f = lib().oracle_detmath_exp_log
    f.restype = None
    f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
    f(_p(x), x.size, _p(ex), _p(lg))
    return ex, lg


def mesh_edge_info(tris, object_ntris=None, arith=0):
    """oracle_mesh_edge_info: btGenerateInternalEdgeInfo restated (edge_ref.hpp) -> [ntris, 4] float32
    (m_edgeV0V1Angle, m_edgeV1V2Angle, m_edgeV2V0Angle, flags bits | 1 << 30 with a record)."""
    tris = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    objs = None if object_ntris is None else np.ascontiguousarray(object_ntris, np.int32)
    out = np.zeros((len(tris), 4), np.float32)
    f = lib().oracle_mesh_edge_info
    f.restype = None
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    f(_p(tris), len(tris), _p(objs), 0 if objs is None else len(objs), int(arith), _p(out))
    return out


def car_box_shape():
    """The Octane hitbox as btBoxShape holds it -> (implicit half extents [3], margin, half extents with
    margin [3]) (btBoxShape.cpp:18-26 + setSafeMargin, btConvexInternalShape.h:63-78)."""
    impl, half, m = np.zeros(3, np.float32), np.zeros(3, np.float32), np.zeros(1, np.float32)
    f = lib().oracle_car_box_shape
    f.restype = None
    f.argtypes = [ctypes.c_void_p] * 3
    f(_p(impl), _p(m), _p(half))
    return impl, float(m[0]), half


def box_triangle(rot, centre, tri, cbt, arith=0):
    """oracle_box_triangle (gjk_ref.hpp): n car-hitbox vs triangle queries as Bullet runs them (normal
    early out, GJK with margins, GJK/EPA penetration solver, normal fix).  rot [n,3,3] rows, centre [n,3],
    tri [n,3,3], cbt [n] -> (out [n,8] = hit, normal, point, depth; counts [2] = GJK queries, penetration-
    solver calls)."""
    rot = np.ascontiguousarray(rot, np.float32).reshape(-1, 9)
    n = len(rot)
    centre = np.ascontiguousarray(centre, np.float32).reshape(n, 3)
    tri = np.ascontiguousarray(tri, np.float32).reshape(n, 9)
    cbt = np.ascontiguousarray(np.broadcast_to(np.asarray(cbt, np.float32), (n,)))
    out = np.zeros((n, 8), np.float32)
    counts = np.zeros(2, np.uint64)
    f = lib().oracle_box_triangle
    f.restype = None
    f.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 6 + [ctypes.c_int]
    f(n, _p(rot), _p(centre), _p(tri), _p(cbt), _p(out), _p(counts), int(arith))
    return out, counts


def gjk_counts():
    """This thread's box-triangle GJK queries, penetration-solver calls, EPA runs, EPA iterations, most
    iterations of one EPA run and most polytope faces one run took, inside oracle arena steps and
    box_triangle() calls since the last call (diagnostics)."""
    c = np.zeros(6, np.uint64)
    f = lib().oracle_gjk_counts
    f.restype = None
    f.argtypes = [ctypes.c_void_p]
    f(_p(c))
    return c


def box_box(rot_a, centre_a, rot_b, centre_b):
    """oracle_box_box (boxbox_ref.hpp, btBoxBoxDetector / dBoxBox2): n car-vs-car hitbox queries ->
    [n, 29] float32 = count, then up to 4 x (normal on B xyz, point xyz, depth)."""
    rot_a = np.ascontiguousarray(rot_a, np.float32).reshape(-1, 9)
    n = len(rot_a)
    rot_b = np.ascontiguousarray(rot_b, np.float32).reshape(n, 9)
    centre_a = np.ascontiguousarray(centre_a, np.float32).reshape(n, 3)
    centre_b = np.ascontiguousarray(centre_b, np.float32).reshape(n, 3)
    out = np.zeros((n, 29), np.float32)
    f = lib().oracle_box_box
    f.restype = None
    f.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 5
    f(n, _p(rot_a), _p(centre_a), _p(rot_b), _p(centre_b), _p(out))
    return out


def bvh_order(tris, object_ntris=None):
    """oracle_bvh_order (bvh_ref.hpp): per collision object, the order its quantized BVH visits the
    triangles -> [ntris] int32, out[k] = the mesh triangle visited k-th (each object's range permuted
    within itself)."""
    tris = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    counts = [len(tris)] if object_ntris is None else [int(c) for c in object_ntris]
    out = np.zeros(len(tris), np.int32)
    f = lib().oracle_bvh_order
    f.restype = None
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    t0 = 0
    for c in counts:
        if c:
            part = np.ascontiguousarray(tris[t0:t0 + c])
            o = np.zeros(c, np.int32)
            f(_p(part), c, _p(o))
            out[t0:t0 + c] = o + t0
        t0 += c
    return out


# ------------------------------------------------------------------ x86 arithmetic (rsim_math.hpp)
def rsqrtss(x):
    """This host's rsqrtss instruction over an array (btVector3::normalize's estimate)."""
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty_like(x)
    f = lib().oracle_rsqrtss
    f.restype = None
    f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    f(_p(x), x.size, _p(out))
    return out


def has_sse41_fma3():
    return bool(lib().oracle_has_sse41_fma3())


def dpps(a, b, restated=False):
    """_mm_dp_ps(a, b, 0x7f) on [n, 3] rows (the instruction), or its restatement (x + y) + (z + 0)."""
    a = np.ascontiguousarray(a, np.float32).reshape(-1, 3)
    b = np.ascontiguousarray(b, np.float32).reshape(-1, 3)
    out = np.empty(len(a), np.float32)
    f = lib().oracle_dpps_restated if restated else lib().oracle_dpps
    f.restype = None
    f.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int64, ctypes.c_void_p]
    f(_p(a), _p(b), len(a), _p(out))
    return out


def fmadd(a, b, c, restated=False):
    """_mm_fmadd_ss (the instruction) or std::fma over arrays."""
    a, b, c = (np.ascontiguousarray(v, np.float32) for v in (a, b, c))
    out = np.empty_like(a)
    f = lib().oracle_fma_restated if restated else lib().oracle_fmadd
    f.restype = None
    f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_void_p]
    f(_p(a), _p(b), _p(c), a.size, _p(out))
    return out


def linear_math(op, arith, inp):
    """oracle_linear_math: the mode-dependent LinearMath operation `op` (0 normalize, 1 setRotation,
    2 getRotation, 3 quaternion product, 4 integrateTransform, 5 wheel-ray convex cast) on rows of 24 floats
    -> [n, 12]."""
    inp = np.ascontiguousarray(inp, np.float32).reshape(-1, 24)
    out = np.zeros((len(inp), 12), np.float32)
    f = lib().oracle_linear_math
    f.restype = None
    f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    f(int(op), int(arith), _p(inp), len(inp), _p(out))
    return out
