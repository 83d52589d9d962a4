"""bench.py -- BASELINE.json metric on MI355X: env-steps/s (whole job) and PPO wall-clock per
1M agent-steps for the C2 workload: 4096 arenas per GPU (2v2, tickSkip 8 / actionDelay 7,
ExampleMain plugin set), rollout T = 128, actor/critic MLP [512, 512] (bf16 inference, fp32
training), PPO epochs 2, minibatch 50k, AdamW.

Contract (driver): python bench.py --gpus N --steps K --warmup W ; for N > 1 launched by
torch.distributed.run, one rank per GPU over RCCL.  Rank 0 prints ONE JSON line.

The loop is the C++ host Learner (reinforcement-learning_amd/host/learner.cpp, GGL::Learner over
the C ABI), driven through rlgpu.learner.  A "step" is one PPO iteration of every rank: T = 128 env steps of all arenas (bf16 policy
inference + fused env kernel with experience append), critic over the rollout, GAE, then
Learn (2 epochs of shuffled 50k minibatches, fp32 forward/backward, RCCL gradient all-reduce
for N > 1, clip_grad_norm_, AdamW).  value = env-steps/s summed over ranks (weak scaling:
4096 arenas per GPU).  Synthetic inputs: random-init weights (seed 123), Philox kickoffs.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-learning_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8 TB/s peak
MFMA_F16_TFS = 2500.0   # dense fp16 MFMA peak (MI355X_MICROARCH.md; no sparsity)
H3_TFS = MFMA_F16_TFS / 3  # fp32 GEMM ceiling of the H3 split: three fp16 MFMAs per fp32 product
ARENAS_PER_GPU = 4096   # BASELINE configs[1] (C2)


def env_bytes_per_step(arena_state_size, append=True, output_only=True):
    """B_env = 2*S_arena + 16 (actions) + 2672 (obs) + 360 (masks) + 16 (rewards) + 1
    (terminal); the fused step's experience append writes the reward / terminal-code rows into the rollout
    buffer (+16 + 4) and the obs / mask rows a second time (+2672 + 360) -- unless the env set is output-only
    (rlgpu_envset_set_output_only, the C++ Learner's mode since round 6): then the rollout rows are the step's
    only obs / mask output and they are counted once."""
    b = 2 * arena_state_size + 16 + 4 * 167 * 4 + 4 * 90 + 16 + 1
    if append:
        b += 16 + 4
        if not output_only:
            b += 4 * 167 * 4 + 4 * 90
    return b


# The env kernel's PMC summary of the committed HEAD (tools/pmc_summary.py over separate FETCH_SIZE /
# WRITE_SIZE rocprofv3 passes of this bench, procedural mesh, ARENAS_PER_GPU arenas).  Named explicitly and
# updated with every re-measurement -- never picked by file-name order.
ENV_PMC_FILE = "profiles/r06zy_env_pmc.json"


def pmc_traffic(kernel_ms, launch_arenas, mesh_name, pmc_file):
    """HBM traffic of the env kernel from the named PMC summary, as GB/s over the average launch
    duration measured here; None when the file is absent or was counted for launches of another arena count
    or another mesh."""
    path = os.path.join(ROOT, pmc_file)
    if not os.path.exists(path):
        return None, None
    d = json.load(open(path))
    if d.get("mesh", "synthetic") != mesh_name or d.get("arenas_per_launch", ARENAS_PER_GPU) != launch_arenas:
        return None, None
    b = d["hbm_bytes_per_launch"]
    src = {"bytes_per_launch": b, "source": pmc_file, "fetch_bytes_per_launch": 2 * d["fetch_size_kb_raw"] * 1024,
           "write_bytes_per_launch": d["write_size_kb"] * 1024}
    if d.get("kernel_us_rocprof"):  # the same profiling session's own kernel duration
        src["pmc_kernel_us"] = d["kernel_us_rocprof"]
        src["traffic_at_pmc_kernel_us"] = b / (d["kernel_us_rocprof"] * 1e-6) / 1e9
    return b / (kernel_ms * 1e-3) / 1e9, src


def cpu_cores():
    """The host cores this process may actually use: its affinity set, capped by the cgroup CPU quota
    (gpurun boxes show the whole machine in os.cpu_count() but grant a share)."""
    n = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    return n


class GpuClock:
    """Samples the GPU's shader clock (sysfs pp_dpm_sclk, the starred level) and board power (hwmon) every
    50 ms in a thread, so a bench line says at what clock its kernels ran: box-to-box spread in the env
    kernel's per-launch time (a latency-bound kernel scales with sclk) shows up here.  Read-only sysfs; on a
    host without it every field is None."""

    def __init__(self, dev):
        import glob
        import threading
        self.path, self.power, self.samples, self.watts = None, None, [], []
        bus = None
        try:
            import torch
            p = torch.cuda.get_device_properties(dev)
            bus = "%04x:%02x:%02x" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
        except Exception:
            pass
        cards = sorted(glob.glob("/sys/bus/pci/devices/*/pp_dpm_sclk"))
        mine = [c for c in cards if bus and os.path.basename(os.path.dirname(c)).startswith(bus)]
        pick = mine or (cards if len(cards) == 1 else [])
        if pick:
            self.path = pick[0]
            pw = sorted(glob.glob(os.path.join(os.path.dirname(self.path), "hwmon", "hwmon*", "power1_average")) +
                        glob.glob(os.path.join(os.path.dirname(self.path), "hwmon", "hwmon*", "power1_input")))
            self.power = pw[0] if pw else None
        self.pci = os.path.basename(os.path.dirname(self.path)) if self.path else bus
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def _read(self):
        try:
            for line in open(self.path):
                if line.rstrip().endswith("*"):
                    return float(line.split(":")[1].strip().rstrip("*").strip().lower().rstrip("mhz").strip())
        except (OSError, ValueError, IndexError):
            return None
        return None

    def _run(self):
        while not self._stop.wait(0.05):
            mhz = self._read()
            if mhz is not None:
                self.samples.append(mhz)
            if self.power:
                try:
                    self.watts.append(int(open(self.power).read()) / 1e6)
                except (OSError, ValueError):
                    pass

    def __enter__(self):
        if self.path:
            self._t.start()
        return self

    def __exit__(self, *a):
        self._stop.set()
        if self._t.is_alive():
            self._t.join()

    def summary(self):
        import statistics

        def mmm(v, unit):
            return None if not v else {"min": min(v), "median": statistics.median(v), "max": max(v), "unit": unit,
                                       "samples": len(v)}
        return {"source": self.path, "pci": self.pci, "sclk": mmm(self.samples, "MHz"),
                "power": mmm(self.watts, "W")}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(mesh=None, mesh_name="synthetic", seconds=12.0, arenas=1024):
    """The CPU restatement (oracle/, reference threading model: contiguous arena chunks over a
    pool) timed on this box's host cores on a bounded sample of the same env workload: the bench's
    own arena mesh, whose objects the oracle queries through their BVHs as Bullet does."""
    import numpy as np
    import oracle
    cores = cpu_cores()
    env = oracle.EnvSet(arenas, seed=1234, threads=cores, mesh=mesh)
    rng = np.random.default_rng(7)
    steps = 0
    t0 = time.perf_counter()
    while True:
        m = env.masks.astype(bool)
        a = np.argmax(rng.random(m.shape) * m, axis=1).astype(np.int32)
        env.step(a, True)
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    out = {"value": arenas * steps / el, "unit": "env-steps/s", "cores": cores, "kind": "port",
           "cpu_model": cpu_model(), "affinity_cpus": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count(),
           "sample": f"env only: {arenas} arenas x {steps} env steps of the oracle/ CPU restatement "
                     f"({cores} threads, uniform valid actions, the reference's x86 (MSVC x64) arithmetic, "
                     f"the bench's {mesh_name} mesh walked through each object's BVH)"}
    # one thread, one 2v2 arena: physics ticks/s beside RocketSim's published 114,481 ticks/s
    # (v2.1.0, i5-11400); the oracle runs tickSkip 8 ticks per env step plus the builders
    one = oracle.EnvSet(1, seed=99, threads=1, mesh=mesh)
    steps1 = 0
    t1 = time.perf_counter()
    while time.perf_counter() - t1 < 4.0:
        m1 = one.masks.astype(bool)
        one.step(np.argmax(rng.random(m1.shape) * m1, axis=1).astype(np.int32), True)
        steps1 += 1
    el1 = time.perf_counter() - t1
    out["one_thread"] = {"ticks_per_s": 8 * steps1 / el1, "env_steps_per_s": steps1 / el1,
                         "reference_published_ticks_per_s": 114481,
                         "sample": f"1 arena x {steps1} env steps (8 ticks + obs / reward builders each), 1 thread"}
    # BASELINE config C1 on CPU (PPO wall-clock per 1M agent-steps with the C1 model):
    # 64 arenas, actor / critic [256, 256], oracle env + torch CPU fp32 MLP / PPO, bounded sample
    from oracle.ppo_cpu import run_c1
    c1 = run_c1(seconds=10.0, threads=cores)
    out["c1_ppo"] = {"ppo_s_per_1M_agent_steps": c1["ppo_s_per_1M_agent_steps"],
                     "env_steps_per_s": c1["env_steps_per_s"], "cores": cores,
                     "sample": f"C1: 64 arenas, [256,256] actor/critic, T=64, {c1['iterations']} PPO iterations "
                               f"({c1['agent_steps']} agent-steps) of oracle env + torch CPU fp32 PPO"}
    # the GAE microbenchmark's inputs through the CPU restatement of GAE::Compute (oracle/gae_ref.c), 1 thread
    for lg in (21, 24):
        r, t, v, tv = gae_inputs(lg)
        t2 = time.perf_counter()
        oracle.gae_flat(r, t, v, tv, 0.99, 0.95, 1.7, 200.0)
        out.setdefault("gae_flat_ms", {})[f"M=2^{lg}"] = (time.perf_counter() - t2) * 1e3
    return out


def learn_roofline(L, train_gemm):
    """Per kernel class of the learn phase: achieved TF/s (fp32-equivalent flops 2*I*J*K of the GEMMs)
    against the H3 ceiling, or GB/s (algorithmic bytes of the LayerNorm kernels) against HBM, from
    one iteration timed per launch."""
    import torch
    from rlgpu.ppo import kernel_timing, kernel_timing_read
    kernel_timing(True)
    L.iterate()
    torch.cuda.synchronize()
    t = kernel_timing_read()
    kernel_timing(False)
    peak = H3_TFS if train_gemm == "h3" else (MFMA_F16_TFS / 6 if train_gemm == "x6" else MFMA_F16_TFS / 16)
    out = {"method": "HIP events around each launch on its own stream, one untimed PPO iteration after the timed ones",
           "gemm_peak_note": f"{train_gemm}: fp32-equivalent ceiling {peak:.0f} TF/s of the {MFMA_F16_TFS:.0f} TF/s dense 16-bit MFMA peak"}
    for name, (ms, work, n) in t.items():
        if n == 0:
            continue
        gemm = "GEMM" in name
        ach = work / (ms * 1e-3) / (1e12 if gemm else 1e9)
        p = peak if gemm else HBM_PEAK_GBS
        out[name] = {"bound": "mfma" if gemm else "hbm", "achieved": ach, "peak": p, "unit": "TF/s" if gemm else "GB/s",
                     "frac": ach / p, "launches": n, "ms_total": ms, "avg_us": ms * 1e3 / n,
                     ("flops_total" if gemm else "bytes_total"): work}
    return out


def gae_inputs(lg):
    """SURVEY.md 8d's GAE microbenchmark inputs: r ~ N(0,1), V ~ N(0,1), terminal NORMAL with p = 1/128 and
    TRUNCATED with p = 1/512, seed 7, M = 2^lg agent-steps, one truncation value per TRUNCATED step."""
    import numpy as np
    M = 1 << lg
    rng = np.random.default_rng(7)
    r = rng.standard_normal(M).astype(np.float32)
    v = rng.standard_normal(M).astype(np.float32)
    u = rng.random(M)
    t = np.where(u < 1 / 128, 1, np.where(u < 1 / 128 + 1 / 512, 2, 0)).astype(np.int8)
    tv = rng.standard_normal(int((t == 2).sum())).astype(np.float32)
    return r, t, v, tv


def gae_micro(dev, reps=20):
    """The GAE microbenchmark (gae_inputs) at M = 2^21 and 2^24: 21 algorithmic bytes per agent-step (r, V, A,
    target, R f32 + the terminal byte; the truncation values are ~M/512 more floats).  The flat
    episode-concatenated layout (GAE::Compute's own, rlgpu_gae_flat, which returns the clip portion to the
    host) and the engine's [T = 128, N] rollout layout (rlgpu_gae_rollout); HIP events around each call on the
    stream it runs on, inputs resident in HBM, median of `reps`."""
    import torch
    from rlgpu.gae import GAE
    out = {"bytes_per_agent_step": 21, "peak_GBps": HBM_PEAK_GBS}
    for lg in (21, 24):
        r, t, v, tv = gae_inputs(lg)
        M, ntr = r.size, tv.size
        dr, dv, dt = (torch.from_numpy(x).to(dev) for x in (r, v, t))
        dtv = torch.from_numpy(tv).to(dev) if ntr else None
        row = {"M": M, "truncations": ntr}
        T = 128
        N = M // T
        boot = torch.zeros(N, device=dev)
        trv = torch.zeros(M, device=dev)
        for name, call in (
                ("flat", lambda: GAE.compute(dr, dt, dv, dtv, 0.99, 0.95, 1.7, 200.0)),
                ("rollout", lambda: GAE.compute_rollout(dr.view(T, N), dt.view(T, N), dv.view(T, N), trv.view(T, N),
                                                        boot, 0.99, 0.95, 1.7, 200.0))):
            call()
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
            for i in range(reps):
                ev[2 * i].record()
                call()
                ev[2 * i + 1].record()
            torch.cuda.synchronize()
            ms = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(reps))[reps // 2]
            gbs = 21 * M / (ms * 1e-3) / 1e9
            row[name] = {"ms_median": ms, "agent_steps_per_s": M / (ms * 1e-3), "achieved_GBps": gbs,
                         "frac": gbs / HBM_PEAK_GBS}
        out[f"M=2^{lg}"] = row
    return out


def extra_leg(dev, name, mesh, iters=1, **kw):
    """One more workload on a fresh C++ Learner, beside the headline (rank 0, N = 1 only): one untimed and
    `iters` timed PPO iterations, their per-phase times and the learn-phase roofline of one more iteration.
    SURVEY.md 8d: C5 = 8,192 arenas, actor / critic [2048] x 4, fp16 inference (the MFMA-bound regime); x6 =
    the C2 workload with the exact fp32 GEMM split (rlgpu_ppo.h GEMM_F32X6) instead of H3."""
    import torch
    from rlgpu.learner import Learner, LearnerConfig
    cfg = LearnerConfig(train_against_old_versions=False, mesh=mesh, **kw)
    L = Learner(cfg, device=dev)
    L.iterate()
    torch.cuda.synchronize()
    ph = {"collect": 0.0, "consume": 0.0, "learn": 0.0}
    t0 = time.perf_counter()
    for _ in range(iters):
        rep = L.iterate()
        for k in ph:
            ph[k] += rep[k + "_s"]
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / iters
    env_steps = cfg.num_arenas * cfg.rollout_len
    gemm = {2: "h3", 0: "x6", 1: "f32"}[cfg.train_gemm]
    out = {"leg": name, "arenas": cfg.num_arenas, "policy_layers": list(cfg.policy_layers),
           "critic_layers": list(cfg.critic_layers), "train_gemm": gemm, "infer_fp16": bool(cfg.infer_fp16),
           "ms_per_iteration": el * 1e3, "env_steps_per_s": env_steps / el,
           "ppo_s_per_1M_agent_steps": el / (4 * env_steps) * 1e6, "iterations": iters,
           "phase_s_per_iteration": {k: v / iters for k, v in ph.items()},
           "learn_roofline": learn_roofline(L, gemm)}
    L.close()
    del L
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3, help="timed PPO iterations")
    ap.add_argument("--warmup", type=int, default=1, help="untimed PPO iterations")
    ap.add_argument("--arenas", type=int, default=ARENAS_PER_GPU)
    ap.add_argument("--rollout", type=int, default=128)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc-file", default=ENV_PMC_FILE,
                    help="the env kernel's PMC summary (tools/pmc_summary.py) that roofline.traffic comes from")
    ap.add_argument("--no-legs", action="store_true", help="skip the C5 and exact-GEMM (x6) legs")
    ap.add_argument("--mesh", choices=("procedural", "synthetic"), default="procedural",
                    help="arena collision mesh: the SOCCAR-sized procedural stand-in (16 objects, 8,800 triangles: "
                         "rlgpu.mesh.procedural_soccar) or the 36-triangle synthetic arena")
    ap.add_argument("--train-gemm", choices=("h3", "x6", "f32"), default="h3",
                    help="fp32 training GEMM arithmetic (include/rlgpu_ppo.h rlgpu_gemm modes)")
    ap.add_argument("--arith", choices=("msvc_x64", "gcc_x64", "scalar"), default="msvc_x64",
                    help="the reference build whose Bullet arithmetic the arenas follow (include/rlgpu_arith.h; "
                         "msvc_x64 = build.ps1's, the reference's own)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"bench.py --gpus {args.gpus} but WORLD_SIZE={world}: launch N > 1 as "
                         f"python -m torch.distributed.run --nproc-per-node {args.gpus} bench.py --gpus {args.gpus}")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; ranks beyond the visible GPUs (single-GPU rehearsals) share them round-robin
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    backend = None
    if world > 1:
        backend = os.environ.get("RLGPU_DIST_BACKEND", "nccl")  # nccl = RCCL over xGMI; gloo only for rehearsals
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)

    from rlgpu.env import arena_state_size
    from rlgpu.learner import Learner, LearnerConfig
    # self-play iterations (15 % chance, LearnerConfig.h:67-68) are off so every timed iteration has
    # the same work; the mixed-policy path is covered by tests/test_learner_gpu.py
    from rlgpu.ppo import GEMM_F16X3, GEMM_F32, GEMM_F32X6
    train_gemm = {"h3": GEMM_F16X3, "x6": GEMM_F32X6, "f32": GEMM_F32}[args.train_gemm]
    from rlgpu.mesh import procedural_soccar
    mesh = procedural_soccar() if args.mesh == "procedural" else None
    arith = {"msvc_x64": 0, "gcc_x64": 1, "scalar": 2}[args.arith]
    cfg = LearnerConfig(num_arenas=args.arenas, rollout_len=args.rollout, train_against_old_versions=False,
                        train_gemm=train_gemm, mesh=mesh, arith=arith,
                        collect_groups=int(os.environ.get("RLGPU_BENCH_COLLECT_GROUPS", "0")))  # 0: automatic
    # the C++ host Learner (host/learner.cpp); for N > 1 on RCCL its exchanges (gradient all-reduce, moments,
    # return samples) run on the native RCCL communicator in C++ (host/rccl_collective.cpp): torch.distributed
    # only broadcasts RCCL's unique id.  A gloo rehearsal (several ranks on one GPU) uses the torch.distributed
    # callbacks instead, since RCCL refuses two ranks on one device.
    native_rccl = world > 1 and backend == "nccl"
    L = None
    if native_rccl:
        # every rank must agree on the collective: a rank whose native communicator could not be created falls
        # back, with all the others, to the torch.distributed (RCCL) callbacks, and the line says so
        try:
            L = Learner(cfg, device=dev, rank=rank, world=world, native_rccl=True)
        except Exception as e:  # noqa: BLE001 - reported, then the consensus decides
            print(f"bench.py rank {rank}: native RCCL collective unavailable ({e}); voting for torch.distributed",
                  file=sys.stderr)
        ok = torch.tensor([1 if L is not None else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0:
            if L is not None:
                L.close()
                L = None
            native_rccl = False
    if L is None:
        L = Learner(cfg, device=dev, rank=rank, world=world, native_rccl=native_rccl)
    # HIP events around every fused env step, on the stream it runs on (RLGPU_BENCH_ENV_TIMING=0: none)
    L.set_env_timing(os.environ.get("RLGPU_BENCH_ENV_TIMING", "1") != "0")

    for _ in range(args.warmup):
        L.iterate()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    phase = {"collect": 0.0, "consume": 0.0, "learn": 0.0, "learn_issue": 0.0, "collect_issue": 0.0}
    kern, kern_min, kern_med, kern_max = [], [], [], []
    clock = GpuClock(dev).__enter__()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rep = L.iterate()
        phase["collect"] += rep["collect_s"]
        phase["consume"] += rep["consume_s"]
        phase["learn"] += rep["learn_s"]
        phase["learn_issue"] += rep["learn_issue_s"]
        phase["collect_issue"] += rep["collect_issue_s"]
        kern.append(rep["env_kernel_ms"])
        kern_min.append(rep["env_kernel_min_ms"])
        kern_med.append(rep["env_kernel_median_ms"])
        kern_max.append(rep["env_kernel_max_ms"])
        launch_arenas = rep["env_launch_arenas"]  # arenas per env launch (the collection's arena groups)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    clock.__exit__()
    from rlgpu.dist import max_over_ranks
    el = max_over_ranks(el, device=dev)
    env_steps = world * args.arenas * cfg.rollout_len * args.steps
    agent_steps = 4 * env_steps
    value = env_steps / el
    kern_ms = sum(kern) / len(kern) or float("nan")
    b_env = env_bytes_per_step(arena_state_size())
    achieved = b_env * launch_arenas / (kern_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(kern_ms, launch_arenas, args.mesh, args.pmc_file)
    out = {
        "metric": "env-steps/sec (whole node) at 32768 arenas; PPO wall-clock per 1M steps",
        "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": el * 1e3 / args.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"measured": f"{world} GPU(s) x {args.arenas} arenas = {world * args.arenas} arenas "
                               f"(the metric is quoted at 32768 arenas = 8 x 4096)",
                   "workload": f"C2: {args.arenas} arenas/GPU 2v2 RocketSim-equivalent physics, tickSkip 8 / actionDelay 7, "
                               "AdvancedObs + DefaultAction(90) + 13 ExampleMain rewards; PPO actor/critic [512,512] "
                               "LayerNorm+LeakyReLU, bf16 inference / fp32 training, T=128, 2 epochs, minibatch 50k",
                   "arenas_per_gpu": args.arenas, "agents_per_gpu": 4 * args.arenas, "rollout_len": cfg.rollout_len,
                   "parallelism": f"arena-sharded dp{world}", "inference_dtype": "bf16", "train_dtype": "f32",
                   "collective": ("native RCCL (host/rccl_collective.cpp)" if native_rccl else
                                  f"torch.distributed {backend} callbacks" if world > 1 else None),
                   "train_gemm": args.train_gemm, "arith": args.arith,
                   "self_play": "off (trainAgainstOldVersions = false: every timed iteration does the same work; "
                                "the old-version path is tested in tests/test_learner_gpu.py)",
                   "mesh": (f"procedural SOCCAR stand-in: {mesh.num_objects} objects, {mesh.num_tris} triangles "
                            "(quarter pipes, rounded corners, goal boxes; floor / walls / ceiling are static planes)"
                            if mesh is not None else "synthetic arena: 1 object, 36 triangles (include/rlgpu_arena_mesh.h)")},
        "agent_steps_per_s": agent_steps / el,
        "ppo_s_per_1M_agent_steps": el / agent_steps * 1e6,
        "phase_s_per_iteration": {k: v / args.steps for k, v in phase.items()},
        # the env kernel is latency-bound (serial per-arena phases, one wave per SIMD at 4096 arenas);
        # SURVEY 8d prescribes reporting it against HBM with algorithmic bytes, so frac is small by nature
        "roofline": {"bound": "hbm", "limiter": "latency (per-arena serial physics phases)", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_pmc": traffic_src,
                     "kernel": "rl::env_kernel", "kernel_ms": kern_ms, "bytes_per_env_step": b_env,
                     # per-launch spread over the timed iterations (min / median of the per-iteration medians /
                     # max) and the shader clock sampled over the timed region: what box-to-box spread is made of
                     "kernel_ms_min": min(kern_min), "kernel_ms_median": sorted(kern_med)[len(kern_med) // 2],
                     "kernel_ms_max": max(kern_max), "gpu_clock": clock.summary(),
                     "units_per_launch": launch_arenas, "collection_groups": args.arenas // launch_arenas,
                     "algorithmic_bytes_per_launch": b_env * launch_arenas},
    }
    # learn-phase roofline: one more (untimed) iteration with HIP events around every training GEMM
    # and LayerNorm launch, on the stream each runs on (rlgpu_kernel_timing)
    out["learn_roofline"] = learn_roofline(L, args.train_gemm)
    if rank == 0 and world == 1:
        out["gae_micro"] = gae_micro(dev)
    if rank == 0 and world == 1 and not args.no_legs:
        L.close()
        torch.cuda.empty_cache()
        from rlgpu.ppo import GEMM_F32X6 as _X6
        out["legs"] = [
            extra_leg(dev, "C5 per GPU", mesh, num_arenas=8192, policy_layers=(2048,) * 4, critic_layers=(2048,) * 4,
                      infer_fp16=True, arith=arith),
            extra_leg(dev, "C2 exact fp32 split (x6)", mesh, num_arenas=args.arenas, rollout_len=args.rollout,
                      train_gemm=_X6, arith=arith),
        ]
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(mesh, args.mesh)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
