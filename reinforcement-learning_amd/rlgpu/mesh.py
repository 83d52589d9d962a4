"""Arena collision meshes -- Python mirror of RocketSim's mesh loading over include/rlgpu_mesh.h.

Reference map:
    CollisionMeshFile::ReadFromStream + UpdateHash   RocketSim/src/CollisionMeshFile/CollisionMeshFile.cpp:11-95
                                                     -> parse_cmf(data)
    CollisionMeshFile::MakeBulletMesh                CollisionMeshFile.cpp:59-68 (vertices as stored,
                                                     bullet units) -> ArenaMesh.tris
    RocketSim::Init(folder) / InitFromMem            RocketSim.cpp:70-170 -> ArenaMesh.from_folder /
                                                     ArenaMesh.from_cmf
    MeshHashSet                                      RocketSim.cpp:12-44 -> known_hash(h, mode)

Each .cmf file becomes one collision object (the reference adds one static btBvhTriangleMeshShape
per file, Arena.cpp:1015-1058).  The reference iterates the folder in directory order, which the
standard leaves unspecified; here files are taken in sorted name order so a set is reproducible.
An ArenaMesh is passed to EnvSet(mesh=...); the library copies it into HBM and indexes it.
"""
import ctypes
import os
import warnings

import numpy as np

from . import _lib

GAMEMODES = {"soccar": 0, "hoops": 1}
MAX_OBJECTS = 32  # RLGPU_MAX_MESH_OBJECTS

_bound = False


def _bind():
    global _bound
    L = _lib.lib()
    if not _bound:
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
        L.rlgpu_cmf_parse.argtypes = [vp, i64, vp, i32, ctypes.POINTER(i32), ctypes.POINTER(i32),
                                      ctypes.POINTER(ctypes.c_uint32)]
        L.rlgpu_mesh_known_hash.argtypes = [i32, ctypes.c_uint32]
        _bound = True
    return L


def parse_cmf(data):
    """(tris [N, 9] float32 in bullet units, num_vertices, hash) of one .cmf image; raises
    RLGPUError on the reference's error conditions."""
    L = _bind()
    buf = bytes(data)
    nt, nv, h = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_uint32()
    _lib.check(L.rlgpu_cmf_parse(buf, len(buf), None, 0, ctypes.byref(nt), ctypes.byref(nv), ctypes.byref(h)),
               "rlgpu_cmf_parse")
    tris = np.empty((nt.value, 9), np.float32)
    _lib.check(L.rlgpu_cmf_parse(buf, len(buf), tris.ctypes.data, nt.value, None, None, None), "rlgpu_cmf_parse")
    return tris, nv.value, h.value


def known_hash(h, game_mode="soccar"):
    """Index of `h` in the reference's known-mesh list for the mode, or -1."""
    return _bind().rlgpu_mesh_known_hash(GAMEMODES[game_mode], h)


class ArenaMesh:
    """Triangles of all collision objects, object by object (bullet units)."""

    def __init__(self, objects, hashes=None):
        objs = [np.ascontiguousarray(o, np.float32).reshape(-1, 9) for o in objects]
        if not objs or len(objs) > MAX_OBJECTS:
            raise _lib.RLGPUError(f"an arena needs 1..{MAX_OBJECTS} collision objects, got {len(objs)}")
        self.tris = np.ascontiguousarray(np.concatenate(objs), np.float32)
        self.object_ntris = np.array([len(o) for o in objs], np.int32)
        self.hashes = list(hashes) if hashes is not None else []

    @property
    def num_tris(self):
        return len(self.tris)

    @property
    def num_objects(self):
        return len(self.object_ntris)

    @classmethod
    def from_cmf(cls, images, game_mode="soccar"):
        """RocketSim::InitFromMem: one object per image; unknown / duplicate hashes warn, as the
        reference does (RocketSim.cpp:140-155)."""
        objects, hashes, seen = [], [], set()
        for i, data in enumerate(images):
            tris, _, h = parse_cmf(data)
            if h in seen:
                warnings.warn(f"collision mesh [{i}] is a duplicate (0x{h:08x})")
            elif known_hash(h, game_mode) < 0:
                warnings.warn(f"collision mesh [{i}] does not match any known {game_mode} mesh (0x{h:08x})")
            seen.add(h)
            objects.append(tris)
            hashes.append(h)
        return cls(objects, hashes)

    @classmethod
    def from_folder(cls, folder, game_mode="soccar"):
        """RocketSim::Init(collisionMeshesFolder): <folder>/<mode>/*.cmf, sorted by name."""
        sub = os.path.join(folder, game_mode)
        names = sorted(n for n in os.listdir(sub) if n.endswith(".cmf"))
        if not names:
            raise _lib.RLGPUError(f"no .cmf meshes in {sub}")
        images = []
        for n in names:
            with open(os.path.join(sub, n), "rb") as f:
                images.append(f.read())
        return cls.from_cmf(images, game_mode)


def cmf_bytes(vertices, triangles):
    """Serialise a mesh in the .cmf layout (test fixtures, tools): int32 nTris, int32 nVerts,
    int32[3] per triangle, float32[3] per vertex, little endian."""
    v = np.ascontiguousarray(vertices, "<f4").reshape(-1, 3)
    t = np.ascontiguousarray(triangles, "<i4").reshape(-1, 3)
    return np.array([len(t), len(v)], "<i4").tobytes() + t.tobytes() + v.tobytes()


def procedural_soccar(arc_segments=10, length_segments=36, goal_segments=10):
    """A SOCCAR-sized stand-in for the absent game meshes (the reference loads 16 .cmf objects,
    ~9k triangles, RocketSim.cpp:100-170 / Arena.cpp:1015-1058; the .cmf files are not in the
    checkout).  It has their structure and density: the floor, ceiling and flat walls stay the
    reference's static planes (Arena.cpp:1052-1100), and the mesh covers what the planes do not --
    quarter-pipe transitions (radius 256 uu) from the floor and the ceiling into the side and back
    walls, rounded vertical corners, and the two goal boxes (back net, side nets, roof) -- split
    into 16 objects.  Vertices in bullet units (uu / 50).  ~9k triangles at the defaults."""
    s = 1.0 / 50.0
    X, Y, H, R, C = 4096.0, 5120.0, 2044.0, 256.0, 1152.0
    GW, GH, NET = 892.755, 642.775, 6000.0
    objs = []

    def grid(P):  # P [a, b, 3] vertex grid -> triangles [2 (a-1)(b-1), 9]
        a, b = P.shape[:2]
        t = []
        for i in range(a - 1):
            for j in range(b - 1):
                p00, p01, p10, p11 = P[i, j], P[i, j + 1], P[i + 1, j], P[i + 1, j + 1]
                t += [np.concatenate([p00, p10, p11]), np.concatenate([p00, p11, p01])]
        return np.array(t, np.float32)

    th = np.linspace(0.0, np.pi / 2, arc_segments + 1)
    # side-wall quarter pipes (floor and ceiling, both sides): along y, the arc in the x-z plane
    for side in (-1.0, 1.0):
        for top in (0, 1):
            ys = np.linspace(-(Y - C), Y - C, length_segments + 1)
            cx, cz = side * (X - R), (H - R) if top else R
            # floor: theta 0 at the floor (z = 0) -> pi/2 on the wall (z = R); ceiling: theta 0 at
            # the ceiling (z = H) -> pi/2 on the wall (z = H - R)
            px = cx + side * R * np.sin(th)
            pz = cz + (R * np.cos(th) if top else -R * np.cos(th))
            P = np.stack(np.broadcast_arrays(px[:, None], ys[None, :], pz[:, None]), -1)
            objs.append(grid(P * s))
    # back-wall quarter pipes (floor and ceiling, both ends), left and right of the goal mouth
    for end in (-1.0, 1.0):
        for top in (0, 1):
            parts = []
            for x0, x1 in ((-(X - C), -GW), (GW, X - C)):
                xs = np.linspace(x0, x1, length_segments // 2 + 1)
                cy, cz = end * (Y - R), (H - R) if top else R
                py = cy + end * R * np.sin(th)
                pz = cz + (R * np.cos(th) if top else -R * np.cos(th))
                P = np.stack(np.broadcast_arrays(xs[None, :], py[:, None], pz[:, None]), -1)
                parts.append(grid(P * s))
            objs.append(np.concatenate(parts))
    # rounded vertical corners (45-degree corner region as a quarter-round, radius C)
    for sx in (-1.0, 1.0):
        for sy in (-1.0, 1.0):
            zs = np.linspace(0.0, H, length_segments // 2 + 1)
            cx, cy = sx * (X - C), sy * (Y - C)
            px, py = cx + sx * C * np.cos(th), cy + sy * C * np.sin(th)
            P = np.stack(np.broadcast_arrays(px[:, None], py[:, None], zs[None, :]), -1)
            objs.append(grid(P * s))
    # goal boxes: back net + roof, and the two side nets (two objects per goal)
    for end in (-1.0, 1.0):
        xs, zs, ys = np.linspace(-GW, GW, goal_segments + 1), np.linspace(0.0, GH, goal_segments + 1), \
            np.linspace(end * Y, end * NET, goal_segments + 1)
        net = np.stack(np.broadcast_arrays(xs[:, None], end * NET, zs[None, :]), -1)
        roof = np.stack(np.broadcast_arrays(xs[:, None], ys[None, :], GH), -1)
        objs.append(np.concatenate([grid(net * s), grid(roof * s)]))
        sides = [np.stack(np.broadcast_arrays(gx, ys[:, None], zs[None, :]), -1) for gx in (-GW, GW)]
        objs.append(np.concatenate([grid(p * s) for p in sides]))
    return ArenaMesh(objs)


def edge_info(mesh, arith=0):
    """The internal-edge records the env set builds for `mesh` (rlgpu_mesh_edge_info): [ntris, 4]
    float32 -- the angle to the neighbour across edges V0V1, V1V2, V2V0 (2 pi: no neighbour) and the
    TRI_INFO_* flags as int32 bits (1 << 30: the triangle has a record).  arith: RLGPU_ARITH_* (the
    build whose arithmetic the records are made in; 0 = the reference's MSVC x64 build)."""
    L = _bind()
    L.rlgpu_mesh_edge_info.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_void_p]
    out = np.zeros((mesh.num_tris, 4), np.float32)
    _lib.check(L.rlgpu_mesh_edge_info(mesh.tris.ctypes.data, mesh.num_tris, mesh.object_ntris.ctypes.data,
                                      mesh.num_objects, int(arith), out.ctypes.data), "rlgpu_mesh_edge_info")
    return out


def bvh_order(mesh):
    """The order the reference's per-object quantized BVH visits the triangles of `mesh`
    (rlgpu_mesh_bvh_order): [ntris] int32, out[k] = the triangle visited k-th."""
    L = _bind()
    L.rlgpu_mesh_bvh_order.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
    out = np.zeros(mesh.num_tris, np.int32)
    _lib.check(L.rlgpu_mesh_bvh_order(mesh.tris.ctypes.data, mesh.num_tris, mesh.object_ntris.ctypes.data,
                                      mesh.num_objects, out.ctypes.data), "rlgpu_mesh_bvh_order")
    return out


def box_triangle_queries(rot, centre, tri, cbt, lds_first=True, arith=0):
    """The env kernel's car-hitbox vs triangle narrowphase (Bullet's GJK / EPA query, include/rlgpu_mesh.h
    rlgpu_box_triangle_queries) on the device, one query per lane.  CUDA tensors: rot [n,3,3] (basis rows),
    centre [n,3], tri [n,3,3], cbt [n] -> [n,8] float32 (hit, normal xyz, point xyz, depth).  lds_first: the
    penetration solver runs in a small LDS set first, else (False) in HBM only; "wave": the env kernel's
    policy (penetration queries deferred, then run by the whole wavefront); "wave-overflow": the same with a
    6-vertex wave set (every longer EPA reruns on the HBM set).  arith: RLGPU_ARITH_*
    (include/rlgpu_arith.h)."""
    import torch
    rot = rot.reshape(-1, 9).contiguous().float()
    n = rot.shape[0]
    centre = centre.reshape(n, 3).contiguous().float()
    tri = tri.reshape(n, 9).contiguous().float()
    cbt = cbt.reshape(n).contiguous().float()
    out = torch.zeros((n, 8), dtype=torch.float32, device=rot.device)
    L = _bind()
    L.rlgpu_box_triangle_queries.argtypes = [ctypes.c_int32] + [ctypes.c_void_p] * 5 + [ctypes.c_int32, ctypes.c_int32,
                                                                                     ctypes.c_void_p]
    _lib.check(L.rlgpu_box_triangle_queries(n, rot.data_ptr(), centre.data_ptr(), tri.data_ptr(), cbt.data_ptr(),
                                            out.data_ptr(), {"wave": 2, "wave-overflow": 3}.get(lds_first, None) if isinstance(lds_first, str)
                                            else int(bool(lds_first)), int(arith),
                                            ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
               "rlgpu_box_triangle_queries")
    return out


def box_box_queries(rot_a, centre_a, rot_b, centre_b):
    """The env kernel's car-vs-car hitbox narrowphase (btBoxBoxDetector / dBoxBox2, include/rlgpu_mesh.h
    rlgpu_box_box_queries) on the device.  CUDA tensors rot_* [n,3,3], centre_* [n,3] -> [n,29] float32
    (count, then up to 4 x normal on B, point, depth)."""
    import torch
    rot_a = rot_a.reshape(-1, 9).contiguous().float()
    n = rot_a.shape[0]
    args = [rot_a, centre_a.reshape(n, 3).contiguous().float(), rot_b.reshape(n, 9).contiguous().float(),
            centre_b.reshape(n, 3).contiguous().float()]
    out = torch.zeros((n, 29), dtype=torch.float32, device=rot_a.device)
    L = _bind()
    L.rlgpu_box_box_queries.argtypes = [ctypes.c_int32] + [ctypes.c_void_p] * 6
    _lib.check(L.rlgpu_box_box_queries(n, *[a.data_ptr() for a in args], out.data_ptr(),
                                       ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "rlgpu_box_box_queries")
    return out
