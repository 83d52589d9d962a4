"""Collision-mesh ingestion (include/rlgpu_mesh.h, rlgpu/mesh.py) and the oracle's mesh path.
CPU only: the .cmf parser and hash are host code of librlgpu.so.

Parity anchors (the reference ships no .cmf files, so no golden meshes exist):
  * the hash is restated here independently in Python from CollisionMeshFile.cpp:70-95 and must
    equal the library's on meshes with positive and negative coordinates (parity unpinned beyond
    the formula: no reference hash of a mesh we hold is known);
  * the reference's error conditions (CollisionMeshFile.cpp:21-51) are reproduced;
  * the known-hash table equals RocketSim.cpp:20-35.
"""
import numpy as np
import pytest

import oracle
from rlgpu import _lib
from rlgpu.mesh import ArenaMesh, cmf_bytes, known_hash, parse_cmf
from rlgpu.state import ARENA, BT_TO_UU, UU_TO_BT
from tests_util import mesh_from_objects, procedural_arena_mesh


def py_cmf_hash(verts, tris):
    """CollisionMeshFile::UpdateHash restated (uint32 arithmetic; float -> uint32 as x86-64
    compilers do it: truncate to int64, keep the low 32 bits)."""
    M = 0xFFFFFFFF
    h = (len(verts) + len(tris) * len(verts)) & M
    for t in tris:
        for i in range(3):
            for j in range(3):
                v = int(np.float32(verts[t[i]][j])) & M  # int() truncates toward zero
                for _ in range(2):
                    v = (((v >> 16) ^ v) * 0x45D9F3B) & M
                v = ((v >> 16) ^ v) & M
                h ^= (v + 0x9E3779B9 + ((h << 6) & M) + (h >> 2)) & M
    return h


def test_parse_roundtrip_and_hash():
    rng = np.random.default_rng(0)
    verts = (rng.random((40, 3)) * 2000 - 1000).astype(np.float32)  # negative coordinates too
    tris = rng.integers(0, 40, (70, 3)).astype(np.int32)
    data = cmf_bytes(verts, tris)
    out, nv, h = parse_cmf(data)
    assert nv == 40 and out.shape == (70, 9)
    np.testing.assert_array_equal(out, verts[tris].reshape(-1, 9))
    assert h == py_cmf_hash(verts, tris)
    # trailing bytes are ignored (the reference only checks for overflow)
    out2, _, h2 = parse_cmf(data + b"\x00" * 7)
    assert h2 == h and (out2 == out).all()


def test_hash_is_order_sensitive():
    verts = np.array([[0, 0, 0], [100, 0, 0], [0, 100, 0], [0, 0, 100]], np.float32)
    a = np.array([[0, 1, 2], [0, 2, 3]], np.int32)
    assert parse_cmf(cmf_bytes(verts, a))[2] != parse_cmf(cmf_bytes(verts, a[::-1].copy()))[2]
    assert parse_cmf(cmf_bytes(verts, a))[2] == py_cmf_hash(verts, a)


@pytest.mark.parametrize("bad", ["count0", "count_big", "short", "index"])
def test_parse_errors_match_reference(bad):
    verts = np.zeros((3, 3), np.float32)
    tris = np.array([[0, 1, 2]], np.int32)
    data = cmf_bytes(verts, tris)
    if bad == "count0":
        data = np.array([0, 3], "<i4").tobytes() + data[8:]
        msg = "bad triangle/vertex count"
    elif bad == "count_big":
        data = np.array([1, 1000001], "<i4").tobytes() + data[8:]
        msg = "bad triangle/vertex count"
    elif bad == "short":
        data = data[:-1]
        msg = "overflown"
    else:
        data = cmf_bytes(verts, np.array([[0, 1, 3]], np.int32))
        msg = "bad triangle vertex index"
    with pytest.raises(_lib.RLGPUError, match=msg):
        parse_cmf(data)


def test_known_hashes():
    assert known_hash(0xA160BAF9) == 0 and known_hash(0xD84C7A68) == 15
    assert known_hash(0x16F3CC19, "hoops") == 11 and known_hash(0x16F3CC19) == -1
    assert known_hash(0x12345678) == -1


def test_arena_mesh_from_cmf_objects_and_warnings():
    objs = procedural_arena_mesh(nx=8, ny=8)
    with pytest.warns(UserWarning, match="does not match any known soccar"):
        m = ArenaMesh.from_cmf([cmf_bytes(v, t) for v, t in objs])
    tris, counts = mesh_from_objects(objs)
    np.testing.assert_array_equal(m.tris, tris)
    np.testing.assert_array_equal(m.object_ntris, counts)
    assert m.num_objects == len(objs) and len(m.hashes) == len(objs)
    with pytest.raises(_lib.RLGPUError):
        ArenaMesh([np.zeros((1, 9), np.float32)] * 33)


def _state(env):
    return np.frombuffer(env.get_arenas().tobytes(), ARENA).copy()


def test_oracle_ball_rolls_off_mesh_ramp():
    """A ball dropped onto the +x side-wall ramp (45 degrees, its own collision object) is pushed
    towards -x; with the built-in mesh (no ramp there) it falls straight onto the floor plane."""
    objs = procedural_arena_mesh(nx=8, ny=8)
    outs = []
    for mesh in (mesh_from_objects(objs), None):
        env = oracle.EnvSet(1, seed=2, mesh=mesh)
        st = _state(env)
        st["ball"][0]["pos"] = np.array([3950, 0, 400], np.float32) * UU_TO_BT
        st["ball"][0]["vel"] = np.array([0, 0, -1e-3], np.float32)
        env.set_arenas(np.frombuffer(st.tobytes(), np.uint8))
        for _ in range(15):
            env.step(np.full(4, 8, np.int32), False)
        outs.append(_state(env)["ball"][0]["vel"] * BT_TO_UU)
    assert outs[0][0] < -200, outs[0]
    assert abs(outs[1][0]) < 1.0, outs[1]


def test_oracle_car_ball_hit_registers():
    """Car driving into the ball at 1500 uu/s: the ball-car manifold is (A = ball, B = car), so the
    callback fires (ballHitInfo valid, Arena.cpp:283-333) and the ball leaves faster than the car."""
    env = oracle.EnvSet(1, seed=3)
    st = _state(env)
    st["ball"][0]["vel"] = np.array([0, 0, 1e-3], np.float32)
    c = st["cars"][0]
    c["body"]["pos"][0] = np.array([0, -250, 17], np.float32) * UU_TO_BT
    c["body"]["rot"][0] = np.array([[0, -1, 0], [1, 0, 0], [0, 0, 1]], np.float32).reshape(-1)
    c["body"]["vel"][0] = np.array([0, 1500, 0], np.float32) * UU_TO_BT
    env.set_arenas(np.frombuffer(st.tobytes(), np.uint8))
    for _ in range(2):
        env.step(np.full(4, 8, np.int32), False)
    s2 = _state(env)
    assert s2["cars"][0]["ball_hit_valid"][0] == 1
    rel = s2["cars"][0]["ball_hit_rel_pos"][0]  # on the ball: |rel| ~ ball radius (uu)
    assert 80 < np.linalg.norm(rel) < 100, rel
    vb = s2["ball"][0]["vel"] * BT_TO_UU
    vc = s2["cars"][0]["body"]["vel"][0] * BT_TO_UU
    assert vb[1] > vc[1] + 300, (vb, vc)


def _edge_flags(info):
    return info[:, 3].view(np.int32)


@pytest.mark.parametrize("which", ["procedural_soccar", "test_mesh"])
def test_internal_edge_info_matches_oracle(which):
    """btGenerateInternalEdgeInfo (RocketSim.cpp:166-170, btInternalEdgeUtility.cpp:50-358): the
    library's records (built at env-set create for the kernel) equal the oracle's independent
    restatement bit for bit, on the SOCCAR-sized procedural mesh and the test mesh."""
    from rlgpu.mesh import edge_info, procedural_soccar
    if which == "procedural_soccar":
        mesh = procedural_soccar()
    else:
        t, o = mesh_from_objects(procedural_arena_mesh())
        mesh = ArenaMesh([t[s:e] for s, e in zip(np.r_[0, np.cumsum(o)[:-1]], np.cumsum(o))])
    got = edge_info(mesh)
    want = oracle.mesh_edge_info(mesh.tris, mesh.object_ntris)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    flags = _edge_flags(got)
    assert (flags & (1 << 30)).mean() > 0.95  # tessellated surfaces: almost every triangle has a neighbour


def test_internal_edge_info_known_answers():
    """Two triangles of a flat quad: the shared diagonal has angle 0 (planar); a 90-degree fold: the
    angle is +-pi/2 with the convex flag when the fold is convex; edges without a neighbour keep 2 pi."""
    from rlgpu.mesh import edge_info
    two_pi = np.float32(2 * np.float32(np.pi))
    quad = np.float32([[0, 0, 0, 1, 0, 0, 1, 1, 0], [0, 0, 0, 1, 1, 0, 0, 1, 0]])
    info = edge_info(ArenaMesh([quad]))
    # triangle 0 shares V0 and V2 with triangle 1: its V2V0 edge; triangle 1 shares its V0V1 edge
    assert info[0, 2] == 0 and info[1, 0] == 0
    assert info[0, 0] == two_pi and info[0, 1] == two_pi
    # convex fold: floor triangle + wall triangle rising along the shared edge x = 1 (a box corner seen
    # from outside) vs concave fold (a wall rising from the floor's far edge, seen from inside)
    floor = [0, 0, 0, 1, 0, 0, 1, 1, 0]
    convex = np.float32([floor, [1, 0, 0, 1, 0, -1, 1, 1, 0]])
    concave = np.float32([floor, [1, 0, 0, 1, 1, 0, 1, 0, 1]])
    for tris, is_convex in ((convex, True), (concave, False)):
        info = edge_info(ArenaMesh([tris]))
        want = oracle.mesh_edge_info(tris)
        np.testing.assert_array_equal(info.view(np.uint32), want.view(np.uint32))
        a = info[0, 1]  # triangle 0's V1V2 edge is the fold
        assert abs(abs(a) - np.pi / 2) < 1e-5, a
        assert bool(_edge_flags(info)[0] & 2) == is_convex  # TRI_INFO_V1V2_CONVEX


@pytest.mark.parametrize("which", ["procedural_soccar", "test_mesh", "random"])
def test_bvh_visit_order_matches_oracle(which):
    """btOptimizedBvh::build / btQuantizedBvh::buildTree (btOptimizedBvh.cpp:28-160, btQuantizedBvh.cpp:
    116-305): the triangle order of each object's quantized BVH walk, which the env kernel commits mesh
    contacts in, equals the oracle's independent restatement (bvh_ref.hpp) exactly."""
    from rlgpu.mesh import bvh_order, procedural_soccar
    if which == "procedural_soccar":
        mesh = procedural_soccar()
    elif which == "test_mesh":
        t, o = mesh_from_objects(procedural_arena_mesh())
        mesh = ArenaMesh([t[s:e] for s, e in zip(np.r_[0, np.cumsum(o)[:-1]], np.cumsum(o))])
    else:  # ragged objects of scattered triangles, one flat in z (the 0.002 widening), one of a single triangle
        rng = np.random.default_rng(7)
        objs = [rng.uniform(-50, 50, (n, 9)).astype(np.float32) for n in (257, 1, 40)]
        objs[2][:, 2::3] = 3.0
        mesh = ArenaMesh(objs)
    got = bvh_order(mesh)
    want = oracle.bvh_order(mesh.tris, mesh.object_ntris)
    np.testing.assert_array_equal(got, want)
    t0 = 0
    for c in mesh.object_ntris:  # a permutation of each object's own range
        assert sorted(got[t0:t0 + c]) == list(range(t0, t0 + c))
        t0 += c
    if which != "random":
        assert (got != np.arange(mesh.num_tris)).any()


def test_bvh_visit_order_known_answers():
    """Hand-worked buildTree partitions: two triangles -> the one whose centre is above the mean first
    (the 1/3 balance fallback splits 1 + 1); five triangles in a row along x -> visited in descending x
    (mean split 2 + 3, then the fallbacks)."""
    from rlgpu.mesh import bvh_order
    tri = np.float32([0, 0, 0, 1, 0, 0, 0, 1, 0])
    row = lambda xs: np.stack([tri + np.float32([x, 0, 0] * 3) for x in xs])
    assert list(bvh_order(ArenaMesh([row([0, 10])]))) == [1, 0]
    assert list(bvh_order(ArenaMesh([row([0, 10, 20, 30, 40])]))) == [4, 3, 2, 1, 0]
    assert list(bvh_order(ArenaMesh([row([40, 0, 30, 10, 20])]))) == list(oracle.bvh_order(row([40, 0, 30, 10, 20])))
    assert list(bvh_order(ArenaMesh([tri[None]]))) == [0]


@pytest.mark.parametrize("perm", [(0, 1, 2), (0, 2, 1), (2, 1, 0)])
def test_internal_edge_info_bvh_neighbour_order(perm):
    """An edge shared by three triangles (floor A, its planar continuation B, a wall C): A's record is
    written by the neighbour the object's BVH query visits last (btInternalEdgeUtility.cpp:340-356),
    0 for B, +-pi/2 for C -- library and oracle agree for every listing order, and the BVH (built from the
    geometry) visits C after B in each of them, so the record does not depend on the listing (an index-
    order walk would give 0 for the (0, 2, 1) listing)."""
    from rlgpu.mesh import bvh_order, edge_info
    base = [np.float32([0, 0, 0, 1, 0, 0, 1, 1, 0]),        # A: the edge (1,0,0)-(1,1,0) is its V1V2
            np.float32([1, 0, 0, 2, 0.5, 0, 1, 1, 0]),      # B: coplanar across the edge
            np.float32([1, 0, 0, 1, 1, 0, 1, 0.5, 1])]     # C: wall rising from the edge
    tris = np.stack([base[i] for i in perm])
    got = edge_info(ArenaMesh([tris]))
    np.testing.assert_array_equal(got.view(np.uint32), oracle.mesh_edge_info(tris).view(np.uint32))
    order = list(bvh_order(ArenaMesh([tris])))
    a, b, c = (perm.index(i) for i in range(3))
    ang = got[a, 1]
    assert order.index(c) > order.index(b), order
    assert abs(abs(ang) - np.pi / 2) < 1e-5, ang
