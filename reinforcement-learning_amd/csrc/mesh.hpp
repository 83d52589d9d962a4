// mesh.hpp -- host-side construction of the env kernel's MeshView (env_kernel.hpp): the triangle
// table in Bullet's BVH visit order and its uniform-grid index.  Implemented in mesh.hip.
#pragma once
#include <cstdint>
#include <vector>

#define RLGPU_PADS_FOR_MAP 34

namespace rlgpu {

struct MeshGrid {
    // one entry per (cell, triangle) listing, ascending triangle index within a cell, the triangle
    // inline: 12 floats = v0.xyz | object id bits, v1.xyz | triangle index bits, v2.xyz | cell x bits
    std::vector<float> cell_tri;
    std::vector<int> cell_start;
    // per triangle in BVH visit order: 12 floats = v0.xyz | object id bits, v1.xyz | 0, v2.xyz | 0, and its
    // internal-edge record (edge_info.hpp EdgeInfo: 3 angles | flags bits)
    std::vector<float> tri, edge;
    // Bullet's BVH visit order (bvh_visit_order): visit position of each triangle (object start + rank
    // within its object) and the triangle at each position
    std::vector<int> visit_pos, visit_tri;
    float ox = 0, oy = 0, oz = 0, inv_cell = 1;
    int nx = 1, ny = 1, nz = 1, ntris = 0;
    // a box of cells that lists no triangle, grown from the grid's centre (x0, x1, y0, y1, z0, z1; x0 > x1: none):
    // a query whose cells all lie in it has nothing to walk
    int empty[6] = {1, 0, 1, 0, 1, 0};
};

// tris_bt: ntris x 9 floats (bullet units); object k owns the next object_ntris[k] triangles
// (object_ntris == nullptr: one object).  Throws rlgpu::Error on invalid input.
MeshGrid build_mesh_grid(const float* tris_bt, int ntris, const int32_t* object_ntris, int nobjects, int arith);

// btGenerateInternalEdgeInfo over every object of a mesh (edge_info.hpp): ntris x 4 floats
// (m_edgeV0V1Angle, m_edgeV1V2Angle, m_edgeV2V0Angle, flags bits; flags 0 = no record)
std::vector<float> mesh_edge_info(const float* tris_bt, int ntris, const int32_t* object_ntris, int nobjects, int arith);

// The order in which Bullet's quantized BVH of one mesh visits its triangles (btBvhTriangleMeshShape with
// quantized AABB compression, RocketSim.cpp:167; btOptimizedBvh::build, btQuantizedBvh::buildTree and the
// stackless walk, btQuantizedBvh.cpp:76-305,676-740): out[k] = the triangle visited k-th.
std::vector<int> bvh_visit_order(const float* tris_bt, int ntris);

// The built-in synthetic arena mesh (include/rlgpu_arena_mesh.h) in bullet units (uu / 50).
std::vector<float> builtin_mesh_bt();

// This host's rsqrtss table for the x86 arithmetic modes (host/x86_arith.cpp, rlgpu_arith.h): 2 << *bits
// entries; throws rlgpu::Error(RLGPU_ERR_UNSUPPORTED) when the host has none usable.
const std::vector<uint32_t>& x86_rsqrt_table_or_throw(int* bits);

// GameState::UpdateFromArena on arena records (host/gamestate.cpp, include/rlgpu_gamestate.h), and the
// pad index map it reads (GameState.cpp:11-51: CommonValues::BOOST_LOCATIONS[i] -> arena pad, env.hip)
void boost_pad_index_map(int out[RLGPU_PADS_FOR_MAP]);
}  // namespace rlgpu
#include "../../include/rlgpu_gamestate.h"
namespace rlgpu {
void gamestates_from_arenas(const rlgpu_arena_state* rec, int count, int tick_skip, rlgpu_gamestate* out);

// Axis cell of a coordinate, the same IEEE operations as the device's grid_cell.
inline int grid_cell_host(float x, float o, float inv, int n) {
    float f = __builtin_floorf((x - o) * inv);
    f = __builtin_fminf(__builtin_fmaxf(f, 0.f), (float)(n - 1));
    return (int)f;
}

}  // namespace rlgpu
