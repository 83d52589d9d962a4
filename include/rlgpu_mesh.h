/*
 * rlgpu_mesh.h -- arena collision-mesh ingestion (host side, no GPU needed).
 *
 * Replaces:
 *   RocketSim::CollisionMeshFile::ReadFromStream   RocketSim/src/CollisionMeshFile/CollisionMeshFile.cpp:11-57
 *   RocketSim::CollisionMeshFile::UpdateHash       CollisionMeshFile.cpp:70-95
 *   CollisionMeshFile::MakeBulletMesh              CollisionMeshFile.cpp:59-68 (vertices as stored,
 *                                                  no de-duplication, no scaling: bullet units)
 *   MeshHashSet (known SOCCAR / HOOPS hashes)      RocketSim/src/RocketSim.cpp:12-44
 *
 * The parsed triangles go to rlgpu_envset_config.mesh_tris (rlgpu_env.h), one collision object per
 * file, where the env builds its device-side triangle table and uniform-grid index.
 */
#ifndef RLGPU_MESH_H
#define RLGPU_MESH_H

#include <stdint.h>
#include "rlgpu_arith.h"
#include "rlgpu_core.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RLGPU_GAMEMODE_SOCCAR 0   /* GameMode::SOCCAR (Sim/GameMode.h:6-16) */
#define RLGPU_GAMEMODE_HOOPS 1    /* GameMode::HOOPS */
#define RLGPU_CMF_MAX_COUNT 1000000 /* MAX_VERT_OR_TRI_COUNT (CollisionMeshFile.cpp:15) */

/* Parse one .cmf image: int32 numTris, int32 numVertices, numTris x int32[3] vertex indices,
 * numVertices x float[3] (little endian).  Errors as the reference: a count <= 0 or > 1e6, data
 * shorter than the counts need ("input data overflown"), a vertex index out of range.  Trailing
 * bytes are ignored.  Outputs (each may be NULL): *out_ntris, *out_nverts, *out_hash (UpdateHash)
 * and, when out_tris != NULL, the triangles expanded to 9 floats each (v0, v1, v2) -- at most
 * max_tris of them are written, call first with out_tris == NULL to size the buffer. */
int rlgpu_cmf_parse(const void* data, int64_t size, float* out_tris, int32_t max_tris, int32_t* out_ntris,
                    int32_t* out_nverts, uint32_t* out_hash);

/* Position of `hash` in the reference's list of known meshes for the game mode, or -1 (the
 * reference only warns about unknown or duplicate meshes, RocketSim.cpp:140-155). */
int rlgpu_mesh_known_hash(int32_t game_mode, uint32_t hash);

/* The internal-edge records the env set builds for its mesh at create (RocketSim.cpp:166-170:
 * btGenerateInternalEdgeInfo per collision object; used by btAdjustInternalEdgeContacts in the contact
 * callback, Arena.cpp:275-279).  tris / object_ntris as rlgpu_envset_config.mesh_* (object_ntris NULL:
 * one object).  out: ntris x 4 floats = m_edgeV0V1Angle, m_edgeV1V2Angle, m_edgeV2V0Angle (2 pi = no
 * neighbour) and the flags as int32 bits (TRI_INFO_* convex 1/2/4, swap 8/16/32; bit 30 = the triangle
 * has a record, 0 = none).  arith: the RLGPU_ARITH_* mode the records are built in (the connectivity
 * processor normalises with btVector3::normalize and rotates with quatRotate, btInternalEdgeUtility.cpp:
 * 159-271, whose arithmetic is the build's, include/rlgpu_arith.h).  Host only. */
int rlgpu_mesh_edge_info(const float* tris, int32_t ntris, const int32_t* object_ntris, int32_t nobjects, int32_t arith,
                         float* out);

/* The order in which the reference's per-object quantized BVH (btBvhTriangleMeshShape with quantized
 * AABB compression, RocketSim.cpp:167; btOptimizedBvh::build, btOptimizedBvh.cpp:28-160, and
 * btQuantizedBvh::buildTree, btQuantizedBvh.cpp:116-305) hands overlapping triangles to the narrowphase:
 * out[k] = the mesh triangle visited k-th (objects in order, each object's triangles permuted within its
 * own range).  The env kernel commits mesh contacts in this order.  tris / object_ntris as
 * rlgpu_mesh_edge_info.  Host only. */
int rlgpu_mesh_bvh_order(const float* tris, int32_t ntris, const int32_t* object_ntris, int32_t nobjects,
                         int32_t* out);

/* The car-hitbox vs mesh-triangle narrowphase of the env kernel on its own (the GJK / EPA query of
 * btConvexTriangleCallback::processTriangle -> btConvexConvexAlgorithm -> btGjkPairDetector with
 * btGjkEpaPenetrationDepthSolver, btConvexConcaveCollisionAlgorithm.cpp:71-138 and
 * btGjkPairDetector.cpp:686-959), on the device, one query per lane: n queries of device arrays rot
 * [n][9] (box basis rows), centre [n][3] (hitbox child origin), tri [n][9] (three vertices), cbt [n]
 * (contact breaking threshold); the box is the Octane hitbox.  d_out [n][8] = {hit, normal xyz,
 * point xyz, depth} (the arguments of btManifoldResult::addContactPoint; zeros when no point).
 * lds_first != 0: the penetration solver first runs in a small LDS work set per lane (24 support
 * vertices, 28 live faces), rerun in the lane's HBM set when it overflows; 0: HBM only; 2: the env
 * kernel's policy -- 64 lanes each stop at the penetration solver, then the whole wavefront runs those
 * queries one at a time with the polytope in its registers (gjk.hpp epa_wave), HBM rerun on overflow;
 * 3: as 2 with a 6-vertex wave set, so that the EPA overflows and reruns (tests of that path).  arith: RLGPU_ARITH_* (the normalisations follow that build, include/rlgpu_arith.h).
 * Asynchronous on `stream`; the HBM sets are allocated per call. */
int rlgpu_box_triangle_queries(int32_t n, const float* d_rot, const float* d_centre, const float* d_tri,
                               const float* d_cbt, float* d_out, int32_t lds_first, int32_t arith, void* stream);

/* The car-vs-car hitbox narrowphase of the env kernel on its own (btBoxBoxDetector::getClosestPoints ->
 * dBoxBox2, btBoxBoxDetector.cpp:267-767), on the device, one query per lane: n queries of device arrays
 * rot_a / rot_b [n][9] (basis rows), centre_a / centre_b [n][3] (hitbox child origins), both boxes the
 * Octane hitbox.  d_out [n][29] = {count, then up to 4 x (normal on B xyz, point xyz, depth)} (the
 * btManifoldResult::addContactPoint calls in order).  Asynchronous on `stream`. */
int rlgpu_box_box_queries(int32_t n, const float* d_rot_a, const float* d_centre_a, const float* d_rot_b,
                          const float* d_centre_b, float* d_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif
