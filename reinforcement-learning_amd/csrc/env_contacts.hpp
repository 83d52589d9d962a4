// env_contacts.hpp -- persistent manifolds, narrowphase, contact callbacks and the
// sequential-impulse solver of the env kernel.  Reference map in env_kernel.hpp; each
// function cites the Bullet / RocketSim code it restates.
#pragma once
#include "boxbox.hpp"
#include "edge_info.hpp"
#include "env_device.hpp"

namespace rl {

// Work items ("ranks") of the narrowphase, in Bullet's pair order: rank body*5 + 0 = the body vs
// every mesh object, body*5 + 1..4 = the body vs plane 0..3; ranks 25..34 = dynamic pairs
// (a, b), a < b: (0,1..4) (1,2..4) (2,3..4) (3,4).
DEV void dyn_pair(int rank, int& a, int& b) {
    int r = rank - 25;
    a = r < 4 ? 0 : (r < 7 ? 1 : (r < 9 ? 2 : 3));
    int first = a == 0 ? 0 : (a == 1 ? 4 : (a == 2 ? 7 : 9));
    b = a + 1 + (r - first);
}
DEV int mesh_key(int body, int obj) { return body * kStat + obj; }
DEV int plane_key(int body, int plane) { return body * kStat + kMaxObj + plane; }
DEV int dyn_key(int a, int b) { return kDynKey + a * 8 + b; }
// manifold body A / B of a key: a body (0 ball, 1..4 cars) or 10 + static slot.  Dynamic pairs:
// A = the lower body, so A = ball for ball-car pairs (Bullet creates that manifold as
// (sphere, box), btSphereBoxCollisionAlgorithm.cpp:30-37).
DEV void key_bodies(int key, int& a, int& b) {
    if (key >= kDynKey) {
        a = (key - kDynKey) / 8;
        b = (key - kDynKey) % 8;
    } else {
        a = key / kStat;
        b = 10 + key % kStat;
    }
}
DEV void side_transform(ArenaLDS* A, int id, v3& p, m3& r) {
    if (id >= 10) {
        p = zero3();
        r = ident3();
    } else {
        p = bpos(A, id);
        r = brot(A, id);
    }
}
DEV float pair_cbt(int a, int b) {
    float ta = a == 0 ? C.ball_cbt : C.car_cbt;
    if (b >= 10) return ta;
    float tb = b == 0 ? C.ball_cbt : C.car_cbt;
    return stdmin(ta, tb);
}

// Manifolds live for one tick (rlgpu_env.h): the commit processes keys in ascending order and
// creates each pair's manifold on its first point, so the current key's manifold, if any, is the
// last one created.
DEV rlgpu_manifold* find_manifold(ArenaLDS* A, int key) {
    const int n = A->a.nmf;
    return (n > 0 && A->mf[n - 1].key == key) ? &A->mf[n - 1] : nullptr;
}
DEV rlgpu_manifold* get_or_new_manifold(ArenaLDS* A, int key) {
    rlgpu_manifold* m = find_manifold(A, key);
    if (m) return m;
    const int n = A->a.nmf;
    if (n >= RLGPU_MANIFOLDS) return nullptr;
    A->a.nmf = n + 1;
    A->mf[n].key = key;
    A->mf[n].count = 0;
    return &A->mf[n];
}

// btPersistentManifold::sortCachedPoints (btPersistentManifold.cpp:110-198)
DEV int sort_cached(const rlgpu_manifold& m, const rlgpu_contact& pt) {
    int max_idx = -1;
    float max_pen = pt.dist;
    for (int i = 0; i < 4; i++)
        if (m.pts[i].dist < max_pen) {
            max_idx = i;
            max_pen = m.pts[i].dist;
        }
    v3 p = ld3(pt.localA);
    v3 l0 = ld3(m.pts[0].localA), l1 = ld3(m.pts[1].localA), l2 = ld3(m.pts[2].localA), l3 = ld3(m.pts[3].localA);
    // four named values, not an array: a lane-indexed private array lives in scratch memory
    const float r0 = max_idx != 0 ? len2(cross(p - l1, l3 - l2)) : 0.f;
    const float r1 = max_idx != 1 ? len2(cross(p - l0, l3 - l2)) : 0.f;
    const float r2 = max_idx != 2 ? len2(cross(p - l0, l3 - l1)) : 0.f;
    const float r3 = max_idx != 3 ? len2(cross(p - l0, l2 - l1)) : 0.f;
    int best = -1;
    float mx = -1e30f;
    if (fabsf(r0) > mx) best = 0, mx = fabsf(r0);
    if (fabsf(r1) > mx) best = 1, mx = fabsf(r1);
    if (fabsf(r2) > mx) best = 2, mx = fabsf(r2);
    if (fabsf(r3) > mx) best = 3, mx = fabsf(r3);
    return best;
}

// Arena::_BtCallback_OnCarBallCollision (Arena.cpp:283-333)
DEV void car_ball_hit(ArenaLDS* A, int ci, rlgpu_contact& cp) {
    rlgpu_car& cs = A->s.cars[ci];
    int bi = ci + 1;
    cp.friction = 2.0f;
    cp.restitution = 0.0f;
    v3 ball_pos = bpos(A, 0) * kBT2UU, car_pos = bpos(A, bi) * kBT2UU;
    v3 ball_vel = bvel(A, 0) * kBT2UU, car_vel = bvel(A, bi) * kBT2UU;
    cs.ball_hit_valid = 1;
    st3(cs.ball_hit_rel_pos, ld3(cp.localA) * kBT2UU);  // ballIsBodyA (Arena.cpp:297)
    cs.ball_hit_tick = A->s.env.tick_count;
    st3(cs.ball_hit_ball_pos, ball_pos);
    st3(cs.ball_hit_extra_vel, zero3());
    int64_t tick = A->s.env.tick_count;
    uint64_t uex = (uint64_t)cs.ball_hit_extra_tick, ut = (uint64_t)tick;
    if ((ut > uex + 1) || (uex > ut)) {
        cs.ball_hit_extra_tick = tick;
    } else {
        return;
    }
    v3 fwd = col(brot(A, bi), 0);
    v3 rel_pos = ball_pos - car_pos;
    v3 rel_vel = ball_vel - car_vel;
    float rel_speed = stdmin(len(rel_vel), 4600.f);
    if (rel_speed > 0) {
        v3 hit_dir = safe_normalized(rel_pos * v3{1, 1, 0.35f});
        v3 adj = fwd * dot(hit_dir, fwd) * (1 - 0.65f);
        hit_dir = safe_normalized(hit_dir - adj);
        v3 added = (hit_dir * rel_speed) * curve_out<kBallCarExtra>(rel_speed) * 1.f;
        st3(cs.ball_hit_extra_vel, added);
        st3(A->s.ball_vel_impulse_cache, ld3(A->s.ball_vel_impulse_cache) + added * kUU2BT);
    }
}

// Arena::_BtCallback_OnCarCarCollision (Arena.cpp:335-415) + EnvSet _BumpCallback (EnvSet.cpp:31-42)
DEV void car_car_hit(ArenaLDS* A, int c1, int c2, rlgpu_contact& cp) {
    cp.friction = 0.09f;
    cp.restitution = 0.1f;
    for (int i = 0; i < 2; i++) {
        bool swapped = i == 1;
        int a = swapped ? c2 : c1, o = swapped ? c1 : c2;
        rlgpu_car& sa = A->s.cars[a];
        rlgpu_car& so = A->s.cars[o];
        if (sa.is_demoed || so.is_demoed) return;
        if (sa.car_contact_other_id == (uint32_t)(o + 1) && sa.car_contact_cooldown > 0) continue;
        v3 pa = bpos(A, a + 1) * kBT2UU, po = bpos(A, o + 1) * kBT2UU;
        v3 va = bvel(A, a + 1) * kBT2UU, vo = bvel(A, o + 1) * kBT2UU;
        v3 delta = po - pa;
        if (dot(va, delta) > 0) {
            v3 vel_dir = rs_norm(va);
            v3 dir_to = rs_norm(delta);
            float speed_towards = dot(va, dir_to);
            float other_away = dot(vo, vel_dir);
            if (speed_towards > other_away) {
                v3 lp = swapped ? ld3(cp.localB) : ld3(cp.localA);
                bool bumper = (lp.x * kBT2UU) > 64.5f;
                if (bumper) {
                    bool demo = sa.is_supersonic;
                    if (demo) demo = (a & 1) != (o & 1);
                    if (demo) {
                        so.is_demoed = 1;
                        so.demo_respawn_timer = 3.f;
                    } else {
                        bool ground = so.is_on_ground;
                        float base = ground ? curve_out<kBumpGround>(speed_towards) : curve_out<kBumpAir>(speed_towards);
                        v3 up = so.is_on_ground ? col(brot(A, o + 1), 2) : v3{0, 0, 1};
                        v3 imp = vel_dir * base + up * curve_out<kBumpUp>(speed_towards) * 1.f;
                        st3(so.vel_impulse_cache, ld3(so.vel_impulse_cache) + imp * kUU2BT);
                    }
                    sa.car_contact_other_id = (uint32_t)(o + 1);
                    sa.car_contact_cooldown = 0.25f;
                    if ((a & 1) != (o & 1)) {
                        A->s.env.ev_bump[a] = 1;
                        A->s.env.ev_bumped[o] = 1;
                        if (demo) {
                            A->s.env.ev_demo[a] = 1;
                            A->s.env.ev_demoed[o] = 1;
                        }
                    }
                }
            }
        }
    }
}

// Arena::_BulletContactAddedCallback (Arena.cpp:218-281): bodies ordered car < ball < world
DEV void contact_callback(ArenaLDS* A, int a, int b, rlgpu_contact& cp) {
    if (a >= 1 && a <= 4) {
        int ci = a - 1;
        if (b >= 1 && b <= 4) {
            car_car_hit(A, ci, b - 1, cp);
        } else if (b >= 10) {  // car-world (Arena.cpp:417-427)
            rlgpu_car& cs = A->s.cars[ci];
            cs.world_contact = 1;
            cs.world_contact_normal[0] = cp.normalB[0];
            cs.world_contact_normal[1] = cp.normalB[1];
            cs.world_contact_normal[2] = cp.normalB[2];
            cp.friction = 0.3f;
            cp.restitution = 0.3f;
        }
    } else if (a == 0) {
        if (b >= 1 && b <= 4) {
            car_ball_hit(A, b - 1, cp);  // manifold A = ball: swapped into (car, ball)
        } else if (b >= 10) {
            cp.special = 1;  // Arena.cpp:265-273
        }
    }
}

// btManifoldResult::addContactPoint (btManifoldResult.cpp:110-200); tri >= 0: the mesh triangle the
// point lies on (its internal-edge adjustment ends the contact callback, Arena.cpp:275-279)
DEV void add_contact(ArenaLDS* A, const MeshView& M, int key, v3 normal_b, v3 point_b, float depth, int tri) {
    int a, b;
    key_bodies(key, a, b);
    float cbt = pair_cbt(a, b);
    if (depth > cbt) return;
    rlgpu_manifold* m = get_or_new_manifold(A, key);
    if (!m) {
        A->s.env.manifold_overflow++;
        return;
    }
    v3 pa = point_b + normal_b * depth;
    v3 ta_p, tb_p;
    m3 ta_r, tb_r;
    side_transform(A, a, ta_p, ta_r);
    side_transform(A, b, tb_p, tb_r);
    rlgpu_contact c;
    st3(c.localA, vmul(pa - ta_p, ta_r));
    st3(c.localB, vmul(point_b - tb_p, tb_r));
    st3(c.normalB, normal_b);
    c.dist = depth;
    c.applied = 0.f;
    bool stat = b >= 10;
    float fa = a == 0 ? 0.35f : 0.3f, ra = a == 0 ? 0.6f : 0.1f;
    float fb = stat ? 0.6f : (b == 0 ? 0.35f : 0.3f), rb = stat ? 0.3f : (b == 0 ? 0.6f : 0.1f);
    c.friction = stat ? stdmin(fa, fb) : fa * fb;
    c.restitution = stat ? stdmax(ra, rb) : ra * rb;
    c.special = 0;
    int idx;
    if (m->count == 4) {
        idx = sort_cached(*m, c);
    } else {
        idx = m->count;
        m->count++;
    }
    if (idx < 0) idx = 0;
    m->pts[idx] = c;
    contact_callback(A, a, b, m->pts[idx]);
    if (tri >= 0) {  // btAdjustInternalEdgeContacts on the stored point (mesh at the identity transform)
        rlgpu_contact& cp = m->pts[idx];
        const float4 t0 = M.tri[3 * tri], t1 = M.tri[3 * tri + 1], t2 = M.tri[3 * tri + 2], ei = M.edge[tri];
        const EdgeInfo info{ei.x, ei.y, ei.z, __float_as_int(ei.w)};
        v3 n = ld3(cp.normalB), pb = ld3(cp.localB);
        adjust_edge_contact(v3{t0.x, t0.y, t0.z}, v3{t1.x, t1.y, t1.z}, v3{t2.x, t2.y, t2.z}, info, n, pb, pa, cp.dist,
                            arith(A));
        st3(cp.normalB, n);
        st3(cp.localB, pb);
    }
}

// btPersistentManifold::refreshContactPoints (btPersistentManifold.cpp:265-330)
DEV bool refresh(ArenaLDS* A, int key) {
    rlgpu_manifold* m = find_manifold(A, key);
    if (!m) return false;
    int a, b;
    key_bodies(key, a, b);
    float cbt = pair_cbt(a, b);
    v3 pa_, pb_;
    m3 ra, rb;
    side_transform(A, a, pa_, ra);
    side_transform(A, b, pb_, rb);
    for (int i = m->count - 1; i >= 0; i--) {
        rlgpu_contact& p = m->pts[i];
        v3 wa = ra * ld3(p.localA) + pa_;
        v3 wb = rb * ld3(p.localB) + pb_;
        p.dist = dot(wa - wb, ld3(p.normalB));
    }
    // (world points recomputed from the local ones: same operations, so the same values as
    // the cached world positions of the reference)
    for (int i = m->count - 1; i >= 0; i--) {
        rlgpu_contact& p = m->pts[i];
        bool remove;
        if (!(p.dist <= cbt)) {
            remove = true;
        } else {
            v3 wa = ra * ld3(p.localA) + pa_;
            v3 wb = rb * ld3(p.localB) + pb_;
            v3 proj = wa - ld3(p.normalB) * p.dist;
            v3 diff = wb - proj;
            remove = dot(diff, diff) > cbt * cbt;
        }
        if (remove) {
            int last = m->count - 1;
            if (i != last) m->pts[i] = m->pts[last];
            m->count--;
        }
    }
    return m->count > 0;
}

// ------------------------------------------------------------------ narrowphase (candidates)
// Commit (= manifold = solver) order of a work item: btRSBroadphase::calculateOverlappingPairs
// (btRSBroadphase.cpp:392-465) walks the dynamic proxies in creation order (ball, then cars 1-4) and adds,
// for each, its pairs with the cell's static proxies (meshes, then planes: creation order), then its
// pairs with the cell's other dynamic proxies not paired yet; the pair cache dispatches in that order.
// Within one proxy's dynamic pairs, the order of its home cell's dynamic list (bp_update).
// btRSBroadphase's cell lists (btRSBroadphase.cpp:90-110,160-176,284-320): a dynamic proxy's home cell is the
// grid cell of its AABB min and the proxy sits in the 27 cells around it, appended when created and re-appended
// whenever its home cell changes (setAabb, called by updateAabbs for the bodies in creation order); so every
// cell lists its dynamic proxies in the order of their last home change.  bp_rank keeps that order per arena.
DEV int bp_home(v3 mn) {
    const v3 f = (mn - C.bp_min) * C.bp_inv_cell;  // (pos - minPos) / cellSize = * (1 / cellSize)
    const int i = min(max((int)f.x, 0), C.bp_cells[0] - 1);
    const int j = min(max((int)f.y, 0), C.bp_cells[1] - 1);
    const int k = min(max((int)f.z, 0), C.bp_cells[2] - 1);
    return (i * C.bp_cells[1] + j) * C.bp_cells[2] + k;
}
// bp_key (env_device.hpp): a body's position in every cell's dynamic list
// one lane per arena, on this tick's broadphase AABBs (after predictUnconstraintMotion) and the home cells the
// body lanes computed into A->u.bp.cell: setAabb for the bodies in creation order
DEV void bp_update(ArenaLDS* A) {
#pragma unroll 1
    for (int bi = 0; bi < 5; bi++) {
        const int cell = A->u.bp.cell[bi];
        if (cell == A->s.env.bp_cell[bi]) continue;
        A->s.env.bp_cell[bi] = (uint16_t)cell;
        int key[5];
#pragma unroll
        for (int c = 0; c < 5; c++) key[c] = c == bi ? 64 : bp_key(A, c);  // bi moves to the lists' end
#pragma unroll
        for (int c = 0; c < 5; c++) {
            int r = 0;
#pragma unroll
            for (int d = 0; d < 5; d++) r += key[d] < key[c];
            A->s.env.bp_rank[c] = (uint8_t)r;
        }
    }
}
DEV int commit_rank(const ArenaLDS* A, int rank) {
    if (rank < 25) return (rank / 5) * 9 + rank % 5;  // body * 9 + (0 mesh objects, 1-4 planes)
    int a, b;
    dyn_pair(rank, a, b);
    // body a's pairs with the later bodies, in its home cell's list order
    const int kb = bp_key(A, b);
    int pos = 0;
#pragma unroll
    for (int c = 1; c < 5; c++) pos += c > a && bp_key(A, c) < kb;
    return a * 9 + 5 + pos;
}
DEV void emit(ArenaLDS* A, int rank, int tri, int key, v3 n, v3 p, float depth) {
    int slot = atomicAdd(&A->a.ncand, 1);
    if (slot >= kMaxCand) return;  // counted by the committing lane
    Cand& c = A->u.cand[slot];
    c.n[0] = n.x; c.n[1] = n.y; c.n[2] = n.z;
    c.p[0] = p.x; c.p[1] = p.y; c.p[2] = p.z;
    c.depth = depth;
    c.order = (commit_rank(A, rank) << 20) | tri;
    c.key = key;
}

// SphereTriangleDetector::pointInTriangle / closestPointTriangle / collide (SphereTriangleDetector.cpp:88-240)
DEV bool point_in_triangle(v3 v0, v3 v1, v3 v2, v3 normal, v3 p) {
    v3 e1 = v1 - v0, e2 = v2 - v1, e3 = v0 - v2;
    v3 n1 = cross(e1, normal), n2 = cross(e2, normal), n3 = cross(e3, normal);
    float r1 = dot(p, n1) - dot(v0, n1);
    float r2 = dot(p, n2) - dot(v1, n2);
    float r3 = dot(p, n3) - dot(v2, n3);
    if (r1 > 0 && r2 > 0 && r3 > 0) return true;
    if (r1 <= 0 && r2 <= 0 && r3 <= 0) return true;
    return false;
}
DEV v3 closest_point_triangle(v3 p, v3 a, v3 b, v3 c) {
    v3 ab = b - a, ac = c - a, ap = p - a;
    float d1 = dot(ab, ap), d2 = dot(ac, ap);
    if (d1 <= 0.f && d2 <= 0.f) return a;
    v3 bp = p - b;
    float d3 = dot(ab, bp), d4 = dot(ac, bp);
    if (d3 >= 0.f && d4 <= d3) return b;
    v3 cp = p - c;
    float d5 = dot(ab, cp), d6 = dot(ac, cp);
    if (d6 >= 0.f && d5 <= d6) return c;
    float vc = d1 * d4 - d3 * d2;
    if (vc <= 0.f && d1 >= 0.f && d3 <= 0.f) {
        float vv = d1 / (d1 - d3);
        return a + ab * vv;
    }
    float vb = d5 * d2 - d1 * d6;
    if (vb <= 0.f && d2 >= 0.f && d6 <= 0.f) {
        float vv = d2 / (d2 - d6);
        return a + ac * vv;
    }
    float va = d3 * d6 - d5 * d4;
    if (va <= 0.f && (d4 - d3) >= 0.f && (d5 - d6) >= 0.f) {
        float vv = (d4 - d3) / ((d4 - d3) + (d5 - d6));
        return b + (c - b) * vv;
    }
    float denom = 1.f / (va + vb + vc);
    float vv = vb * denom, ww = vc * denom;
    return a + ab * vv + ac * ww;
}
DEV bool sphere_triangle(v3 center, float radius, v3 v0, v3 v1, v3 v2, float cbt, v3& point, v3& normal_out,
                         float& depth, int ar) {
    float rwt = radius + cbt;
    v3 normal = cross(v1 - v0, v2 - v0);
    float l2 = len2(normal);
    bool has = false;
    v3 cp = zero3();
    if (l2 >= kEps * kEps) {
        normal = normal / sqrtf(l2);
        v3 p1c = center - v0;
        float dfp = dot(p1c, normal);
        if (dfp < 0.f) {
            dfp *= -1.f;
            normal = normal * -1.f;
        }
        if (dfp < rwt) {
            if (point_in_triangle(v0, v1, v2, normal, center)) {
                has = true;
                cp = center - normal * dfp;
            } else {
                v3 nr = closest_point_triangle(center, v0, v1, v2);
                float d2 = len2(nr - center);
                if (d2 < rwt * rwt) {
                    has = true;
                    cp = nr;
                }
            }
        }
    }
    if (!has) return false;
    v3 c2c = center - cp;
    float d2 = len2(c2c);
    if (!(d2 < rwt * rwt)) return false;
    if (d2 > kEps) {
        float d = sqrtf(d2);
        normal_out = bt_normalize(c2c, ar);  // resultNormal.normalize() (SphereTriangleDetector.cpp:228)
        point = cp;
        depth = -(radius - d);
    } else {
        normal_out = normal;
        point = cp;
        depth = -radius;
    }
    return true;
}
DEV v3 box_support(const m3& R, v3 c, v3 dir_world) {
    v3 dl = vmul(dir_world, R);
    v3 lv = v3{dl.x >= 0 ? C.car_half.x : -C.car_half.x, dl.y >= 0 ? C.car_half.y : -C.car_half.y,
               dl.z >= 0 ? C.car_half.z : -C.car_half.z};
    return R * lv + c;
}
// Deferred box-triangle queries (narrow_queue -> narrow_deferred): a queue entry's top 4 bits tag it --
// 0 not deferred, 1..kPenSave its saved GJK state's slot + 1, kPenNoSave deferred without one (the rerun
// starts over).  The states sit in the workgroup's LDS (kPenSave x 44 B fits the allocation's rounding).
constexpr int kPenSave = 8;
constexpr uint32_t kPenTagShift = 28, kPenNoSave = 15;
struct PenSave {
    gjk::PenState st[kPenSave];
    int n;
    int cap;  // slots in use this launch (StepArgs::pen_slots: kPenSave, fewer to test the restart path)
};
static __shared__ PenSave g_pen_save;
// One car hitbox vs mesh triangle: Bullet's GJK / EPA query (gjk.hpp) and its candidate.  defer: a query
// that needs the penetration solver stops there and returns its tag (narrow_deferred reruns it on the whole
// wave); else the solver runs here, in the arena's small LDS set past the candidate list (free during the
// narrowphase), one lane at a time, or in this lane's HBM scratch.
__device__ __noinline__ uint32_t box_tri_query(ArenaLDS* A, const MeshView& M, int bi, int t, int obj, v3 v0, v3 v1, v3 v2, bool defer) {
    const m3 R = brot(A, bi);
    const v3 c = car_box_center(A, bi);
    gjk::Scr slow = gjk::hbm_view(M.gjk + ((size_t)blockIdx.x * kWG + threadIdx.x));
    gjk::Scr fast = gjk::lds_view((char*)&A->u.cand[kMaxCand]);
    const gjk::Shape sh{C.car_impl, C.car_margin, v0, v1, v2, arith(A)};
    v3 n, pb;
    float d;
    bool deferred = false;
    gjk::PenState st;
    if (gjk::box_triangle(R, c, sh, pair_cbt(bi, 10), &fast, &A->a.epa_lock, slow, n, pb, d, &A->a.npen,
                          defer ? gjk::kPenDefer : gjk::kPenInline, &deferred, &st))
        emit(A, bi * 5, t, mesh_key(bi, obj), n, pb, d);
    if (!deferred) return 0u;
    const int slot = atomicAdd(&g_pen_save.n, 1);
    if (slot >= g_pen_save.cap) return kPenNoSave;
    g_pen_save.st[slot] = st;
    return (uint32_t)slot + 1u;
}
// A deferred query (queue entry e, tag stripped; saved: its GJK state or null) on every lane of the wave:
// the penetration solver's EPA keeps its polytope in the wave's registers (gjk::epa_wave), its support
// vertices in the arena's small LDS set
__device__ __noinline__ void box_tri_query_wave(ArenaLDS* A, const MeshView& M, uint32_t e, const gjk::PenState* saved) {
    const int t = (int)(e & 0xFFFFFu), obj = (int)((e >> 20) & 31u), bi = (int)((e >> 25) & 7u);
    const float4 a = M.tri[3 * (size_t)t], b = M.tri[3 * (size_t)t + 1], cc = M.tri[3 * (size_t)t + 2];
    const m3 R = brot(A, bi);
    const v3 c = car_box_center(A, bi);
    gjk::Scr slow = gjk::hbm_view(M.gjk + ((size_t)blockIdx.x * kWG + threadIdx.x));
    gjk::Scr wave = gjk::wave_view((char*)&A->u.cand[kMaxCand]);
    const gjk::Shape sh{C.car_impl, C.car_margin, v3{a.x, a.y, a.z}, v3{b.x, b.y, b.z}, v3{cc.x, cc.y, cc.z}, arith(A)};
    v3 n, pb;
    float d;
    const bool hit = gjk::box_triangle(R, c, sh, pair_cbt(bi, 10), &wave, nullptr, slow, n, pb, d, &A->a.npen, gjk::kPenWave,
                                       nullptr, nullptr, saved);
    if (hit && threadIdx.x == 0) emit(A, bi * 5, t, mesh_key(bi, obj), n, pb, d);
}
// the queued box-triangle queries of the workgroup's arenas, dealt round-robin over all its lanes (an
// arena with many triangle contacts borrows the lanes of quiet ones); base = the workgroup's arenas,
// nvalid = how many of them exist.  Queries that need the penetration solver are flagged for
// narrow_deferred (a full wave: kWG == 64), else run it in place.  Each query is a call (inlining the
// queue's loop into one called function instead costs 1.08 -> 1.13 ms and 59 -> 89 MB of scratch writes
// per launch: the kernel's whole live state is saved around it every tick).
DEV void narrow_queue(ArenaLDS* base, int nvalid, const MeshView& M) {
    int start[kArenas + 1];
    start[0] = 0;
#pragma unroll
    for (int a = 0; a < kArenas; a++) start[a + 1] = start[a] + (a < nvalid ? stdmin(base[a].a.nq, kQueue) : 0);
    for (int k = threadIdx.x; k < start[kArenas]; k += kWG) {
        int ar = 0;
#pragma unroll
        for (int j = 1; j < kArenas; j++) ar += k >= start[j] ? 1 : 0;
        int off = start[0];
#pragma unroll
        for (int j = 1; j < kArenas; j++) off = ar == j ? start[j] : off;
        ArenaLDS* A = base + ar;
        const uint32_t e = A->a.q[k - off];
        const int t = (int)(e & 0xFFFFFu), obj = (int)((e >> 20) & 31u), bi = (int)((e >> 25) & 7u);
        const float4 a = M.tri[3 * (size_t)t], b = M.tri[3 * (size_t)t + 1], c = M.tri[3 * (size_t)t + 2];
        const uint32_t tag = box_tri_query(A, M, bi, t, obj, v3{a.x, a.y, a.z}, v3{b.x, b.y, b.z}, v3{c.x, c.y, c.z}, kWG == 64);
        if (tag) A->a.q[k - off] = e | (tag << kPenTagShift);
    }
}
// the flagged queries, arena by arena and in queue order, each on the whole wave (every lane calls this)
DEV void narrow_deferred(ArenaLDS* base, int nvalid, const MeshView& M) {
    if (kWG != 64) return;
    for (int ar = 0; ar < nvalid; ar++) {
        ArenaLDS* A = base + ar;
        const int nq = stdmin(A->a.nq, kQueue);
        for (int k0 = 0; k0 < nq; k0 += kWG) {
            const int k = k0 + (int)threadIdx.x;
            const uint32_t e = k < nq ? A->a.q[k] : 0u;
            uint64_t m = __ballot((e >> kPenTagShift) != 0);
            while (m) {
                const uint32_t ej = gjk::rdl(e, gjk::lowbit(m));
                m &= m - 1ull;
                const uint32_t tag = ej >> kPenTagShift;
                box_tri_query_wave(A, M, ej & ((1u << kPenTagShift) - 1u), tag <= kPenSave ? &g_pen_save.st[tag - 1] : nullptr);
            }
        }
    }
}

// ---- body-vs-mesh grid walks: each body's walk split over kMeshChunks lanes of its arena (narrow_pair).
// Dealing the entries of a workgroup's four arenas over all 64 lanes shortened the walk phase but not the
// launch (1.040 -> 1.053 ms, profiles/r05l_env_mesh_deal_ab.txt) and was removed.
// body bi's query box: the ball's sphere grown by 0.08 (SphereTriangleDetector's contact threshold margin),
// a car's compound AABB
DEV void mesh_box(ArenaLDS* A, int bi, v3& mn, v3& mx) {
    if (bi == 0) {
        const v3 c = bpos(A, 0);
        const float ext = C.ball_radius + 0.08f;
        mn = c - v3{ext, ext, ext};
        mx = c + v3{ext, ext, ext};
    } else {
        body_aabb(bi, bpos(A, bi), brot(A, bi), mn, mx);
    }
}
// one triangle of body bi's query: the ball's sphere-triangle test (SphereTriangleDetector, RocketSim
// variant), a car's box-triangle query queued for narrow_queue (a full queue runs it here)
DEV void mesh_hit(ArenaLDS* A, const MeshView& M, int bi, int t, v3 v0, v3 v1, v3 v2, int obj) {
    if (bi == 0) {
        v3 pt, nrm;
        float depth;
        if (sphere_triangle(bpos(A, 0), C.ball_radius, v0, v1, v2, pair_cbt(0, 10), pt, nrm, depth, arith(A)))
            emit(A, 0, t, mesh_key(0, obj), nrm, pt, depth);
    } else {
        const int slot = atomicAdd(&A->a.nq, 1);
        if (slot < kQueue)
            A->a.q[slot] = (uint32_t)t | ((uint32_t)obj << 20) | ((uint32_t)bi << 25);
        else
            box_tri_query(A, M, bi, t, obj, v0, v1, v2, false);
    }
}
// runs the narrowphase of one canonical pair rank and emits candidates; returns 1 when it ran.
// Body-vs-mesh ranks are split over `parts` lanes (grid entries dealt round-robin); candidates
// carry (rank, triangle), so the commit order does not depend on the split.
DEV int narrow_pair(ArenaLDS* A, const MeshView& M, int rank, int part = 0, int parts = 1) {
    const int ar = arith(A);
    if (rank < 25) {
        const int bi = rank / 5, st = rank % 5;
        bool active = bi == 0 ? A->a.ball_awake != 0 : A->a.active[bi] != 0;
        if (!active) return 0;
        const int pl = st - 1;
        if (bi == 0) {
            v3 c = bpos(A, 0);
            if (st > 0) {  // sphere vs plane (btConvexPlaneCollisionAlgorithm.cpp:53-90)
                v3 n = C.plane_n[pl];
                v3 vtx = c + (-n) * C.ball_radius;
                float dist = dot(n, vtx - C.plane_p[pl]);
                v3 on_plane = vtx - n * dist;
                if (dist < pair_cbt(0, 10)) emit(A, rank, 0, plane_key(0, pl), n, on_plane, dist);
            } else {  // sphere vs mesh triangles
                v3 mn, mx;
                mesh_box(A, 0, mn, mx);
                grid_query(M, mn, mx, part, parts, [&](int t, v3 v0, v3 v1, v3 v2, int obj) { mesh_hit(A, M, 0, t, v0, v1, v2, obj); });
            }
        } else {
            m3 R = brot(A, bi);
            if (st > 0) {  // box vs plane
                v3 n = C.plane_n[pl];
                v3 vtx = box_support(R, car_box_center(A, bi), -n);
                float dist = dot(n, vtx - C.plane_p[pl]);
                v3 on_plane = vtx - n * dist;
                if (dist < pair_cbt(bi, 10)) emit(A, rank, 0, plane_key(bi, pl), n, on_plane, dist);
            } else {
                // triangles past the AABB test are queued for Bullet's GJK / EPA query (box_tri_query),
                // which the workgroup's lanes then share (narrow_queue); a full queue runs them here
                v3 mn, mx;
                mesh_box(A, bi, mn, mx);
                grid_query(M, mn, mx, part, parts, [&](int t, v3 v0, v3 v1, v3 v2, int obj) { mesh_hit(A, M, bi, t, v0, v1, v2, obj); });
            }
        }
        return 1;
    }
    int ka, kb;
    dyn_pair(rank, ka, kb);
    const int key = dyn_key(ka, kb);
    // ball pairs are computed with the box as the algorithm's body (A_ = car, B_ = ball)
    int A_ = ka == 0 ? kb : ka, B_ = ka == 0 ? 0 : kb;
    bool dem = (A_ >= 1 && !A->a.active[A_]) || (B_ >= 1 && !A->a.active[B_]);
    v3 m0, m1, n0, n1;
    broad_aabb(A, A_, m0, m1);
    broad_aabb(A, B_, n0, n1);
    if (dem || !aabb_overlap(m0, m1, n0, n1)) return 0;
    bool act_a = A_ == 0 ? A->a.ball_awake != 0 : A->a.active[A_] != 0;
    bool act_b = B_ == 0 ? A->a.ball_awake != 0 : A->a.active[B_] != 0;
    if (!act_a && !act_b) return 0;
    if (B_ == 0) {  // btSphereBoxCollisionAlgorithm::getSphereDistance, A = car, B = ball
        m3 R = brot(A, A_);
        v3 c = car_box_center(A, A_);
        const float margin = C.car_margin;  // boxShape->getMargin() (btSphereBoxCollisionAlgorithm.cpp:82-90)
        const v3 he = C.car_impl;          // getHalfExtentsWithoutMargin
        v3 rel = vmul(bpos(A, 0) - c, R);
        v3 cp = v3{stdmax(-he.x, stdmin(he.x, rel.x)), stdmax(-he.y, stdmin(he.y, rel.y)), stdmax(-he.z, stdmin(he.z, rel.z))};
        float r = C.ball_radius;
        float inter = r + margin;
        float cbt = pair_cbt(A_, 0);
        float contact_dist = inter + cbt;
        v3 normal = rel - cp;
        float d2 = len2(normal);
        if (d2 > contact_dist * contact_dist) return 1;
        float distance;
        if (d2 <= kEps) {
            float fd[6] = {he.x - rel.x, he.x + rel.x, he.y - rel.y, he.y + rel.y, he.z - rel.z, he.z + rel.z};
            int bf = 0;
            float fmin = fd[0];
#pragma unroll
            for (int k = 1; k < 6; k++)
                if (fd[k] < fmin) bf = k, fmin = fd[k];
            cp = rel;
            int axis = bf / 2;
            float sg = (bf % 2 == 0) ? 1.f : -1.f;
            set_comp(cp, axis, sg * comp(he, axis));
            v3 nn = zero3();
            set_comp(nn, axis, sg);
            normal = nn;
            distance = -fmin;
        } else {
            distance = len(normal);
            normal = normal / distance;
        }
        v3 point_on_box = R * (cp + normal * margin) + c;
        float pen = distance - inter;
        v3 nw = R * normal;
        // manifold (A = ball, B = car): normal on the car towards the ball, point on the car
        // (btSphereBoxCollisionAlgorithm.cpp:66-75 -> btManifoldResult::addContactPoint unswapped)
        emit(A, rank, 0, key, nw, point_on_box, pen);
        return 1;
    }
    // car vs car: btBoxBoxDetector / dBoxBox2 (boxbox.hpp), A = car ka, B = car kb, up to 4 points in
    // emission order (the point index orders them at the commit)
    {
        int j = 0;
        boxbox::box_box(car_box_center(A, A_), brot(A, A_), C.car_half, car_box_center(A, B_), brot(A, B_), C.car_half,
                        [&](v3 n, v3 p, float d) { emit(A, rank, j++, key, n, p, d); });
    }
    return 1;
}

// the commit order of this tick's candidates, on the arena's 16 lanes: candidate i goes to position
// #{j : order_j < order_i, or order_j == order_i and j < i} -- the stable order the single-lane insertion sort
// gave -- written as a permutation into the narrowphase's free LDS tail (the penetration solver's small set)
DEV uint8_t* cand_perm(ArenaLDS* A) { return (uint8_t*)&A->u.cand[kMaxCand]; }
DEV void sort_candidates(ArenaLDS* A, int l) {
    const int n = min(A->a.ncand, kMaxCand);
    uint8_t* perm = cand_perm(A);
    for (int i = l; i < n; i += kTeam) {
        const int oi = A->u.cand[i].order;
        int r = 0;
        for (int j = 0; j < n; j++) {
            const int oj = A->u.cand[j].order;
            r += (oj < oi) || (oj == oi && j < i);
        }
        perm[r] = (uint8_t)i;
    }
}
// single lane: commit this tick's candidates in the broadphase's pair order (sort_candidates) -- per pair
// (key): add its points (contact callbacks fire here), then refresh its manifold, as Bullet's dispatch loop
// does (btCollisionDispatcher::dispatchAllCollisionPairs, processCollision -> refreshContactPoints)
DEV void commit_contacts(ArenaLDS* A, const MeshView& M, Prof* P = nullptr) {
    int n = A->a.ncand;
    if (n > kMaxCand) {
        A->s.env.manifold_overflow += (uint32_t)(n - kMaxCand);
        n = kMaxCand;
    }
    const uint8_t* perm = cand_perm(A);
    pmark(P, 17);
    if (P && P->p && threadIdx.x == 0) atomicAdd(&P->p[24], (unsigned long long)n);
    A->a.nmf = 0;  // the previous tick's manifolds were destroyed with their pairs
    int cur = -1;
    for (int ci = 0; ci < n; ci++) {
        const Cand& c = A->u.cand[perm[ci]];
        if (c.key != cur) {
            if (cur >= 0) refresh(A, cur);
            cur = c.key;
        }
        // mesh-object keys carry their triangle in the low bits of the commit order
        int ka, kb;
        key_bodies(c.key, ka, kb);
        const int tri = (c.key < kDynKey && kb - 10 < kMaxObj) ? (c.order & (kMaxTris - 1)) : -1;
        add_contact(A, M, c.key, v3{c.n[0], c.n[1], c.n[2]}, v3{c.p[0], c.p[1], c.p[2]}, c.depth, tri);
    }
    if (cur >= 0) refresh(A, cur);
    if (P && P->p && threadIdx.x == 0) atomicAdd(&P->p[26], (unsigned long long)A->a.nmf);
}

// ------------------------------------------------------------------ sequential impulse solver
DEV void setup_contact(ArenaLDS* A, Solver& S, CRow& row, int ia, int ib, const rlgpu_contact& cp, v3 rel1, v3 rel2,
                       float dist) {
    SB& Sa = S.sb[ia];
    SB& Sb = S.sb[ib];
    bool r0 = Sa.real != 0, r1 = Sb.real != 0;
    v3 n = ld3(cp.normalB);
    v3 t0 = cross(rel1, n);
    row.angA = r0 ? A->a.iiw[ia] * t0 : zero3();
    v3 t1 = cross(rel2, n);
    row.angB = r1 ? A->a.iiw[ib] * -t1 : zero3();
    float d0 = 0, d1 = 0;
    if (r0) d0 = binv_mass(ia) + dot(n, cross(row.angA, rel1));
    if (r1) d1 = binv_mass(ib) + dot(n, cross(-row.angB, rel2));
    row.jinv = 1.f / (d0 + d1 + 0.f);
    row.n1 = r0 ? n : zero3();
    row.rc1 = r0 ? t0 : zero3();
    row.n2 = r1 ? -n : zero3();
    row.rc2 = r1 ? -t1 : zero3();
    float penetration = dist + 0.f;
    v3 v1 = r0 ? vel_at(A, ia, rel1) : zero3();
    v3 v2 = r1 ? vel_at(A, ib, rel2) : zero3();
    float rel_vel = dot(n, v1 - v2);
    row.friction = cp.friction;
    float restitution = fabsf(rel_vel) < 0.2f ? 0.f : cp.restitution * -rel_vel;
    if (restitution <= 0.f) restitution = 0.f;
    row.applied = cp.applied * 0.85f;
    // warm start (a fresh point's applied impulse is 0: adding the zero product leaves the +0 deltas
    // unchanged, so it is skipped and rows can be set up concurrently)
    if (r0 && row.applied != 0.f) {
        Sa.dlin += row.n1 * v3{Sa.inv_mass, Sa.inv_mass, Sa.inv_mass} * row.applied;
        Sa.dang += row.angA * row.applied;
    }
    if (r1 && row.applied != 0.f) {
        Sb.dlin += (-row.n2 * v3{Sb.inv_mass, Sb.inv_mass, Sb.inv_mass}) * -row.applied;
        Sb.dang += -row.angB * -row.applied;
    }
    row.applied_push = 0;
    float v1n = dot(row.n1, Sa.lin + (r0 ? Sa.ext_f : zero3())) + dot(row.rc1, Sa.ang + (r0 ? Sa.ext_t : zero3()));
    float v2n = dot(row.n2, Sb.lin + (r1 ? Sb.ext_f : zero3())) + dot(row.rc2, Sb.ang + (r1 ? Sb.ext_t : zero3()));
    float rv = v1n + v2n;
    float pos_err = 0, vel_err = restitution - rv;
    if (penetration > 0) {
        pos_err = 0;
    } else {
        pos_err = -penetration * 0.8f * (1.f / kTick);
    }
    row.rhs = vel_err * row.jinv;
    row.rhs_pen = pos_err * row.jinv;
}

DEV void add_friction(ArenaLDS* A, Solver& S, int ia, int ib, const rlgpu_contact& cp, v3 rel1, v3 rel2, int cidx,
                      float friction) {
    SB& Sa = S.sb[ia];
    SB& Sb = S.sb[ib];
    bool r0 = Sa.real != 0, r1 = Sb.real != 0;
    v3 n = ld3(cp.normalB);
    v3 va = r0 ? Sa.lin + Sa.ext_f + cross(Sa.ang + Sa.ext_t, rel1) : zero3();
    v3 vb = r1 ? Sb.lin + Sb.ext_f + cross(Sb.ang + Sb.ext_t, rel2) : zero3();
    v3 vel = va - vb;
    float rel_vel = dot(n, vel);
    v3 dir = vel - n * rel_vel;
    float lat = len2(dir);
    if (lat > kEps) {
        dir = dir * (1.f / sqrtf(lat));
    } else {  // btPlaneSpace1
        if (fabsf(n.z) > 0.7071067811865475244008443621048490f) {
            float a = n.y * n.y + n.z * n.z;
            float k = 1.f / sqrtf(a);
            dir = v3{0, -n.z * k, n.y * k};
        } else {
            float a = n.x * n.x + n.y * n.y;
            float k = 1.f / sqrtf(a);
            dir = v3{-n.y * k, n.x * k, 0};
        }
    }
    FRow& f = S.frows[cidx];
    f.a = ia;
    f.b = ib;
    f.friction = friction;
    f.applied = 0;
    f.cidx = cidx;
    if (r0) {
        f.n1 = dir;
        v3 ta = cross(rel1, dir);
        f.rc1 = ta;
        f.angA = A->a.iiw[ia] * ta;
    } else {
        f.n1 = f.rc1 = f.angA = zero3();
    }
    if (r1) {
        f.n2 = -dir;
        v3 tb = cross(rel2, f.n2);
        f.rc2 = tb;
        f.angB = A->a.iiw[ib] * tb;
    } else {
        f.n2 = f.rc2 = f.angB = zero3();
    }
    float d0 = 0, d1 = 0;
    if (r0) d0 = binv_mass(ia) + dot(dir, cross(f.angA, rel1));
    if (r1) d1 = binv_mass(ib) + dot(dir, cross(-f.angB, rel2));
    f.jinv = 1.f / (d0 + d1);
    float v1n = dot(f.n1, r0 ? Sa.lin + Sa.ext_f : zero3()) + dot(f.rc1, r0 ? Sa.ang : zero3());
    float v2n = dot(f.n2, r1 ? Sb.lin + Sb.ext_f : zero3()) + dot(f.rc2, r1 ? Sb.ang : zero3());
    f.rhs = (0.f - (v1n + v2n)) * f.jinv;
    f.lower = -friction;
    f.upper = friction;
}

// A row's dot with a body's velocity deltas, in the order of the row function the reference build runs:
// the _sse2 rows' btSimdDot3 x + (y + z) (btSequentialImpulseConstraintSolver.cpp:106-110), the MSVC
// _sse4_1_fma3 rows' _mm_dp_ps(a, b, 0x7f) -- products, then lanes (0 + 1) + (2 + 3) with lane 3 zeroed --
// i.e. (x + y) + (z + 0) (:122-124), and the scalar rows' btVector3::dot (x + y) + z.
enum { kDotScalar = 0, kDotSse2 = 1, kDotDpps = 2 };
DEV float row_dot(v3 a, v3 b, int how) {
    const float x = a.x * b.x, y = a.y * b.y, z = a.z * b.z;
    if (how == kDotSse2) return x + (y + z);
    if (how == kDotDpps) return (x + y) + (z + 0.f);
    return (x + y) + z;
}

// One contact (lower limit only) or friction (generic) row: gResolveSingleConstraintRow{LowerLimit,Generic}_
// scalar_reference (:46-100), _sse2 (:149-177, 207-233) or _sse4_1_fma3 (:180-205, 235-260) by the set's
// arithmetic mode.  The x86 rows differ from the scalar one in the dot order, in the clamp at equality
// (_sse2 clamps to the upper limit when sum == upper; _sse4_1_fma3 clamps when sum <= lower or sum >= upper)
// and, for _sse4_1_fma3, in fused multiply-adds for the delta and the velocity updates.  Static / inactive
// bodies are not updated: the reference adds (n * 0) * di to its fixed body's zero deltas, which stay +0.
template <class Row>
DEV void resolve_row(Solver& S, Row& c, float lower, float upper, bool generic, int ar) {
    SB& A = S.sb[c.a];
    SB& B = S.sb[c.b];
    const bool fma3 = ar == RLGPU_ARITH_MSVC_X64;
    const int how = fma3 ? kDotDpps : (ar == RLGPU_ARITH_GCC_X64 ? kDotSse2 : kDotScalar);
    float di = c.rhs - c.applied * 0.f;
    const float dv1 = row_dot(c.n1, A.dlin, how) + row_dot(c.rc1, A.dang, how);
    const float dv2 = row_dot(c.n2, B.dlin, how) + row_dot(c.rc2, B.dang, how);
    if (fma3) {  // FMNADD: -(dv * jac) + di, fused
        di = fmaf(-dv1, c.jinv, di);
        di = fmaf(-dv2, c.jinv, di);
    } else {
        di -= dv1 * c.jinv;
        di -= dv2 * c.jinv;
    }
    const float applied = c.applied, sum = applied + di;
    if (fma3) {  // blendv on sum > lower and upper > sum
        const bool above = sum > lower, below = !generic || upper > sum;
        di = above ? (below ? di : upper - applied) : lower - applied;
        c.applied = above ? (below ? sum : upper) : lower;
    } else if (ar == RLGPU_ARITH_GCC_X64) {  // and / andnot selects on sum < lower, then sum < upper
        const bool low = sum < lower;
        float d = low ? lower - applied : di, ap = low ? lower : sum;
        if (generic && !(sum < upper)) {
            d = upper - applied;
            ap = upper;
        }
        di = d;
        c.applied = ap;
    } else if (sum < lower) {
        di = lower - applied;
        c.applied = lower;
    } else if (generic && sum > upper) {
        di = upper - applied;
        c.applied = upper;
    } else {
        c.applied = sum;
    }
    if (fma3) {  // FMADD(n * invMass, di, delta), FMADD(angular component, di, delta)
        if (A.real) {
            const v3 la = c.n1 * v3{A.inv_mass, A.inv_mass, A.inv_mass};
            A.dlin = v3{fmaf(la.x, di, A.dlin.x), fmaf(la.y, di, A.dlin.y), fmaf(la.z, di, A.dlin.z)};
            A.dang = v3{fmaf(c.angA.x, di, A.dang.x), fmaf(c.angA.y, di, A.dang.y), fmaf(c.angA.z, di, A.dang.z)};
        }
        if (B.real) {
            const v3 lb = c.n2 * v3{B.inv_mass, B.inv_mass, B.inv_mass};
            B.dlin = v3{fmaf(lb.x, di, B.dlin.x), fmaf(lb.y, di, B.dlin.y), fmaf(lb.z, di, B.dlin.z)};
            B.dang = v3{fmaf(c.angB.x, di, B.dang.x), fmaf(c.angB.y, di, B.dang.y), fmaf(c.angB.z, di, B.dang.z)};
        }
    } else {
        if (A.real) {
            A.dlin += c.n1 * v3{A.inv_mass, A.inv_mass, A.inv_mass} * di;
            A.dang += c.angA * di;
        }
        if (B.real) {
            B.dlin += c.n2 * v3{B.inv_mass, B.inv_mass, B.inv_mass} * di;
            B.dang += c.angB * di;
        }
    }
}
// gResolveSplitPenetrationImpulse_scalar_reference (:283-313) / _sse2 (:315-350; both x86 builds, MSVC has no
// fused split row): only the dot order differs.  The residual is deltaImpulse * (1. / jacDiagABInv) in
// double, returned as float.
DEV float resolve_split(Solver& S, CRow& c, int ar) {
    float di = 0.f;
    if (c.rhs_pen != 0.f) {
        SB& A = S.sb[c.a];
        SB& B = S.sb[c.b];
        const int how = sse_api(ar) ? kDotSse2 : kDotScalar;
        di = c.rhs_pen - c.applied_push * 0.f;
        float dv1 = row_dot(c.n1, A.push, how) + row_dot(c.rc1, A.turn, how);
        float dv2 = row_dot(c.n2, B.push, how) + row_dot(c.rc2, B.turn, how);
        di -= dv1 * c.jinv;
        di -= dv2 * c.jinv;
        float sum = c.applied_push + di;
        if (sum < 0.f) {
            di = 0.f - c.applied_push;
            c.applied_push = 0.f;
        } else {
            c.applied_push = sum;
        }
        if (A.real) {
            A.push += c.n1 * v3{A.inv_mass, A.inv_mass, A.inv_mass} * di;
            A.turn += c.angA * di;
        }
        if (B.real) {
            B.push += c.n2 * v3{B.inv_mass, B.inv_mass, B.inv_mass} * di;
            B.turn += c.angB * di;
        }
    }
    return (float)((double)di * (1. / (double)c.jinv));
}

// max over the 16 lanes of an arena (xor partners stay inside the 16-lane group)
DEV float group16_max(float v) {
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) v = stdmax(v, __shfl_xor(v, o, 64));
    return v;
}

// btSequentialImpulseConstraintSolver::solveGroup on the 16 lanes of an arena.
// Bullet sweeps the rows in order (Gauss-Seidel), and a row reads and writes only the velocity
// deltas of its own two bodies.  Lane 0 gives row r the level 1 + max(level of the last earlier row
// sharing a dynamic body with it); level L's rows then run concurrently, row r on lane r
// (kMaxRows <= 16), after level L - 1's.  Every body therefore receives its updates in the
// sequential order, from the same operands: the same bits as the one-lane sweep, in as many steps
// as the longest chain of rows on one body instead of one step per row.  Rows are set up
// concurrently too (independent: a fresh point's warm start is zero), bodies one per lane.
// Called by all threads of the workgroup (it synchronises); `valid`: this lane's arena exists.
DEV void solve_lanes(ArenaLDS* A, int l, bool valid, Prof* P = nullptr) {
    Solver& S = A->u.sv;
    const int ar = arith(A);
    static_assert(kMaxRows <= kTeam, "one lane per solver row");
    if (valid && l < 5) {  // bodies (btSolverBody init), one per lane
        const int i = l;
        bool act = i == 0 ? A->a.ball_awake != 0 : A->a.active[i] != 0;
        SB& x = S.sb[i];
        x.dlin = x.dang = x.push = x.turn = zero3();
        x.real = act;
        if (act) {
            float im = binv_mass(i);
            x.inv_mass = im;
            x.lin = bvel(A, i);
            x.ang = bang(A, i);
            x.ext_f = A->a.force[i] * im * kTick;
            x.ext_t = vmul(A->a.torque[i], A->a.iiw[i]) * kTick;
        } else {
            x.inv_mass = 0.f;
            x.lin = x.ang = x.ext_f = x.ext_t = zero3();
        }
        S.spec_num[i] = 0;
        S.spec_fric[i] = 0;
        S.spec_rest[i] = 0;
        S.spec_d[i] = 0;
        S.spec_n[i] = zero3();
    } else if (valid && l == 5) {
        SB& f = S.sb[5];
        f.dlin = f.dang = f.push = f.turn = f.lin = f.ang = f.ext_f = f.ext_t = zero3();
        f.inv_mass = 0.f;
        f.real = 0;
    }
    sync();
    pmark(P, 19);
    if (valid && l == 0) {  // the rows' (manifold, point) in creation order; the special-point sums
        unsigned in_solver = 0;
        for (int i = 0; i < 5; i++)
            if (S.sb[i].real) in_solver |= 1u << i;
        S.in_solver = in_solver;
        int nrows = 0;
        for (int mi = 0; mi < A->a.nmf; mi++) {
            rlgpu_manifold& mf = A->mf[mi];
            if (mf.count == 0) continue;
            int a, b;
            key_bodies(mf.key, a, b);
            bool aact = a < 10 && ((in_solver >> a) & 1u);
            bool bact = b < 10 && ((in_solver >> b) & 1u);
            if (!aact && !bact) continue;
            for (int j = 0; j < mf.count; j++) {
                if (nrows >= kMaxRows) {
                    A->s.env.manifold_overflow++;
                    continue;
                }
                rlgpu_contact& cp = mf.pts[j];
                if (cp.special) {
                    v3 pa_, pb_;
                    m3 ra, rb;
                    side_transform(A, a, pa_, ra);
                    side_transform(A, b, pb_, rb);
                    v3 wa = ra * ld3(cp.localA) + pa_;
                    v3 wb = rb * ld3(cp.localB) + pb_;
                    v3 rel1 = wa - pa_;
                    v3 rel2 = wb - (b >= 10 ? zero3() : pb_);
                    for (int side = 0; side < 2; side++) {
                        int bid = side ? b : a;
                        if (bid < 10) {
                            S.spec_num[bid]++;
                            S.spec_fric[bid] = cp.friction;
                            S.spec_rest[bid] = cp.restitution;
                            S.spec_n[bid] += ld3(cp.normalB);
                            S.spec_d[bid] += len(side ? rel2 : rel1);
                        }
                    }
                }
                S.rmf[nrows] = (int8_t)mi;
                S.rpt[nrows] = (int8_t)j;
                nrows++;
            }
        }
        S.nmrows = nrows;
        for (int i = 0; i < 5; i++) {  // the averaged special rows, after the manifold rows
            if (S.spec_num[i] <= 0 || !((in_solver >> i) & 1u)) continue;
            if (nrows >= kMaxRows) {
                A->s.env.manifold_overflow++;
                continue;
            }
            float distance = S.spec_d[i] / S.spec_num[i];
            v3 normal = S.spec_n[i] / (float)S.spec_num[i];
            rlgpu_contact tmp;
            st3(tmp.localA, zero3());
            st3(tmp.localB, zero3());
            st3(tmp.normalB, normal);
            tmp.dist = distance;
            tmp.applied = 0.f;
            tmp.friction = S.spec_fric[i];
            tmp.restitution = S.spec_rest[i];
            tmp.special = 0;
            v3 rel1 = normal * -distance, rel2 = zero3();
            CRow& row = S.rows[nrows];
            row.a = i;
            row.b = 5;
            row.special = 0;
            setup_contact(A, S, row, i, 5, tmp, rel1, rel2, distance);
            add_friction(A, S, i, 5, tmp, rel1, rel2, nrows, tmp.friction);
            nrows++;
        }
        S.nrows = nrows;
    }
    sync();
    if (valid && l < S.nmrows) {  // manifold row l
        const unsigned in_solver = S.in_solver;
        rlgpu_manifold& mf = A->mf[S.rmf[l]];
        int a, b;
        key_bodies(mf.key, a, b);
        bool aact = a < 10 && ((in_solver >> a) & 1u);
        bool bact = b < 10 && ((in_solver >> b) & 1u);
        int ia = aact ? a : 5, ib = bact ? b : 5;
        v3 pa_, pb_;
        m3 ra, rb;
        side_transform(A, a, pa_, ra);
        side_transform(A, b, pb_, rb);
        rlgpu_contact& cp = mf.pts[S.rpt[l]];
        v3 wa = ra * ld3(cp.localA) + pa_;
        v3 wb = rb * ld3(cp.localB) + pb_;
        v3 rel1 = wa - pa_;
        v3 rel2 = wb - (b >= 10 ? zero3() : pb_);
        CRow& row = S.rows[l];
        row.a = ia;
        row.b = ib;
        row.special = cp.special != 0;
        setup_contact(A, S, row, ia, ib, cp, rel1, rel2, cp.dist);
        add_friction(A, S, ia, ib, cp, rel1, rel2, l, cp.friction);
    }
    sync();
    if (valid && l == 0) {  // sweep levels
        for (int i = 0; i < 6; i++) S.blev[i] = -1;
        int nlev = 0;
        for (int r = 0; r < S.nrows; r++) {
            const int a = S.rows[r].a, b = S.rows[r].b;  // 5 = static / inactive: never written
            const int lv = stdmax(a < 5 ? S.blev[a] : -1, b < 5 ? S.blev[b] : -1) + 1;
            S.lvl[r] = (int8_t)lv;
            if (a < 5) S.blev[a] = lv;
            if (b < 5) S.blev[b] = lv;
            nlev = stdmax(nlev, lv + 1);
        }
        S.nlev = nlev;
    }
    sync();
    pmark(P, 20);
    int nlev = valid ? S.nlev : 0;  // workgroup-uniform: the max over its arenas
#pragma unroll
    for (int o = kWG / 2; o > 0; o >>= 1) nlev = stdmax(nlev, __shfl_xor(nlev, o, 64));
    const bool mine = valid && l < S.nrows;
    const int lv = mine ? S.lvl[l] : -1;
    // this lane's contact and friction rows stay in registers for the sweeps (only the bodies'
    // deltas travel through LDS); the impulses they accumulate die with the tick
    CRow cr;
    FRow fr;
    if (mine) {
        cr = S.rows[l];
        fr = S.frows[l];
    }
    // split-impulse iterations (solveGroupCacheFriendlySplitImpulseIterations): until no row pushes
    bool done = !valid;
    for (int it = 0; it < 10; it++) {
        float lsr = 0.f;
        for (int L = 0; L < nlev; L++) {
            if (!done && lv == L) {
                float res = resolve_split(S, cr, ar);
                lsr = stdmax(lsr, res * res);
            }
            sync();
        }
        lsr = group16_max(lsr);
        if (lsr <= 0.f || it >= 9) done = true;
        if (__all(done)) break;
    }
    // velocity iterations: every contact row, then every friction row (bounded by its contact's impulse)
    const bool special = mine && cr.special;
    for (int it = 0; it < 10; it++) {
        for (int L = 0; L < nlev; L++) {
            if (lv == L && !special) resolve_row(S, cr, 0.f, 1e10f, false, ar);
            sync();
        }
        for (int L = 0; L < nlev; L++) {
            if (lv == L) {
                float total = cr.applied;  // frows[l].cidx == l
                if (total > 0.f) {
                    fr.lower = -(fr.friction * total);
                    fr.upper = fr.friction * total;
                    resolve_row(S, fr, fr.lower, fr.upper, true, ar);
                }
            }
            sync();
        }
    }
    pmark(P, 21);
    // (the applied impulses are not written back: the manifolds die with this tick)
    if (valid && l < 5 && ((S.in_solver >> l) & 1u)) {  // one body per lane
        const int i = l;
        SB& x = S.sb[i];
        rlgpu_body* bd = body(A, i);
        x.lin += x.dlin;
        x.ang += x.dang;
        if (!(x.push.x == 0 && x.push.y == 0 && x.push.z == 0 && x.turn.x == 0 && x.turn.y == 0 && x.turn.z == 0)) {
            if (i == 0) {
                st3(bd->pos, ld3(bd->pos) + x.push * kTick);
            } else {
                v3 np;
                m3 nr;
                integrate_transform(ld3(bd->pos), ldm(bd->rot), x.push, x.turn * 0.1f, kTick, np, nr, ar);
                st3(bd->pos, np);
                stm(bd->rot, nr);
            }
        }
        st3(bd->vel, x.lin + x.ext_f);
        st3(bd->angvel, x.ang + x.ext_t);
    }
}

}  // namespace rl
