// gae.hip -- GAE on MI355X.
//
// Semantics follow GGL::GAE::Compute
// (GigaLearnCPP/src/private/GigaLearnCPP/PPO/GAE.cpp:7-208):
//   * rewards normalised by 1/returnStd when returnStd is not 0 or 1 (:74-76,104-167),
//     then clipped to +-clipRange (clipRange > 0);
//   * nextVal = 0 on NORMAL, truncValPreds[k] on the k-th TRUNCATED step (:86-96),
//     V[t+1] otherwise, 0 on the last step (:97-101);
//   * delta = r_hat + gamma*nextVal - V;  A_t = delta + gamma*lambda*nd_t*A_{t+1} (:177-190);
//   * returns use the RAW reward: R_t = r_t + R_{t+1}*gamma*nd_t (:183-185);
//   * target = V + A (:200); clip portion = (sum|n| - sum|clip(n)|)/max(sum|n|,1e-7) (:202-206).
//
// Two device layouts:
//   * rollout [T][N]: one lane per agent column walks t backwards in the reference's
//     operation order (compiled with -ffp-contract=off) -> bit-identical to the oracle;
//     memory access is coalesced across the agent dimension, so it is an HBM-streaming
//     kernel (21 B per agent-step algorithmic).
//   * flat (episode-concatenated, the reference's own input): A_t = d_t + c_t*A_{t+1} is a
//     composition of affine maps, (cL,dL)o(cR,dR) = (cL*cR, dL + cL*dR).  Terminals make c=0,
//     so one non-segmented reverse scan is exactly the segmented GAE.  Three streaming passes
//     over 8192-element tiles (tile summaries with the truncation value left symbolic -> one
//     workgroup resolves truncation indices and tile carries -> apply), float4 accesses, a
//     fixed composition order (the same result on every run); see k_flat_summary.
#include <mutex>
#include <vector>

#include "common.hpp"
#include "../../include/rlgpu_gae.h"

namespace {

constexpr int8_t kNormal = 1, kTruncated = 2;   // RLGC::TerminalType (TerminalCondition.h:6-11)

struct Aff {
    float c, d;
};
__device__ __forceinline__ Aff compose(Aff L, Aff R) { return {L.c * R.c, L.d + L.c * R.d}; }
__device__ __forceinline__ Aff shfl_down_aff(Aff a, int off) {
    return {__shfl_down(a.c, off, 64), __shfl_down(a.d, off, 64)};
}

// Per-element GAE parameters shared by the flat kernels.
struct GaeParams {
    const float* rews;
    const int8_t* terms;
    const float* vals;
    const float* trunc_vals;
    int64_t M;
    int64_t num_truncs;
    float gamma, gamma_lambda, inv_std;
    bool normalize, clip;
    float clip_range;
};

// ---- flat layout: three passes, each a streaming pass over 8192-element tiles ---------------------------------
// The apply pass walks a tile in 8 rounds of 1024 elements, thread l owning elements 4l .. 4l + 3 of a round
// (one float4 of each array: every load and store of a wave is one contiguous 1 KB); the summary pass in 4
// rounds of 2048, 8 elements per thread (8 per thread in the apply pass measured 65 -> 69 us at 2^24).  Pass 1 (k_flat_summary) composes each
// tile's maps and counts its truncations; pass 2 (k_flat_carry, one workgroup) turns the counts into each
// tile's first truncation index and the maps into the value entering each tile from the right; pass 3
// (k_flat_apply) rebuilds the maps with the exact truncation values and writes A, target, R.  The
// composition order is fixed by the tiling, so the result is the same on every run.
//
// The summary cannot know its truncation values (their index is a forward count over the tiles to its
// left), so it composes maps of the form x -> c x + d + b T, T = the value of the tile's first truncation:
// the tile's first terminal zeroes every coefficient to its right, so only that T can survive.  The carry pass
// resolves such a tile as d + b T, i.e. the truncation element's delta as (n - v) + gamma T, where the apply
// pass writes that element as (n + gamma T) - v: the carry into the tile to the left is the reassociated form
// (same inputs, fixed order -- deterministic, within the 1e-5 contract of tests/test_gae.py, but not the
// bits of a single sequential walk at those elements).
constexpr int kFT = 256, kFV = 4;
constexpr int kFTile = 8192;
constexpr int kFRound = kFT * kFV, kFRounds = kFTile / kFRound;  // the apply pass: rounds of 1024
constexpr int kCT = 1024;  // the carry pass's workgroup

struct Aff3 {
    float c, d, b;
};
__device__ __forceinline__ Aff3 compose3(Aff3 L, Aff3 R) { return {L.c * R.c, L.d + L.c * R.d, L.b + L.c * R.b}; }

// one thread's 4 elements of a round starting at i0 (tail elements past M load as NORMAL zeros: their
// maps are never applied and the tile's real maps end before them)
struct Quad {
    float r[kFV], v[kFV];
    int8_t t[kFV];
    float vnext;  // vals[i0 + 4] (0 past the end)
};
template <bool VEC>
__device__ __forceinline__ void load_quad_raw(const GaeParams& p, int64_t i0, Quad& q) {
    if (VEC && i0 + kFV <= p.M) {
        const float4 r = *reinterpret_cast<const float4*>(p.rews + i0);
        const float4 v = *reinterpret_cast<const float4*>(p.vals + i0);
        const uint32_t t = *reinterpret_cast<const uint32_t*>(p.terms + i0);
        q.r[0] = r.x, q.r[1] = r.y, q.r[2] = r.z, q.r[3] = r.w;
        q.v[0] = v.x, q.v[1] = v.y, q.v[2] = v.z, q.v[3] = v.w;
#pragma unroll
        for (int j = 0; j < kFV; j++) q.t[j] = (int8_t)(t >> (8 * j));
    } else {
#pragma unroll
        for (int j = 0; j < kFV; j++) {
            const bool in = i0 + j < p.M;
            q.r[j] = in ? p.rews[i0 + j] : 0.f;
            q.v[j] = in ? p.vals[i0 + j] : 0.f;
            q.t[j] = in ? p.terms[i0 + j] : kNormal;
        }
    }
}
// the value after element i0 + span - 1 when the next lane's first element is i0 + span: its v0, lane 63 (and
// the array's end) from memory
__device__ __forceinline__ float next_lane_val(const GaeParams& p, int64_t i0, int span, float v0) {
    const float nb = __shfl_down(v0, 1, 64);
    if (i0 + span >= p.M) return 0.f;
    return ((threadIdx.x & 63) != 63) ? nb : p.vals[i0 + span];
}
template <bool VEC>
__device__ __forceinline__ void load_quad(const GaeParams& p, int64_t i0, Quad& q) {
    load_quad_raw<VEC>(p, i0, q);
    q.vnext = next_lane_val(p, i0, kFV, q.v[0]);
}
// elements i0 .. i0 + 7 of a thread whose next lane starts at i0 + 8
template <bool VEC>
__device__ __forceinline__ void load_octet(const GaeParams& p, int64_t i0, Quad (&e)[2]) {
    load_quad_raw<VEC>(p, i0, e[0]);
    load_quad_raw<VEC>(p, i0 + kFV, e[1]);
    e[0].vnext = i0 + kFV < p.M ? e[1].v[0] : 0.f;
    e[1].vnext = next_lane_val(p, i0, 2 * kFV, e[0].v[0]);
}

__device__ __forceinline__ float norm_rew(const GaeParams& p, float rew) {
    float n = rew;
    if (p.normalize) {
        n = rew * p.inv_std;
        if (p.clip) n = fminf(fmaxf(n, -p.clip_range), p.clip_range);
    }
    return n;
}

// the next value of element j of the quad (non-terminal: V[i + 1], 0 on the array's last step)
__device__ __forceinline__ float next_val(const Quad& q, int j) { return j + 1 < kFV ? q.v[j + 1] : q.vnext; }

// Inclusive suffix scan over the 64 lanes of a wave: S_l = f_l o ... o f_63.
__device__ __forceinline__ Aff wave_suffix_inclusive(Aff a, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        Aff o = shfl_down_aff(a, off);
        if (lane + off < 64) a = compose(a, o);
    }
    return a;
}

// ordered wave reduction (lane 0 receives f_0 o f_1 o ... o f_63)
__device__ __forceinline__ Aff3 wave_reduce3(Aff3 a) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        Aff3 o{__shfl_down(a.c, off, 64), __shfl_down(a.d, off, 64), __shfl_down(a.b, off, 64)};
        if ((threadIdx.x & 63) + off < 64) a = compose3(a, o);
    }
    return a;
}
__device__ __forceinline__ Aff wave_reduce(Aff a) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        Aff o = shfl_down_aff(a, off);
        if ((threadIdx.x & 63) + off < 64) a = compose(a, o);
    }
    return a;
}

// Pass 1: per tile, the composed adv map (c, d, b), the composed return map, the truncation count and the
// clip-portion partial sums (sum |r / std|, sum |clip(r / std)|).  Rounds of 2048 elements, 8 per thread (two
// float4 of each array; 4 per thread took twice the cross-lane reductions: 45.6 -> 37.8 us at 2^24).
constexpr int kSRound = kFT * 2 * kFV, kSRounds = kFTile / kSRound;
template <bool VEC>
__global__ void __launch_bounds__(kFT) k_flat_summary(GaeParams p, float4* sumA, float2* sumR, int* cnt, float2* clipp) {
    __shared__ Aff3 sa[kSRounds][kFT / 64];
    __shared__ Aff sr[kSRounds][kFT / 64];
    __shared__ float sc[3][kFT / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t t0 = (int64_t)blockIdx.x * kFTile;
    int c = 0;
    float sabs = 0.f, sclip = 0.f;
#pragma unroll
    for (int q = 0; q < kSRounds; q++) {
        const int64_t i0 = t0 + (int64_t)q * kSRound + threadIdx.x * 2 * kFV;
        Quad e2[2];
        load_octet<VEC>(p, i0, e2);
        Aff3 A{1.f, 0.f, 0.f};
        Aff R{1.f, 0.f};
#pragma unroll
        for (int h = 1; h >= 0; h--) {
            const Quad& e = e2[h];
            const int64_t j0 = i0 + h * kFV;
#pragma unroll
            for (int j = kFV - 1; j >= 0; j--) {
                const int8_t t = e.t[j];
                const float n = norm_rew(p, e.r[j]);
                if (p.normalize && j0 + j < p.M) {
                    sabs += fabsf(e.r[j] * p.inv_std);
                    sclip += fabsf(n);
                }
                const bool term = t == kNormal || t == kTruncated;
                const float nd = term ? 0.f : 1.f;
                Aff3 f;
                if (t == kTruncated) {
                    f = {0.f, n - e.v[j], p.gamma};  // (n + gamma T) - V with T symbolic
                    c += j0 + j < p.M;
                } else {
                    const float next = t == kNormal ? 0.f : next_val(e, j);
                    f = {p.gamma_lambda * nd, (n + p.gamma * next) - e.v[j], 0.f};
                }
                A = compose3(f, A);
                R = compose(Aff{p.gamma * nd, e.r[j]}, R);
            }
        }
        A = wave_reduce3(A);
        R = wave_reduce(R);
        if (lane == 0) {
            sa[q][w] = A;
            sr[q][w] = R;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        c += __shfl_down(c, o, 64);
        sabs += __shfl_down(sabs, o, 64);
        sclip += __shfl_down(sclip, o, 64);
    }
    if (lane == 0) {
        sc[0][w] = (float)c;
        sc[1][w] = sabs;
        sc[2][w] = sclip;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        Aff3 A{1.f, 0.f, 0.f};
        Aff R{1.f, 0.f};
        for (int q = kSRounds - 1; q >= 0; q--)
            for (int ww = kFT / 64 - 1; ww >= 0; ww--) {
                A = compose3(sa[q][ww], A);
                R = compose(sr[q][ww], R);
            }
        sumA[blockIdx.x] = make_float4(A.c, A.d, A.b, 0.f);
        sumR[blockIdx.x] = make_float2(R.c, R.d);
        float cs = 0.f, s1 = 0.f, s2 = 0.f;
        for (int ww = 0; ww < kFT / 64; ww++) {
            cs += sc[0][ww];
            s1 += sc[1][ww];
            s2 += sc[2][ww];
        }
        cnt[blockIdx.x] = (int)cs;
        clipp[blockIdx.x] = make_float2(s1, s2);
    }
}

struct FlatScratch {
    std::mutex mu;  // held for one call on this device (calls on other devices run concurrently)
    char* p = nullptr;
    size_t bytes = 0;
    void* host = nullptr;  // pinned, mapped: the carry pass writes the FlatResult straight to the host
};
constexpr int kMaxDevices = 64;
FlatScratch g_flat_scratch[kMaxDevices];  // rlgpu_gae_flat's tile summaries, per device

struct FlatResult {
    int64_t total;  // truncations found (GAE.cpp:196-197 checks it against the values given)
    float sabs, sclip;
};

// Pass 2 (one workgroup): base[t] = truncations before tile t (base[n] = total), carry[t] = (A, R) entering
// tile t from its right neighbour, the clip sums; all in a fixed order.
__global__ void __launch_bounds__(kCT) k_flat_carry(const float4* sumA, const float2* sumR, const int* cnt,
                                                    const float2* clipp, int n, const float* trunc_vals,
                                                    int64_t num_truncs, int64_t* base, float2* carry, FlatResult* res) {
    __shared__ int64_t s_cnt[kCT / 64];
    __shared__ Aff s_a[kCT / 64], s_r[kCT / 64];
    __shared__ float s_c[2][kCT / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int per = (n + kCT - 1) / kCT, b0 = threadIdx.x * per, b1 = min(b0 + per, n);
    // forward exclusive prefix of the counts
    int64_t mine = 0;
    float s1 = 0.f, s2 = 0.f;
    for (int b = b0; b < b1; b++) {
        mine += cnt[b];
        const float2 cp = clipp[b];
        s1 += cp.x;
        s2 += cp.y;
    }
    int64_t inc = mine;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int64_t o = __shfl_up(inc, off, 64);
        if (lane >= off) inc += o;
    }
    for (int o = 32; o > 0; o >>= 1) {
        s1 += __shfl_down(s1, o, 64);
        s2 += __shfl_down(s2, o, 64);
    }
    if (lane == 63) s_cnt[w] = inc;
    if (lane == 0) {
        s_c[0][w] = s1;
        s_c[1][w] = s2;
    }
    __syncthreads();
    int64_t run = inc - mine;
    for (int ww = 0; ww < w; ww++) run += s_cnt[ww];
    // the tiles' resolved maps, composed right to left over this thread's range
    Aff ta{1.f, 0.f}, tr{1.f, 0.f};
    {
        int64_t k = run;
        for (int b = b0; b < b1; b++) {
            base[b] = k;
            k += cnt[b];
        }
        if (b0 < n && b1 == n) {
            base[n] = k;
            float a1 = 0.f, a2 = 0.f;
            for (int ww = 0; ww < kCT / 64; ww++) {
                a1 += s_c[0][ww];
                a2 += s_c[1][ww];
            }
            res->total = k;
            res->sabs = a1;
            res->sclip = a2;
        }
    }
    auto resolved = [&](int b, int64_t kb) {
        const float4 s = sumA[b];
        const float T = (s.z != 0.f && kb < num_truncs) ? trunc_vals[kb] : 0.f;
        return Aff{s.x, s.y + s.z * T};
    };
    for (int b = b1 - 1; b >= b0; b--) {
        ta = compose(resolved(b, base[b]), ta);
        const float2 r = sumR[b];
        tr = compose(Aff{r.x, r.y}, tr);
    }
    // exclusive suffix over the threads: the composition of every range to this one's right
    Aff sa = wave_suffix_inclusive(ta, lane), sr = wave_suffix_inclusive(tr, lane);
    Aff ea = shfl_down_aff(sa, 1), er = shfl_down_aff(sr, 1);
    if (lane == 63) ea = er = Aff{1.f, 0.f};
    if (lane == 0) {
        s_a[w] = sa;
        s_r[w] = sr;
    }
    __syncthreads();
    Aff xa{1.f, 0.f}, xr{1.f, 0.f};
    for (int ww = kCT / 64 - 1; ww > w; ww--) {
        xa = compose(s_a[ww], xa);
        xr = compose(s_r[ww], xr);
    }
    ea = compose(ea, xa);
    er = compose(er, xr);
    float va = ea.d, vr = er.d;  // the value entering this range's right edge (0 past the array's end)
    for (int b = b1 - 1; b >= b0; b--) {
        carry[b] = make_float2(va, vr);
        const Aff a = resolved(b, base[b]);
        const float2 r = sumR[b];
        va = a.d + a.c * va;
        vr = r.y + r.x * vr;
    }
}

// block-wide inclusive suffix sum of an int (threads l .. kFT - 1)
__device__ __forceinline__ int block_suffix_int(int v, int* s4) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_down(v, off, 64);
        if (lane + off < 64) v += o;
    }
    if (lane == 0) s4[w] = v;
    __syncthreads();
    for (int ww = kFT / 64 - 1; ww > w; ww--) v += s4[ww];
    return v;
}

// Pass 3: per tile, rounds right to left; exact maps (the truncation values by their forward index), the
// carry composed in, A / target / R written as float4s.
template <bool VEC>
__global__ void __launch_bounds__(kFT) k_flat_apply(GaeParams p, const int64_t* base, const float2* carry, float* adv,
                                                    float* target, float* ret) {
    __shared__ int s_cnt[kFRounds][kFT / 64];
    __shared__ Aff s_a[kFRounds][kFT / 64], s_r[kFRounds][kFT / 64];
    __shared__ float2 s_x[kFRounds];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t t0 = (int64_t)blockIdx.x * kFTile;
    const int64_t knext = base[blockIdx.x + 1];  // truncations before the next tile
    float2 cin = carry[blockIdx.x];
    int after = 0;  // truncations in this tile's rounds to the right of the current one
    for (int q = kFRounds - 1; q >= 0; q--) {
        const int64_t i0 = t0 + (int64_t)q * kFRound + threadIdx.x * kFV;
        Quad e;
        load_quad<VEC>(p, i0, e);
        int c = 0;
#pragma unroll
        for (int j = 0; j < kFV; j++) c += (e.t[j] == kTruncated && i0 + j < p.M);
        const int suf = block_suffix_int(c, s_cnt[q]);  // truncations at this thread's first element or later
        int k_after = after + suf - c;  // truncations after this thread's 4 elements within the tile
        Aff fa[kFV], fr[kFV];
        float n[kFV];
#pragma unroll
        for (int j = kFV - 1; j >= 0; j--) {
            const int8_t t = e.t[j];
            n[j] = norm_rew(p, e.r[j]);
            const bool term = t == kNormal || t == kTruncated;
            const float nd = term ? 0.f : 1.f;
            float next;
            if (t == kNormal) next = 0.f;
            else if (t == kTruncated) {
                k_after += i0 + j < p.M;
                const int64_t k = knext - k_after;  // the forward index of this truncation
                next = (k >= 0 && k < p.num_truncs) ? p.trunc_vals[k] : 0.f;
            } else next = next_val(e, j);
            fa[j] = Aff{p.gamma_lambda * nd, (n[j] + p.gamma * next) - e.v[j]};
            fr[j] = Aff{p.gamma * nd, e.r[j]};
        }
        Aff ta{1.f, 0.f}, tr{1.f, 0.f};
#pragma unroll
        for (int j = kFV - 1; j >= 0; j--) {
            ta = compose(fa[j], ta);
            tr = compose(fr[j], tr);
        }
        // exclusive suffix over the block's threads, then the round's carry
        Aff sa = wave_suffix_inclusive(ta, lane), sr = wave_suffix_inclusive(tr, lane);
        Aff ea = shfl_down_aff(sa, 1), er = shfl_down_aff(sr, 1);
        if (lane == 63) ea = er = Aff{1.f, 0.f};
        if (lane == 0) {
            s_a[q][w] = sa;
            s_r[q][w] = sr;
        }
        __syncthreads();
        Aff xa{1.f, 0.f}, xr{1.f, 0.f};
        for (int ww = kFT / 64 - 1; ww > w; ww--) {
            xa = compose(s_a[q][ww], xa);
            xr = compose(s_r[q][ww], xr);
        }
        ea = compose(ea, xa);
        er = compose(er, xr);
        float va = ea.d + ea.c * cin.x, vr = er.d + er.c * cin.y;
        float oa[kFV], ot[kFV], orr[kFV];
#pragma unroll
        for (int j = kFV - 1; j >= 0; j--) {
            va = fa[j].d + fa[j].c * va;
            vr = fr[j].d + fr[j].c * vr;
            oa[j] = va;
            ot[j] = e.v[j] + va;
            orr[j] = vr;
        }
        if (VEC && i0 + kFV <= p.M) {
            *reinterpret_cast<float4*>(adv + i0) = make_float4(oa[0], oa[1], oa[2], oa[3]);
            *reinterpret_cast<float4*>(target + i0) = make_float4(ot[0], ot[1], ot[2], ot[3]);
            *reinterpret_cast<float4*>(ret + i0) = make_float4(orr[0], orr[1], orr[2], orr[3]);
        } else {
#pragma unroll
            for (int j = 0; j < kFV; j++)
                if (i0 + j < p.M) {
                    adv[i0 + j] = oa[j];
                    target[i0 + j] = ot[j];
                    ret[i0 + j] = orr[j];
                }
        }
        if (threadIdx.x == 0) s_x[q] = make_float2(va, vr);  // the value at the round's first element
        __syncthreads();
        cin = s_x[q];
        after += s_cnt[q][0] + s_cnt[q][1] + s_cnt[q][2] + s_cnt[q][3];  // the round's truncations
    }
}

// Rollout layout: one lane per agent column, exact reference order (GAE.cpp:169-193).
constexpr int kGaeU = 8;
__global__ void __launch_bounds__(256) k_gae_rollout(const float* __restrict__ rews, const int8_t* __restrict__ terms,
                                                     const float* __restrict__ vals, const float* __restrict__ trunc_vals,
                                                     const float* __restrict__ boot_vals, int T, int N, float gamma,
                                                     float gamma_lambda, float inv_std, int normalize, int clip,
                                                     float clip_range, float* __restrict__ adv,
                                                     float* __restrict__ target, float* __restrict__ ret,
                                                     float* clip_sums) {
    int n = blockIdx.x * blockDim.x + threadIdx.x;
    float sabs = 0.f, sclip = 0.f;
    if (n < N) {
        // kGaeU steps' loads are issued before their recursion (the loads do not depend on it; one
        // global-load latency per kGaeU steps instead of per step); V[t + 1] is the previous step's V
        float prevLambda = 0.f, prevRet = 0.f;
        float vnext = boot_vals ? boot_vals[n] : 0.f;  // the value after the last step
        for (int t1 = T - 1; t1 >= 0; t1 -= kGaeU) {
            float rr[kGaeU], vv[kGaeU];
            int8_t tt[kGaeU];
#pragma unroll
            for (int u = 0; u < kGaeU; u++) {
                const int64_t i = (int64_t)max(t1 - u, 0) * N + n;
                rr[u] = rews[i];
                vv[u] = vals[i];
                tt[u] = terms[i];
            }
#pragma unroll
            for (int u = 0; u < kGaeU; u++) {
                const int t = t1 - u;
                if (t < 0) break;
                const int64_t i = (int64_t)t * N + n;
                const int8_t term = tt[u];
                const float rew = rr[u];
                float cur = rew;
                if (normalize) {
                    cur = rew * inv_std;
                    sabs += fabsf(cur);
                    if (clip) cur = fminf(fmaxf(cur, -clip_range), clip_range);
                    sclip += fabsf(cur);
                }
                float done = (term == kNormal) ? 1.f : 0.f;
                float trunc = (term == kTruncated) ? 1.f : 0.f;
                float nd = (1.f - done) * (1.f - trunc);
                float nextVal;
                if (term == kNormal) nextVal = 0.f;
                else if (term == kTruncated) nextVal = trunc_vals ? trunc_vals[i] : 0.f;
                else nextVal = vnext;  // V[t + 1], or the bootstrap value at t = T - 1
                float v = vv[u];
                float predReturn = cur + gamma * nextVal;
                float delta = predReturn - v;
                float curReturn = rew + prevRet * gamma * nd;
                ret[i] = curReturn;
                prevLambda = delta + gamma_lambda * nd * prevLambda;
                adv[i] = prevLambda;
                target[i] = v + prevLambda;
                prevRet = curReturn;
                vnext = v;
            }
        }
    }
    if (clip_sums && normalize) {
        for (int off = 32; off > 0; off >>= 1) {
            sabs += __shfl_down(sabs, off, 64);
            sclip += __shfl_down(sclip, off, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&clip_sums[0], sabs);
            atomicAdd(&clip_sums[1], sclip);
        }
    }
}

// One lane per complete trajectory of a flat batch (rlgpu_gae_segments): the same recursion as
// k_gae_rollout over rows off + len - 1 .. off, the segment's terminal bootstrapped from trunc_vals[tidx]
// (code 2) or 0 (code 1), prevLambda / prevRet starting at 0.
__global__ void __launch_bounds__(256) k_gae_segments(const float* __restrict__ rews, const int8_t* __restrict__ terms,
                                                      const float* __restrict__ vals, const float* __restrict__ trunc_vals,
                                                      const int64_t* __restrict__ seg_off, const int32_t* __restrict__ seg_len,
                                                      const int32_t* __restrict__ seg_tidx, int64_t K, float gamma,
                                                      float gamma_lambda, float inv_std, int normalize, int clip,
                                                      float clip_range, float* __restrict__ adv, float* __restrict__ target,
                                                      float* __restrict__ ret, float* clip_sums) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    float sabs = 0.f, sclip = 0.f;
    if (k < K) {
        const int64_t off = seg_off[k];
        const int L = seg_len[k], tidx = seg_tidx[k];
        float prevLambda = 0.f, prevRet = 0.f;
        for (int j = L - 1; j >= 0; --j) {
            const int64_t i = off + j;
            const int8_t term = terms[i];
            const float rew = rews[i];
            float cur = rew;
            if (normalize) {
                cur = rew * inv_std;
                sabs += fabsf(cur);
                if (clip) cur = fminf(fmaxf(cur, -clip_range), clip_range);
                sclip += fabsf(cur);
            }
            const float done = (term == kNormal) ? 1.f : 0.f;
            const float trunc = (term == kTruncated) ? 1.f : 0.f;
            const float nd = (1.f - done) * (1.f - trunc);
            float nextVal;
            if (term == kNormal) nextVal = 0.f;
            else if (term == kTruncated) nextVal = (trunc_vals && tidx >= 0) ? trunc_vals[tidx] : 0.f;
            else nextVal = vals[i + 1];  // a segment's non-final rows are never its last row
            const float v = vals[i];
            const float predReturn = cur + gamma * nextVal;
            const float delta = predReturn - v;
            const float curReturn = rew + prevRet * gamma * nd;
            ret[i] = curReturn;
            prevLambda = delta + gamma_lambda * nd * prevLambda;
            adv[i] = prevLambda;
            target[i] = v + prevLambda;
            prevRet = curReturn;
        }
    }
    if (clip_sums && normalize) {
        for (int o = 32; o > 0; o >>= 1) {
            sabs += __shfl_down(sabs, o, 64);
            sclip += __shfl_down(sclip, o, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&clip_sums[0], sabs);
            atomicAdd(&clip_sums[1], sclip);
        }
    }
}

}  // namespace

extern "C" int rlgpu_gae_segments(const float* d_rews, const int8_t* d_terms, const float* d_vals, const float* d_trunc_vals,
                                  const int64_t* d_seg_off, const int32_t* d_seg_len, const int32_t* d_seg_tidx,
                                  int64_t num_segments, float gamma, float lambda, float return_std, float clip_range,
                                  float* d_adv, float* d_target, float* d_ret, float* d_clip_partials, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(num_segments >= 0, "rlgpu_gae_segments: negative segment count");
        if (num_segments == 0) return;
        RLGPU_REQUIRE(d_rews && d_terms && d_vals && d_seg_off && d_seg_len && d_seg_tidx && d_adv && d_target && d_ret,
                      "rlgpu_gae_segments: null argument");
        hipStream_t s = rlgpu::as_stream(stream);
        const bool normalize = (return_std != 0.f && return_std != 1.f);  // GAE.cpp:47-49
        const float inv_std = normalize ? 1.f / return_std : 1.f;
        hipLaunchKernelGGL(k_gae_segments, dim3(rlgpu::ceil_div(num_segments, 256)), dim3(256), 0, s, d_rews, d_terms, d_vals,
                           d_trunc_vals, d_seg_off, d_seg_len, d_seg_tidx, num_segments, gamma, gamma * lambda, inv_std,
                           (int)normalize, (int)(clip_range > 0.f), clip_range, d_adv, d_target, d_ret, d_clip_partials);
        RLGPU_CHECK_HIP(hipGetLastError());
    });
}

extern "C" int rlgpu_gae_flat(const float* d_rews, const int8_t* d_terms, const float* d_vals,
                              const float* d_trunc_vals, int64_t num_returns, int64_t num_truncs, float gamma,
                              float lambda, float return_std, float clip_range, float* d_adv, float* d_target,
                              float* d_ret, float* h_clip_portion, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(num_returns >= 0 && num_truncs >= 0, "rlgpu_gae_flat: negative size");
        if (num_returns == 0) {  // GAE.cpp:16-23
            if (h_clip_portion) *h_clip_portion = 0.f;
            return;
        }
        RLGPU_REQUIRE(d_rews && d_terms && d_vals && d_adv && d_target && d_ret, "rlgpu_gae_flat: null pointer");
        RLGPU_REQUIRE(num_truncs == 0 || d_trunc_vals, "rlgpu_gae_flat: trunc values missing");
        hipStream_t s = rlgpu::as_stream(stream);
        const int n = (int)rlgpu::ceil_div(num_returns, kFTile);
        // scratch: tile maps (f4, f2) | counts (i32) | clip partials (f2) | bases (i64, n + 1) | carries (f2) | result
        size_t bytes = 0;
        auto take = [&](size_t sz) {
            bytes = (bytes + 15) / 16 * 16;
            const size_t off = bytes;
            bytes += sz;
            return off;
        };
        const size_t o_a = take(sizeof(float4) * n), o_r = take(sizeof(float2) * n), o_c = take(sizeof(int) * n),
                     o_p = take(sizeof(float2) * n), o_b = take(sizeof(int64_t) * (n + 1)),
                     o_x = take(sizeof(float2) * n), o_res = take(sizeof(FlatResult));
        // one scratch buffer per device, grown on demand and held for the call (the call ends synchronised)
        int dev = 0;
        RLGPU_CHECK_HIP(hipGetDevice(&dev));
        RLGPU_REQUIRE(dev >= 0 && dev < kMaxDevices, "rlgpu_gae_flat: device index beyond the scratch table");
        FlatScratch& sc = g_flat_scratch[dev];
        std::lock_guard<std::mutex> lock(sc.mu);
        if (sc.bytes < bytes) {
            if (sc.p) RLGPU_CHECK_HIP(hipFree(sc.p));
            sc.p = nullptr;
            sc.bytes = 0;
            RLGPU_CHECK_HIP(hipMalloc((void**)&sc.p, bytes));
            sc.bytes = bytes;
        }
        char* scratch = sc.p;
        float4* sumA = (float4*)(scratch + o_a);
        float2* sumR = (float2*)(scratch + o_r);
        int* cnt = (int*)(scratch + o_c);
        float2* clipp = (float2*)(scratch + o_p);
        int64_t* base = (int64_t*)(scratch + o_b);
        float2* carry = (float2*)(scratch + o_x);
        if (!sc.host) RLGPU_CHECK_HIP(hipHostMalloc(&sc.host, sizeof(FlatResult), hipHostMallocMapped));
        FlatResult* res = nullptr;
        RLGPU_CHECK_HIP(hipHostGetDevicePointer((void**)&res, sc.host, 0));
        (void)o_res;

        GaeParams p;
        p.rews = d_rews;
        p.terms = d_terms;
        p.vals = d_vals;
        p.trunc_vals = d_trunc_vals;
        p.M = num_returns;
        p.num_truncs = num_truncs;
        p.normalize = (return_std != 0.f && return_std != 1.f);  // GAE.cpp:73
        p.clip = clip_range > 0.f;                                  // GAE.cpp:74
        p.inv_std = p.normalize ? (1.0f / return_std) : 1.0f;
        p.gamma = gamma;
        p.gamma_lambda = gamma * lambda;
        p.clip_range = clip_range;

        // float4 / 4-byte accesses when every array is aligned for them (torch allocations are)
        auto al = [](const void* q, uintptr_t a) { return ((uintptr_t)q % a) == 0; };
        const bool vec = al(d_rews, 16) && al(d_vals, 16) && al(d_terms, 4) && al(d_adv, 16) && al(d_target, 16) &&
                         al(d_ret, 16);
        if (vec) hipLaunchKernelGGL(k_flat_summary<true>, dim3(n), dim3(kFT), 0, s, p, sumA, sumR, cnt, clipp);
        else hipLaunchKernelGGL(k_flat_summary<false>, dim3(n), dim3(kFT), 0, s, p, sumA, sumR, cnt, clipp);
        hipLaunchKernelGGL(k_flat_carry, dim3(1), dim3(kCT), 0, s, sumA, sumR, cnt, clipp, n, d_trunc_vals, num_truncs, base,
                           carry, res);
        if (vec) hipLaunchKernelGGL(k_flat_apply<true>, dim3(n), dim3(kFT), 0, s, p, base, carry, d_adv, d_target, d_ret);
        else hipLaunchKernelGGL(k_flat_apply<false>, dim3(n), dim3(kFT), 0, s, p, base, carry, d_adv, d_target, d_ret);
        RLGPU_CHECK_HIP(hipGetLastError());
        RLGPU_CHECK_HIP(hipStreamSynchronize(s));
        const volatile FlatResult* hv = reinterpret_cast<volatile FlatResult*>(sc.host);
        FlatResult h;
        h.total = hv->total;
        h.sabs = hv->sabs;
        h.sclip = hv->sclip;
        const int64_t h_total = h.total;
        const float h_clip[2] = {h.sabs, h.sclip};
        // GAE.cpp:196-197: truncation count must match the provided bootstrap values.
        if (num_truncs > 0 && h_total != num_truncs)
            throw rlgpu::Error(RLGPU_ERR_INVALID_ARG, "GAE: truncation count mismatch (" + std::to_string(h_total) +
                                                          "/" + std::to_string(num_truncs) + ")");
        if (h_clip_portion)
            *h_clip_portion = p.normalize ? (h_clip[0] - h_clip[1]) / fmaxf(h_clip[0], 1e-7f) : 0.f;
    });
}

extern "C" int rlgpu_gae_rollout(const float* d_rews, const int8_t* d_terms, const float* d_vals,
                                 const float* d_trunc_vals, const float* d_boot_vals, int32_t T, int32_t N,
                                 float gamma, float lambda, float return_std, float clip_range, float* d_adv,
                                 float* d_target, float* d_ret, float* d_clip_partials, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(T >= 0 && N >= 0, "rlgpu_gae_rollout: negative size");
        if (T == 0 || N == 0) return;
        RLGPU_REQUIRE(d_rews && d_terms && d_vals && d_adv && d_target && d_ret, "rlgpu_gae_rollout: null pointer");
        hipStream_t s = rlgpu::as_stream(stream);
        bool normalize = (return_std != 0.f && return_std != 1.f);
        float inv_std = normalize ? (1.0f / return_std) : 1.0f;
        hipLaunchKernelGGL(k_gae_rollout, dim3(rlgpu::ceil_div(N, 256)), dim3(256), 0, s, d_rews, d_terms, d_vals,
                           d_trunc_vals, d_boot_vals, T, N, gamma, gamma * lambda, inv_std, (int)normalize,
                           (int)(clip_range > 0.f), clip_range, d_adv, d_target, d_ret, d_clip_partials);
        RLGPU_CHECK_HIP(hipGetLastError());
    });
}
