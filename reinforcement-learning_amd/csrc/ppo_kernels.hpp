// ppo_kernels.hpp -- policy head, PPO losses and optimizer kernels (gfx950, one wave per row).
// Semantics follow GigaLearnCPP PPOLearner.cpp (InferPolicyProbsFromModels :78-112,
// InferActionsFromModels :114-184, Learn :278-581) with the libtorch op semantics spelled out
// where they matter (clamp / min tie gradients, softmax backward, AdamW, clip_grad_norm_).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rlgpu_detmath.h"
#include "mlp_kernels.hpp"

namespace ppo {

using mlp::bf2f;
using mlp::wave_max;
using mlp::wave_sum;

constexpr float kMinProb = 1e-11f;        // ACTION_MIN_PROB
constexpr float kDisabledLogit = -1e10f;  // ACTION_DISABLED_LOGIT
constexpr int kMaxA = 128;                // actions per row: 2 per lane

// The sampler's Philox key for a draw step: the seed, with the step's high 32 bits folded in (the counter carries its
// low 32), so streams on separate step ranges -- the skill matches' 2^40 + k (rlgpu/skill.py) against the rollout's
// k -- never share uniforms; steps below 2^32 keep key = seed.
__host__ __device__ __forceinline__ uint64_t sample_key(uint64_t seed, uint64_t step) {
    return seed ^ ((step >> 32) * 0x9E3779B97F4A7C15ull);
}

__device__ __forceinline__ uint32_t philox(uint64_t key, uint32_t c0, uint32_t c1) {
    uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
    uint32_t x0 = c0, x1 = c1, x2 = 0x2545F491u, x3 = 0x4F6CDD1Du;
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * x0, p1 = (uint64_t)0xCD9E8D57u * x2;
        uint32_t y0 = (uint32_t)(p1 >> 32) ^ x1 ^ k0, y1 = (uint32_t)p1, y2 = (uint32_t)(p0 >> 32) ^ x3 ^ k1,
                 y3 = (uint32_t)p0;
        x0 = y0;
        x1 = y1;
        x2 = y2;
        x3 = y3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return x0;
}

// masked softmax of one row held 2 per lane (actions 2l, 2l+1); returns probs (unclamped)
__device__ __forceinline__ void masked_softmax(float z0, float z1, bool v0, bool v1, float& p0, float& p1) {
    float m = wave_max(fmaxf(v0 ? z0 : -INFINITY, v1 ? z1 : -INFINITY));
    float e0 = v0 ? __expf(z0 - m) : 0.f, e1 = v1 ? __expf(z1 - m) : 0.f;
    float s = wave_sum(e0 + e1);
    p0 = e0 / s;
    p1 = e1 / s;
}

// InferActions: logits bf16 [n, A] -> action (int32), log prob (PPOLearner.cpp:78-184).  The probs are the
// masked softmax clamped to [1e-11, 1]; deterministic: argmax (lowest index on ties); otherwise the
// reference's CPU sampler (PPOLearner.cpp:157-178): r uniform in [0, 1), the first action whose running sum
// of the clamped probs, accumulated in column order, reaches r (r <= running), the last column when none
// does, and log(max(1e-12, p)) of the pick.  The uniform is a Philox draw of (seed, row0 + row, step) --
// global row numbers, so chunked launches draw the same uniforms as one launch -- where the reference uses
// an unseeded thread-local mt19937.
// Bit-exact against the CPU oracle (oracle/sampler_ref.c): IEEE + - * / only, exp / log by the shared
// rs_expf / rs_logf (include/rlgpu_detmath.h), no FMA contraction, max / sum by xor butterflies (= pairwise
// trees), and the running sum sequential: one lane per row walks the row's probs staged in LDS.
// row_sel (optional): only rows with (row_sel[row] != 0) == sel are written (mixed-policy inference).
// RG rows, one wave, interleaved (each cross-lane step issues for all RG rows before the next, so
// one wave hides the shuffle latency of RG independent rows): lg[g] = row g's A logits (global or
// LDS), mk[g] its masks, pr[g] A floats of LDS scratch for its probs; writes act[row[g]], logp[row[g]]
// where ok[g].  sample_actions runs it with RG = 1; the fused inference kernel (infer_kernels.hpp) runs
// sample_rows_looped (below) over 8 rows -- the per-row arithmetic is the same, so both draw the same actions
// from the same logits.
// a logit as the sampler reads it: 16-bit storage (bf16 / fp16), or fp32 (useHalfPrecision = false)
template <bool F16>
__device__ __forceinline__ float logit_f(uint16_t u) { return mlp::h2f<F16>(u); }
template <bool F16>
__device__ __forceinline__ float logit_f(float x) { return x; }

template <int RG, bool F16, typename LT = uint16_t>
__device__ __forceinline__ void sample_rows(const LT* const (&lg)[RG], const uint8_t* const (&mk)[RG],
                                            float* const (&pr)[RG], int A, int deterministic, uint64_t seed,
                                            uint64_t step, int64_t row0, const int (&row)[RG], const bool (&ok)[RG],
                                            int lane, int32_t* act, float* logp) {
#pragma clang fp contract(off)
    const int a0 = 2 * lane, a1 = 2 * lane + 1;
    const bool in0 = a0 < A, in1 = a1 < A;
    float z0[RG], z1[RG], m[RG], s[RG], p0[RG], p1[RG];
    int pick[RG];
    const int c0 = min(a0, A - 1), c1 = min(a1, A - 1);  // loads stay unconditional (no branches between them)
#pragma unroll
    for (int g = 0; g < RG; g++) {
        const float l0 = logit_f<F16>(lg[g][c0]), l1 = logit_f<F16>(lg[g][c1]);
        const uint8_t m0 = mk[g][c0], m1 = mk[g][c1];
        z0[g] = in0 ? l0 + (m0 ? 0.f : kDisabledLogit) : 0.f;
        z1[g] = in1 ? l1 + (m1 ? 0.f : kDisabledLogit) : 0.f;
        // softmax over all A columns (masked ones carry -1e10, exactly as the reference)
        m[g] = fmaxf(in0 ? z0[g] : -INFINITY, in1 ? z1[g] : -INFINITY);
    }
#pragma unroll
    for (int g = 0; g < RG; g++) m[g] = mlp::wave_max_x(m[g]);
#pragma unroll
    for (int g = 0; g < RG; g++) {
        z0[g] = in0 ? rs_expf(z0[g] - m[g]) : 0.f;  // e0, e1
        z1[g] = in1 ? rs_expf(z1[g] - m[g]) : 0.f;
        s[g] = z0[g] + z1[g];
    }
#pragma unroll
    for (int g = 0; g < RG; g++) s[g] = mlp::wave_sum_x(s[g]);
#pragma unroll
    for (int g = 0; g < RG; g++) {
        p0[g] = in0 ? fminf(fmaxf(z0[g] / s[g], kMinProb), 1.f) : 0.f;
        p1[g] = in1 ? fminf(fmaxf(z1[g] / s[g], kMinProb), 1.f) : 0.f;
    }
    if (deterministic) {
        float best[RG];
        int bi[RG];
#pragma unroll
        for (int g = 0; g < RG; g++) {
            best[g] = fmaxf(p0[g], p1[g]);
            bi[g] = p0[g] >= p1[g] ? a0 : a1;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
#pragma unroll
            for (int g = 0; g < RG; g++) {
                float ob = __shfl_xor(best[g], o, 64);
                int oi = __shfl_xor(bi[g], o, 64);
                const bool take = ob > best[g] || (ob == best[g] && oi < bi[g]);
                best[g] = take ? ob : best[g];
                bi[g] = take ? oi : bi[g];
            }
#pragma unroll
        for (int g = 0; g < RG; g++) pick[g] = bi[g];
    } else {
        // the probs into LDS (lane l holds actions 2l, 2l + 1), then lane g < RG walks row g
#pragma unroll
        for (int g = 0; g < RG; g++) {
            if (in0) pr[g][a0] = p0[g];
            if (in1) pr[g][a1] = p1[g];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        int mine = A - 1;  // picked = cols - 1 when no running sum reaches r
        if (lane < RG) {
            const float* p = pr[0];
            int rw = row[0];
#pragma unroll
            for (int g = 1; g < RG; g++)
                if (lane == g) {
                    p = pr[g];
                    rw = row[g];
                }
            const float r = (float)(philox(sample_key(seed, step), (uint32_t)(row0 + rw), (uint32_t)step) >> 8) *
                            (1.f / 16777216.f);
            // the sequential running sum, 8 probs' LDS loads issued ahead of their adds (the loads do not depend
            // on the sum; one LDS round trip per 8 columns instead of per column)
            float running = 0.f;
            bool found = false;
            int j = 0;
            for (; j + 8 <= A; j += 8) {
                float q[8];
#pragma unroll
                for (int k = 0; k < 8; k++) q[k] = p[j + k];
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    running += q[k];
                    const bool hit = !found && r <= running;
                    mine = hit ? j + k : mine;
                    found = found || hit;
                }
            }
            for (; j < A; j++) {
                running += p[j];
                const bool hit = !found && r <= running;
                mine = hit ? j : mine;
                found = found || hit;
            }
        }
#pragma unroll
        for (int g = 0; g < RG; g++) pick[g] = __shfl(mine, g, 64);
    }
#pragma unroll
    for (int g = 0; g < RG; g++) {
        float pp0 = __shfl(p0[g], pick[g] >> 1, 64), pp1 = __shfl(p1[g], pick[g] >> 1, 64);
        if (lane == 0 && ok[g]) {
            act[row[g]] = pick[g];
            const float pp = (pick[g] & 1) ? pp1 : pp0;
            if (logp) logp[row[g]] = rs_logf(1e-12f < pp ? pp : 1e-12f);  // log(std::max(1e-12f, p))
        }
    }
}
// sample_rows with the softmax and the writes in a loop over the RG rows instead of unrolled, for the fused
// inference kernel: the unrolled form is ~1,900 instructions that each call executes once, so instruction
// fetch, not arithmetic, set its time (its phase trace: 17 us from the staged logits to the probs).  Same
// per-row operations in the same order (the probs go to LDS in both modes and the pick's prob is read back
// from there: the same float), so the same actions and log probs; the running-sum walk keeps one lane per row,
// all RG rows at once.  rowfn(g, lg, mk, pr, row, ok) gives row g's logits, masks, LDS probs, row and write flag;
// mark(k) optional phase timestamps (the fused kernel's trace): 0 = probs in LDS, 1 = picks known.
struct NoMark {
    __device__ void operator()(int) const {}
};
template <int RG, bool F16, typename RowFn, typename Mark = NoMark>
__device__ __forceinline__ void sample_rows_looped(RowFn rowfn, int A, int deterministic, uint64_t seed, uint64_t step,
                                                   int64_t row0, int lane, int32_t* act, float* logp,
                                                   Mark mark = Mark{}) {
#pragma clang fp contract(off)
    const int a0 = 2 * lane, a1 = 2 * lane + 1;
    const bool in0 = a0 < A, in1 = a1 < A;
    const int c0 = min(a0, A - 1), c1 = min(a1, A - 1);
    int mine = A - 1;  // lane g < RG: row g's pick (deterministic: its argmax)
#pragma unroll 1
    for (int g = 0; g < RG; g++) {
        const uint16_t* lg;
        const uint8_t* mk;
        float* pr;
        int rw;
        bool ok;
        rowfn(g, lg, mk, pr, rw, ok);
        const float l0 = mlp::h2f<F16>(lg[c0]), l1 = mlp::h2f<F16>(lg[c1]);
        const uint8_t m0 = mk[c0], m1 = mk[c1];
        float z0 = in0 ? l0 + (m0 ? 0.f : kDisabledLogit) : 0.f;
        float z1 = in1 ? l1 + (m1 ? 0.f : kDisabledLogit) : 0.f;
        const float m = mlp::wave_max_x(fmaxf(in0 ? z0 : -INFINITY, in1 ? z1 : -INFINITY));
        z0 = in0 ? rs_expf(z0 - m) : 0.f;
        z1 = in1 ? rs_expf(z1 - m) : 0.f;
        const float s = mlp::wave_sum_x(z0 + z1);
        const float p0 = in0 ? fminf(fmaxf(z0 / s, kMinProb), 1.f) : 0.f;
        const float p1 = in1 ? fminf(fmaxf(z1 / s, kMinProb), 1.f) : 0.f;
        if (deterministic) {
            float best = fmaxf(p0, p1);
            int bi = p0 >= p1 ? a0 : a1;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const float ob = __shfl_xor(best, o, 64);
                const int oi = __shfl_xor(bi, o, 64);
                const bool take = ob > best || (ob == best && oi < bi);
                best = take ? ob : best;
                bi = take ? oi : bi;
            }
            mine = lane == g ? bi : mine;
        }
        if (in0) pr[a0] = p0;
        if (in1) pr[a1] = p1;
    }
    mark(0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (!deterministic && lane < RG) {
        const uint16_t* lg;
        const uint8_t* mk;
        float* p;
        int rw;
        bool ok;
        rowfn(lane, lg, mk, p, rw, ok);
        const float r = (float)(philox(sample_key(seed, step), (uint32_t)(row0 + rw), (uint32_t)step) >> 8) *
                        (1.f / 16777216.f);
        float running = 0.f;
        bool found = false;
        int j = 0;
        for (; j + 8 <= A; j += 8) {
            float q[8];
#pragma unroll
            for (int k = 0; k < 8; k++) q[k] = p[j + k];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                running += q[k];
                const bool hit = !found && r <= running;
                mine = hit ? j + k : mine;
                found = found || hit;
            }
        }
        for (; j < A; j++) {
            running += p[j];
            const bool hit = !found && r <= running;
            mine = hit ? j : mine;
            found = found || hit;
        }
    }
    mark(1);
#pragma unroll 1
    for (int g = 0; g < RG; g++) {
        const int pk = __shfl(mine, g, 64);
        const uint16_t* lg;
        const uint8_t* mk;
        float* pr;
        int rw;
        bool ok;
        rowfn(g, lg, mk, pr, rw, ok);
        if (lane == 0 && ok) {
            act[rw] = pk;
            const float pp = pr[pk];
            if (logp) logp[rw] = rs_logf(1e-12f < pp ? pp : 1e-12f);  // log(std::max(1e-12f, p))
        }
    }
}

template <bool F16, typename LT = uint16_t>
__global__ void __launch_bounds__(256) sample_actions(const LT* logits, const uint8_t* masks, int n, int A,
                                                     int deterministic, uint64_t seed, uint64_t step, int64_t row0,
                                                     int32_t* act, float* logp, const uint8_t* row_sel = nullptr,
                                                     int sel = 0) {
    __shared__ float probs[4][kMaxA];  // one row of probs per wave (sample_rows' running sum)
    int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= n) return;
    if (row_sel && ((row_sel[row] != 0) != (sel != 0))) return;
    const LT* const lg[1] = {logits + (int64_t)row * A};
    const uint8_t* const mk[1] = {masks + (int64_t)row * A};
    float* const pr[1] = {probs[threadIdx.x >> 6]};
    const int rw[1] = {row};
    const bool ok[1] = {true};
    sample_rows<1, F16, LT>(lg, mk, pr, A, deterministic, seed, step, row0, rw, ok, lane, act, logp);
}

// PPO policy loss + entropy and its gradient w.r.t. the fp32 training logits.
// Rows are minibatch-ordered; sample s = idx ? idx[start + r] : start + r addresses the
// batch buffers.  Metrics are reduced per block (one atomic each).
// 16 lanes per row, 4 rows in parallel per wave (lane group q = lane / 16 owns row q of the pass),
// each lane holding the PL_K actions i, i + 16, .., i + 16 (PL_K - 1) of its row: the row's
// reductions take 4 shuffle steps and one instruction stream serves 4 rows.
constexpr int PL_K = (kMaxA + 15) / 16;  // actions per lane (A <= 128)
constexpr int PL_PASSES = 2;             // passes of 4 rows per wave
constexpr int PL_ROWS = 4 * 4 * PL_PASSES;  // rows per 256-thread block
__device__ __forceinline__ float grp_sum(float v) {
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float grp_max(float v) {
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
template <int K>
__global__ void __launch_bounds__(256) policy_loss(const float* logits, const uint8_t* masks, const int32_t* actions,
                                                  const float* old_logp, const float* adv, const int32_t* idx, int64_t start,
                                                  int n, int A, const float* adv_stats, float bsr, float clip_range,
                                                  float ent_scale, float inv_log_a, float* dlogits, int ldd,
                                                  float* metrics, float* bias_part, float* amax) {
    __shared__ float red[16][5];
    __shared__ float colred[16][16 * K];  // per (wave, lane group) column sums of dlogits
    uint32_t vmax = 0;  // max |dlogits| (H3 operand scale, when amax is given)
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, grp = lane >> 4, i = lane & 15;
    const float mean = adv_stats[0], sd = adv_stats[1];
    float m_ent = 0.f, m_kl = 0.f, m_pl = 0.f, m_ratio = 0.f, m_clip = 0.f;
    float col[K];
#pragma unroll
    for (int k = 0; k < K; k++) col[k] = 0.f;
    const float g_pl = -bsr / (float)n;
    const float g_ent = -ent_scale * bsr * inv_log_a / (float)n;  // d loss / d H_i (H_i unnormalised)
#pragma unroll
    for (int pass = 0; pass < PL_PASSES; pass++) {
        const int row = blockIdx.x * PL_ROWS + (w * PL_PASSES + pass) * 4 + grp;
        const bool valid = row < n;
        const int rowc = valid ? row : n - 1;
        const int64_t sidx = idx ? (int64_t)idx[start + rowc] : start + rowc;
        const float* lg = logits + (int64_t)rowc * A;
        const uint8_t* mk = masks + sidx * A;
        float z[K];
        bool in[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const int a = i + 16 * k;
            in[k] = a < A;
            z[k] = in[k] ? lg[a] + (mk[a] ? 0.f : kDisabledLogit) : -INFINITY;
        }
        const int a_raw = actions[sidx];
        const float old = old_logp[sidx], advr = adv[sidx];
        float m = z[0];
#pragma unroll
        for (int k = 1; k < K; k++) m = fmaxf(m, z[k]);
        m = grp_max(m);
        float e[K], esum = 0.f;
#pragma unroll
        for (int k = 0; k < K; k++) {
            e[k] = in[k] ? expf(z[k] - m) : 0.f;
            esum += e[k];
        }
        const float sum = grp_sum(esum);
        float p[K], c[K], lgc[K], ent_l = 0.f;
#pragma unroll
        for (int k = 0; k < K; k++) {
            p[k] = e[k] / sum;
            c[k] = fminf(fmaxf(p[k], kMinProb), 1.f);
            lgc[k] = in[k] ? logf(c[k]) : 0.f;
            ent_l += in[k] ? lgc[k] * c[k] : 0.f;
        }
        const float ent = -grp_sum(ent_l);
        const int a = a_raw < 0 ? 0 : (a_raw > A - 1 ? A - 1 : a_raw);
        // the action's clamped probability: lane a % 16 of the group holds it in slot a / 16
        float mine = 0.f;
#pragma unroll
        for (int k = 0; k < K; k++)
            if (a == i + 16 * k) mine = c[k];
        const float pa = __shfl(mine, (lane & ~15) | (a & 15), 64);
        const float lp = logf(pa);
        const float ratio = expf(lp - old);
        const float advn = (advr - mean) / (sd + 1e-8f);
        const float clipped = fminf(fmaxf(ratio, 1.f - clip_range), 1.f + clip_range);
        const float s1 = ratio * advn, s2 = clipped * advn;
        const float pl = fminf(s1, s2);
        // ---- backward (torch semantics: min() ties split the gradient, clamp passes inside [lo, hi])
        const float g_s1 = s1 < s2 ? g_pl : (s1 == s2 ? g_pl * 0.5f : 0.f);
        const float g_s2 = s2 < s1 ? g_pl : (s1 == s2 ? g_pl * 0.5f : 0.f);
        const float in_rng = (ratio >= 1.f - clip_range && ratio <= 1.f + clip_range) ? 1.f : 0.f;
        const float g_ratio = g_s1 * advn + g_s2 * advn * in_rng;
        const float g_lp = g_ratio * ratio;
        float d[K], dot_l = 0.f;
#pragma unroll
        for (int k = 0; k < K; k++) {
            d[k] = in[k] ? -g_ent * (lgc[k] + 1.f) : 0.f;
            if (a == i + 16 * k) d[k] += g_lp / c[k];
            d[k] = (p[k] >= kMinProb && p[k] <= 1.f) ? d[k] : 0.f;
            dot_l += in[k] ? d[k] * p[k] : 0.f;
        }
        const float dot = grp_sum(dot_l);
        if (valid) {
            // dlogits rows of ldd >= A floats: the columns [A, ldd) are written as zeros, so the
            // output layer's GEMMs read 16-byte vectors across the row end
            float* dl = dlogits + (int64_t)row * ldd;
#pragma unroll
            for (int k = 0; k < K; k++) {
                if (!in[k]) {
                    if (i + 16 * k < ldd) dl[i + 16 * k] = 0.f;
                    continue;
                }
                const float gk = p[k] * (d[k] - dot);
                dl[i + 16 * k] = gk;
                col[k] += gk;
                const uint32_t b = mlp::abs_bits(gk);
                vmax = b > vmax ? b : vmax;
            }
            const float lr = lp - old;
            m_ent += ent * inv_log_a;
            m_kl += expf(lr) - 1.f - lr;
            m_pl += -pl;
            m_ratio += ratio;
            m_clip += fabsf(ratio - 1.f) > clip_range ? 1.f : 0.f;
        }
    }
    const int slot = w * 4 + grp;
#pragma unroll
    for (int k = 0; k < K; k++) colred[slot][i + 16 * k] = col[k];
    if (i == 0) {
        red[slot][0] = m_ent;
        red[slot][1] = m_kl;
        red[slot][2] = m_pl;
        red[slot][3] = m_ratio;
        red[slot][4] = m_clip;
    }
    __syncthreads();
    if (bias_part)  // output-bias gradient partials of this block's rows: part[blk][A]
        for (int c2 = threadIdx.x; c2 < A; c2 += 256) {
            float t = 0.f;
            for (int q = 0; q < 16; q++) t += colred[q][c2];
            bias_part[(int64_t)blockIdx.x * A + c2] = t;
        }
    if (threadIdx.x < 5 && metrics) {
        const int mslot[5] = {0, 1, 2, 4, 5};  // entropy, KL, policy loss, ratio, clip fraction
        float v = 0.f;
        for (int q = 0; q < 16; q++) v += red[q][threadIdx.x];
        atomicAdd(&metrics[mslot[threadIdx.x]], v / (float)n);
    }
    if (amax) mlp::h3_amax_commit(amax, vmax);
}

// the instantiation with ceil(A / 16) actions per lane (A = 90: 6 of the 8 slots PL_K allows)
inline decltype(&policy_loss<PL_K>) policy_loss_any(int A) {
    switch ((A + 15) / 16) {
        case 1: return &policy_loss<1>;
        case 2: return &policy_loss<2>;
        case 3: return &policy_loss<3>;
        case 4: return &policy_loss<4>;
        case 5: return &policy_loss<5>;
        case 6: return &policy_loss<6>;
        case 7: return &policy_loss<7>;
        default: return &policy_loss<PL_K>;
    }
}

// Critic MSE: loss = mean((v - t)^2) * bsr ; dv = 2 (v - t) / n * bsr.
__global__ void critic_loss(const float* vals, const float* target, const int32_t* idx, int64_t start, int n, float bsr,
                            float* dvals, float* metrics) {
    int r = blockIdx.x * blockDim.x + threadIdx.x;
    float contrib = 0.f;
    if (r < n) {
        int64_t s = idx ? (int64_t)idx[start + r] : start + r;
        float d = vals[r] - target[s];
        dvals[r] = 2.f * d / (float)n * bsr;
        contrib = d * d / (float)n * bsr;
    }
    contrib = wave_sum(contrib);
    if ((threadIdx.x & 63) == 0 && metrics) atomicAdd(&metrics[3], contrib);
}

// out = a + b over n floats (the shared head's output gradient: policy + critic input gradients),
// 4 per thread where the three spans are 16-byte aligned
__global__ void add2(const float* a, const float* b, float* out, int64_t n) {
    const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (e >= n) return;
    const bool vec = e + 4 <= n && ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) |
                                     reinterpret_cast<uintptr_t>(out)) & 15) == 0;
    if (vec) {
        const float4 x = *reinterpret_cast<const float4*>(a + e), y = *reinterpret_cast<const float4*>(b + e);
        *reinterpret_cast<float4*>(out + e) = make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
        return;
    }
    for (int64_t k = e; k < e + 4 && k < n; k++) out[k] = a[k] + b[k];
}

// sum of squares partials (fixed grid -> deterministic)
__global__ void __launch_bounds__(256) sumsq_partial(const float* x, int64_t n, float* part) {
    __shared__ float red[4];
    float s = 0.f;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) s += x[e] * x[e];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// clip_grad_norm_: coef = min(max_norm / (||g|| + 1e-6), 1) (torch/csrc/api/src/nn/utils/clip_grad.h)
__global__ void clip_coef(const float* part, int nblk, float max_norm, float* coef, float* norm_out) {
    if (threadIdx.x != 0) return;
    float s = 0.f;
    for (int b = 0; b < nblk; b++) s += part[b];
    float norm = sqrtf(s);
    float c = max_norm / (norm + 1e-6f);
    *coef = c < 1.f ? c : 1.f;
    if (norm_out) *norm_out = norm;
}

// AdamW step, libtorch semantics (torch/csrc/api/src/optim/adamw.cpp): grads pre-scaled by the
// clip coefficient; grads zeroed after use (the bf16 copy is refreshed afterwards).
__global__ void adamw(float* p, float* g, float* m, float* v, int64_t n, const float* coef, float decay_mul,
                      float beta1, float beta2, float one_m_b1, float one_m_b2, float step_size, float bc2_sqrt, float eps) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    float gr = g[e] * *coef;
    float pv = p[e] * decay_mul;
    float mv = m[e] * beta1 + gr * one_m_b1;
    float vv = v[e] * beta2 + one_m_b2 * gr * gr;
    float denom = sqrtf(vv) / bc2_sqrt + eps;
    pv = pv + (-step_size) * (mv / denom);
    p[e] = pv;
    m[e] = mv;
    v[e] = vv;
    g[e] = 0.f;
}

template <bool F16>
__global__ void to_half(const float* p, uint16_t* h, int64_t n) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < n) h[e] = mlp::f2h<F16>(p[e]);
}

template <bool F16>
__global__ void bf16_to_f32(const uint16_t* h, float* f, int64_t n) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < n) f[e] = mlp::h2f<F16>(h[e]);
}

// torch-default Linear init U(-1/sqrt(fan_in), 1/sqrt(fan_in)) (kaiming_uniform a=sqrt(5) for
// weights, the same bound for biases); LayerNorm weight 1, bias 0.
__global__ void init_uniform(float* p, int64_t n, float bound, uint64_t seed, uint32_t stream_id) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    float u = (float)(philox(seed, (uint32_t)e, stream_id) >> 8) * (1.f / 16777216.f);
    p[e] = (2.f * u - 1.f) * bound;
}
__global__ void fill(float* p, int64_t n, float v) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < n) p[e] = v;
}

// mean / unbiased std (fp64 accumulation): part[blk] = (sum, sumsq)
__global__ void __launch_bounds__(256) moments_partial(const float* x, int64_t n, double* part) {
    __shared__ double red[2][256];
    double s = 0, s2 = 0;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
        double v = x[e];
        s += v;
        s2 += v * v;
    }
    red[0][threadIdx.x] = s;
    red[1][threadIdx.x] = s2;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            red[0][threadIdx.x] += red[0][threadIdx.x + o];
            red[1][threadIdx.x] += red[1][threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = red[0][0];
        part[2 * blockIdx.x + 1] = red[1][0];
    }
}
__global__ void moments_final(const double* part, int nblk, int64_t n, float* out) {
    if (threadIdx.x != 0) return;
    double s = 0, s2 = 0;
    for (int b = 0; b < nblk; b++) {
        s += part[2 * b];
        s2 += part[2 * b + 1];
    }
    double mean = s / (double)n;
    double var = n > 1 ? (s2 - s * mean) / (double)(n - 1) : 0.0;
    out[0] = (float)mean;
    out[1] = (float)sqrt(var > 0 ? var : 0.0);
}

__global__ void perm_keys(uint32_t* keys, int32_t* vals, int64_t n, uint64_t seed, uint32_t counter) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    keys[e] = philox(seed, (uint32_t)e, counter);
    vals[e] = (int32_t)e;
}

}  // namespace ppo
