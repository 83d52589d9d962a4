/*
 * sampler_ref.c -- ORACLE (test infrastructure only): CPU restatement of the action sampler of
 * PPOLearner::InferActionsFromModels / InferPolicyProbsFromModels
 * (GigaLearnCPP/src/private/GigaLearnCPP/PPO/PPOLearner.cpp:78-184):
 *   logits + ACTION_DISABLED_LOGIT (-1e10) * !mask           :97-105
 *   softmax over all A columns, clamp [ACTION_MIN_PROB 1e-11, 1] :107-115
 *   deterministic: argmax (lowest index on ties)              :124-128
 *   otherwise the reference's CPU sampler (:143-178): r uniform in [0, 1), running += p[j] in column
 *     order, the first j with r <= running, cols - 1 when none; log(std::max(1e-12f, p[picked])).  The
 *     uniform is a Philox4x32-10 draw, key = seed, counter = (global row, step) -- the reference's
 *     thread-local mt19937 is unseeded, so the draw is injected and both sides use this one;
 * with the softmax in the GPU kernel's operation order (reinforcement-learning_amd/csrc/ppo_kernels.hpp
 * sample_rows: lane l of a 64-lane wave holds actions 2l and 2l+1; max and sum are xor butterflies,
 * i.e. pairwise trees over the lanes; libtorch's softmax order is unpinned), with exp / log from
 * include/rlgpu_detmath.h.  Built with -ffp-contract=off.
 * Logits are the policy's 16-bit (bf16 or fp16) outputs, as the sampler reads them.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "../include/rlgpu_detmath.h"

#define NL 64
static const float kMinProb = 1e-11f, kDisabled = -1e10f;

/* the sampler's key: the step's high 32 bits folded into the seed (ppo_kernels.hpp sample_key) */
static uint64_t sample_key(uint64_t seed, uint64_t step) { return seed ^ ((step >> 32) * 0x9E3779B97F4A7C15ull); }

static uint32_t philox(uint64_t key, uint32_t c0, uint32_t c1) {
    uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
    uint32_t x0 = c0, x1 = c1, x2 = 0x2545F491u, x3 = 0x4F6CDD1Du;
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * x0, p1 = (uint64_t)0xCD9E8D57u * x2;
        uint32_t y0 = (uint32_t)(p1 >> 32) ^ x1 ^ k0, y1 = (uint32_t)p1, y2 = (uint32_t)(p0 >> 32) ^ x3 ^ k1, y3 = (uint32_t)p0;
        x0 = y0;
        x1 = y1;
        x2 = y2;
        x3 = y3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return x0;
}

/* 16-bit storage -> float, exact (bf16: the high half of an f32; fp16: IEEE binary16) */
static float h2f(uint16_t h, int f16) {
    if (!f16) return rs_bits_float((uint32_t)h << 16);
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16, ex = (h >> 10) & 0x1fu, man = h & 0x3ffu;
    if (ex == 0x1f) return rs_bits_float(sign | 0x7f800000u | (man << 13));
    if (ex == 0) {
        if (man == 0) return rs_bits_float(sign);
        float v = (float)man * (1.0f / 16777216.0f); /* man * 2^-24, exact */
        return sign ? -v : v;
    }
    return rs_bits_float(sign | ((ex + 112) << 23) | (man << 13));
}

/* logit idx of a row block: kind 0 bf16, 1 fp16 (16-bit storage), 2 fp32 (the pointer holds floats: the
 * useHalfPrecision = false inference, Models.cpp:36-68) */
static float logit_at(const uint16_t* base, int64_t idx, int kind) {
    if (kind == 2) return ((const float*)(const void*)base)[idx];
    return h2f(base[idx], kind);
}

/* pairwise tree over the 64 lanes (the xor butterfly's result on every lane) */
static float tree_sum(float* v) {
    for (int w = NL / 2; w >= 1; w >>= 1)
        for (int l = 0; l < w; l++) v[l] = v[l] + v[l + w];
    return v[0];
}
static float tree_max(float* v) {
    for (int w = NL / 2; w >= 1; w >>= 1)
        for (int l = 0; l < w; l++) v[l] = fmaxf(v[l], v[l + w]);
    return v[0];
}

void oracle_sample_actions(const uint16_t* logits, const uint8_t* masks, int64_t n, int A, int deterministic,
                           uint64_t seed, uint64_t step, int64_t row0, int f16, int32_t* act, float* logp) {
    for (int64_t row = 0; row < n; row++) {
        const int64_t lg = row * A;
        const uint8_t* mk = masks + row * A;
        float z0[NL], z1[NL], p0[NL], p1[NL], t[NL];
        int in0[NL], in1[NL];
        for (int l = 0; l < NL; l++) {
            const int a0 = 2 * l, a1 = 2 * l + 1;
            in0[l] = a0 < A;
            in1[l] = a1 < A;
            z0[l] = in0[l] ? logit_at(logits, lg + a0, f16) + (mk[a0] ? 0.f : kDisabled) : 0.f;
            z1[l] = in1[l] ? logit_at(logits, lg + a1, f16) + (mk[a1] ? 0.f : kDisabled) : 0.f;
            t[l] = fmaxf(in0[l] ? z0[l] : -INFINITY, in1[l] ? z1[l] : -INFINITY);
        }
        const float m = tree_max(t);
        for (int l = 0; l < NL; l++) {
            z0[l] = in0[l] ? rs_expf(z0[l] - m) : 0.f;
            z1[l] = in1[l] ? rs_expf(z1[l] - m) : 0.f;
            t[l] = z0[l] + z1[l];
        }
        const float s = tree_sum(t);
        for (int l = 0; l < NL; l++) {
            p0[l] = in0[l] ? fminf(fmaxf(z0[l] / s, kMinProb), 1.f) : 0.f;
            p1[l] = in1[l] ? fminf(fmaxf(z1[l] / s, kMinProb), 1.f) : 0.f;
        }
        int pick = 0;
        if (deterministic) {
            float best = -1.f;
            for (int a = 0; a < A; a++) {
                const float p = (a & 1) ? p1[a >> 1] : p0[a >> 1];
                if (p > best) {
                    best = p;
                    pick = a;
                }
            }
        } else {  /* PPOLearner.cpp:157-173 */
            const float r = (float)(philox(sample_key(seed, step), (uint32_t)(row0 + row), (uint32_t)step) >> 8) * (1.f / 16777216.f);
            float running = 0.f;
            pick = A - 1;
            for (int j = 0; j < A; j++) {
                running += (j & 1) ? p1[j >> 1] : p0[j >> 1];
                if (r <= running) {
                    pick = j;
                    break;
                }
            }
        }
        act[row] = pick;
        const float pp = (pick & 1) ? p1[pick >> 1] : p0[pick >> 1];
        if (logp) logp[row] = rs_logf(1e-12f < pp ? pp : 1e-12f); /* std::log(std::max(1e-12f, p)) :176 */
    }
}

/* The clamped probs [n][A] the sampler draws from and each row's uniform r (tests restate the reference's
 * CPU loop, PPOLearner.cpp:157-178, on them in numpy). */
void oracle_sampler_probs(const uint16_t* logits, const uint8_t* masks, int64_t n, int A, uint64_t seed, uint64_t step,
                          int64_t row0, int f16, float* probs, float* r) {
    for (int64_t row = 0; row < n; row++) {
        const int64_t lg = row * A;
        const uint8_t* mk = masks + row * A;
        float z0[NL], z1[NL], t[NL];
        int in0[NL], in1[NL];
        for (int l = 0; l < NL; l++) {
            const int a0 = 2 * l, a1 = 2 * l + 1;
            in0[l] = a0 < A;
            in1[l] = a1 < A;
            z0[l] = in0[l] ? logit_at(logits, lg + a0, f16) + (mk[a0] ? 0.f : kDisabled) : 0.f;
            z1[l] = in1[l] ? logit_at(logits, lg + a1, f16) + (mk[a1] ? 0.f : kDisabled) : 0.f;
            t[l] = fmaxf(in0[l] ? z0[l] : -INFINITY, in1[l] ? z1[l] : -INFINITY);
        }
        const float m = tree_max(t);
        for (int l = 0; l < NL; l++) {
            z0[l] = in0[l] ? rs_expf(z0[l] - m) : 0.f;
            z1[l] = in1[l] ? rs_expf(z1[l] - m) : 0.f;
            t[l] = z0[l] + z1[l];
        }
        const float s = tree_sum(t);
        for (int a = 0; a < A; a++) {
            const float e = (a & 1) ? z1[a >> 1] : z0[a >> 1];
            probs[row * A + a] = fminf(fmaxf(e / s, kMinProb), 1.f);
        }
        r[row] = (float)(philox(sample_key(seed, step), (uint32_t)(row0 + row), (uint32_t)step) >> 8) * (1.f / 16777216.f);
    }
}

/* rs_expf / rs_logf over arrays (known-answer tests of the shared kernels against libm) */
/* rs_sinf / rs_cosf / rs_atan2f / rs_asinf over arrays (op 0 sin x, 1 cos x, 2 atan2(y, x), 3 asin x, 4 atan x);
 * liboracle_libm.so returns the host libm's values at the call sites selected by oracle_set_libm_sites */
#ifdef RLGPU_DETMATH_LIBM
int rlgpu_libm_sites = RS_SITE_ANY;
void oracle_set_libm_sites(int mask) { rlgpu_libm_sites = mask; }
#endif
void oracle_detmath_trig(int op, const float* x, const float* y, int64_t n, float* out) {
    for (int64_t i = 0; i < n; i++) {
        switch (op) {
        case 0: out[i] = rs_sinf(x[i]); break;
        case 1: out[i] = rs_cosf(x[i]); break;
        case 2: out[i] = rs_atan2f(y[i], x[i]); break;
        case 3: out[i] = rs_asinf(x[i]); break;
        default: out[i] = rs_atanf(x[i]); break;
        }
    }
}

void oracle_detmath_exp_log(const float* x, int64_t n, float* ex, float* lg) {
    for (int64_t i = 0; i < n; i++) {
        if (ex) ex[i] = rs_expf(x[i]);
        if (lg) lg[i] = rs_logf(x[i]);
    }
}
