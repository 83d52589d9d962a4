/*
 * gae_ref.c -- ORACLE (test infrastructure only; never linked into the product).
 *
 * Plain-C restatement of GGL::GAE::Compute,
 * GigaLearnCPP/src/private/GigaLearnCPP/PPO/GAE.cpp:7-208, used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.
 * Parity status: UNPINNED by the reference (it ships no tests or fixtures,
 * SURVEY.md section 4); pinned here by closed-form known-answer cases in
 * tests/test_gae_oracle.py and by the committed golden vectors in tests/golden/.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#define TERM_NORMAL 1    /* RLGC::TerminalType::NORMAL,    TerminalCondition.h:8 */
#define TERM_TRUNCATED 2 /* RLGC::TerminalType::TRUNCATED, TerminalCondition.h:9 */

/* Returns 0, or -1 when the truncation count does not match (GAE.cpp:196-197). */
int oracle_gae_flat(const float* rews, const int8_t* terms, const float* vals, const float* trunc_vals,
                    int64_t num_returns, int64_t num_truncs, float gamma, float lambda, float return_std,
                    float clip_range, float* out_adv, float* out_target, float* out_ret, float* out_clip_portion) {
    if (num_returns == 0) { /* GAE.cpp:16-23 */
        if (out_clip_portion) *out_clip_portion = 0;
        return 0;
    }
    const int should_normalize = (return_std != 0 && return_std != 1); /* :73 */
    const int should_clip = (clip_range > 0);                            /* :74 */
    const float inv_std = should_normalize ? (1.0f / return_std) : 1.0f;
    const float gamma_lambda = gamma * lambda;
    const int64_t last = num_returns - 1;

    float* next_vals = (float*)malloc(sizeof(float) * num_returns);
    float* nd = (float*)malloc(sizeof(float) * num_returns);
    float* nrew = (float*)malloc(sizeof(float) * num_returns);
    int64_t trunc_seen = 0;
    /* :80-101 -- the k-th truncated step takes trunc_vals[k] */
    for (int64_t step = 0; step < num_returns; step++) {
        int8_t t = terms[step];
        float done = (t == TERM_NORMAL) ? 1.0f : 0.0f;
        float trunc = (t == TERM_TRUNCATED) ? 1.0f : 0.0f;
        nd[step] = (1.0f - done) * (1.0f - trunc);
        if (t == TERM_NORMAL) {
            next_vals[step] = 0.0f;
        } else if (t == TERM_TRUNCATED && num_truncs > 0) {
            next_vals[step] = (trunc_seen < num_truncs) ? trunc_vals[trunc_seen] : 0.0f;
        } else if (step < last) {
            next_vals[step] = vals[step + 1];
        } else {
            next_vals[step] = 0.0f;
        }
        if (t == TERM_TRUNCATED) trunc_seen++;
    }
    /* :104-167 normalisation + clip; the clip-portion sums in float in the reference's order: groups
       of 8 summed left to right, each group added to the running total (:113-141), then the
       remainder one by one (:153-162). */
    float tot = 0.0f, tot_clip = 0.0f;
    if (should_normalize) {
        const int64_t unroll_end = num_returns - (num_returns % 8);
        int64_t i = 0;
        for (; i < unroll_end; i += 8) {
            float n[8];
            for (int k = 0; k < 8; k++) n[k] = rews[i + k] * inv_std;
            tot += fabsf(n[0]) + fabsf(n[1]) + fabsf(n[2]) + fabsf(n[3]) + fabsf(n[4]) + fabsf(n[5]) + fabsf(n[6]) +
                   fabsf(n[7]);
            if (should_clip)
                for (int k = 0; k < 8; k++) n[k] = fminf(fmaxf(n[k], -clip_range), clip_range);
            tot_clip += fabsf(n[0]) + fabsf(n[1]) + fabsf(n[2]) + fabsf(n[3]) + fabsf(n[4]) + fabsf(n[5]) + fabsf(n[6]) +
                        fabsf(n[7]);
            for (int k = 0; k < 8; k++) nrew[i + k] = n[k];
        }
        for (; i < num_returns; i++) {
            float n = rews[i] * inv_std;
            tot += fabsf(n);
            if (should_clip) n = fminf(fmaxf(n, -clip_range), clip_range);
            tot_clip += fabsf(n);
            nrew[i] = n;
        }
    } else {
        for (int64_t i = 0; i < num_returns; i++) nrew[i] = rews[i];
    }
    /* :169-193 backward recursion */
    float prev_lambda = 0.0f, prev_ret = 0.0f;
    for (int64_t step = last; step >= 0; step--) {
        float pred_return = nrew[step] + gamma * next_vals[step];
        float delta = pred_return - vals[step];
        float cur_return = rews[step] + prev_ret * gamma * nd[step];
        out_ret[step] = cur_return;
        prev_lambda = delta + gamma_lambda * nd[step] * prev_lambda;
        out_adv[step] = prev_lambda;
        prev_ret = cur_return;
    }
    for (int64_t i = 0; i < num_returns; i++) out_target[i] = vals[i] + out_adv[i]; /* :200 */
    if (out_clip_portion)
        *out_clip_portion = should_normalize ? (tot - tot_clip) / fmaxf(tot, 1e-7f) : 0.0f; /* :202-206 */
    free(next_vals);
    free(nd);
    free(nrew);
    return (num_truncs > 0 && trunc_seen != num_truncs) ? -1 : 0;
}

/* Rollout layout [T][N]: each agent column is an independent flat sequence whose last
   step bootstraps from boot_vals[n] (NULL -> 0, the reference's last-step rule). */
void oracle_gae_rollout(const float* rews, const int8_t* terms, const float* vals, const float* trunc_vals,
                        const float* boot_vals, int32_t T, int32_t N, float gamma, float lambda,
                        float return_std, float clip_range, float* out_adv, float* out_target, float* out_ret) {
    const int should_normalize = (return_std != 0 && return_std != 1);
    const int should_clip = (clip_range > 0);
    const float inv_std = should_normalize ? (1.0f / return_std) : 1.0f;
    const float gamma_lambda = gamma * lambda;
    for (int32_t n = 0; n < N; n++) {
        float prev_lambda = 0.0f, prev_ret = 0.0f;
        for (int32_t t = T - 1; t >= 0; t--) {
            int64_t i = (int64_t)t * N + n;
            int8_t term = terms[i];
            float rew = rews[i];
            float cur = rew;
            if (should_normalize) {
                cur = rew * inv_std;
                if (should_clip) cur = fminf(fmaxf(cur, -clip_range), clip_range);
            }
            float done = (term == TERM_NORMAL) ? 1.0f : 0.0f;
            float trunc = (term == TERM_TRUNCATED) ? 1.0f : 0.0f;
            float nd = (1.0f - done) * (1.0f - trunc);
            float next;
            if (term == TERM_NORMAL) next = 0.0f;
            else if (term == TERM_TRUNCATED) next = trunc_vals ? trunc_vals[i] : 0.0f;
            else if (t < T - 1) next = vals[i + N];
            else next = boot_vals ? boot_vals[n] : 0.0f;
            float pred_return = cur + gamma * next;
            float delta = pred_return - vals[i];
            float cur_return = rew + prev_ret * gamma * nd;
            out_ret[i] = cur_return;
            prev_lambda = delta + gamma_lambda * nd * prev_lambda;
            out_adv[i] = prev_lambda;
            out_target[i] = vals[i] + prev_lambda;
            prev_ret = cur_return;
        }
    }
}
