/*
 * rlgpu_gae.h -- C ABI for the GAE (generalised advantage estimation) stage of
 * the MI355X rollout engine.
 *
 * Replaces: GGL::GAE::Compute
 *   GigaLearnCPP/src/private/GigaLearnCPP/PPO/GAE.h:9-13
 *   GigaLearnCPP/src/private/GigaLearnCPP/PPO/GAE.cpp:7-208
 * whose libtorch tensors become plain device pointers here.  Semantics (reward
 * normalisation by returnStd when returnStd is not 0 or 1, clip to +-clipRange,
 * NORMAL/TRUNCATED terminal handling with the k-th truncation bootstrapped from
 * truncValPreds[k], returns computed from the RAW rewards, target = V + A, and
 * the clipped-reward-portion metric) follow GAE.cpp line by line.
 *
 * All pointers are device pointers (HBM) unless the name starts with h_.
 * Every function returns 0 on success and a negative rlgpu_status on error;
 * rlgpu_last_error() (rlgpu_core.h) gives the message.  No C++ exception
 * crosses this boundary (reference convention: RG_ERR_CLOSE throws,
 * GigaLearnCPP/RLGymCPP/src/RLGymCPP/Framework.h:16-21).
 */
#ifndef RLGPU_GAE_H
#define RLGPU_GAE_H

#include <stdint.h>
#include "rlgpu_core.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Flat, episode-concatenated layout (exactly GAE::Compute's input):
 *   d_rews[M] f32, d_terms[M] int8 in {0,1=NORMAL,2=TRUNCATED},
 *   d_vals[M] f32, d_trunc_vals[num_truncs] f32 (may be NULL if num_truncs==0)
 * Outputs d_adv[M], d_target[M], d_ret[M] f32 and, if h_clip_portion != NULL,
 * the clipped-reward portion (this synchronises the stream).
 * Computed with a chunked, wavefront-segmented affine reverse scan; results
 * agree with the sequential reference to float rounding (tests use 1e-5 rel). */
int rlgpu_gae_flat(const float* d_rews, const int8_t* d_terms, const float* d_vals,
                   const float* d_trunc_vals, int64_t num_returns, int64_t num_truncs,
                   float gamma, float lambda, float return_std, float clip_range,
                   float* d_adv, float* d_target, float* d_ret, float* h_clip_portion,
                   void* stream);

/* Rollout layout [T][N] (time-major, N agents contiguous): the engine's own
 * experience buffer.  d_trunc_vals[T][N] holds V(obs before reset) where the
 * terminal is TRUNCATED (ignored elsewhere); d_boot_vals[N] = V(obs_T) for the
 * unfinished tail (pass NULL for 0, i.e. reference behaviour of the last step).
 * One lane per agent walks t = T-1..0 in the reference's exact operation order,
 * so results are bit-identical to the CPU oracle.  d_clip_partials (optional,
 * 2 floats) receives sum|r/std| and sum|clip(r/std)| via atomics. */
int rlgpu_gae_rollout(const float* d_rews, const int8_t* d_terms, const float* d_vals,
                      const float* d_trunc_vals, const float* d_boot_vals,
                      int32_t T, int32_t N, float gamma, float lambda,
                      float return_std, float clip_range,
                      float* d_adv, float* d_target, float* d_ret, float* d_clip_partials,
                      void* stream);

/* Complete trajectories of a flat batch -- the reference's combinedTraj (Learner.cpp:823-861), whose
 * every trajectory ends in its only nonzero code: segment k covers rows [d_seg_off[k],
 * d_seg_off[k] + d_seg_len[k]), d_seg_tidx[k] is its index into d_trunc_vals when it ends TRUNCATED
 * (else -1).  One lane per segment walks it backwards in GAE::Compute's operation order
 * (GAE.cpp:169-193).  This equals rlgpu_gae_flat's sequential reference over the concatenation BIT
 * FOR BIT whenever no reward is -0: across a terminal the recursion's carry is multiplied by
 * notDoneNotTrunc = 0, so only a -0 reward could expose the carry's sign (the env's weighted reward
 * sums start at +0 and are never -0).  d_clip_partials as rlgpu_gae_rollout. */
int rlgpu_gae_segments(const float* d_rews, const int8_t* d_terms, const float* d_vals, const float* d_trunc_vals,
                       const int64_t* d_seg_off, const int32_t* d_seg_len, const int32_t* d_seg_tidx,
                       int64_t num_segments, float gamma, float lambda, float return_std, float clip_range,
                       float* d_adv, float* d_target, float* d_ret, float* d_clip_partials, void* stream);

#ifdef __cplusplus
}
#endif
#endif
