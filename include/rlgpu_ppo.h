/*
 * rlgpu_ppo.h -- C ABI for the PPO actor/critic of the MI355X rollout engine.
 *
 * Replaces (GigaLearnCPP, libtorch-based):
 *   GGL::Model  [Linear -> LayerNorm -> LeakyReLU] x k -> Linear
 *                                   src/private/GigaLearnCPP/Util/Models.cpp:7-69, Models.h:21-163
 *   PPOLearner::InferActionsFromModels / InferPolicyProbsFromModels
 *                                   src/private/GigaLearnCPP/PPO/PPOLearner.cpp:78-184
 *   PPOLearner::InferCritic / InferCriticBatched     PPOLearner.cpp:186-251
 *   PPOLearner::Learn (minibatch loss + backward, clip_grad_norm_, optimizer step)
 *                                   PPOLearner.cpp:278-581
 *   AdamW (libtorch defaults)        Models.h:40-56, torch/csrc/api/src/optim/adamw.cpp
 *
 * One handle owns, in HBM: the flat fp32 parameters of every model (torch parameters()
 * order: per layer Linear.weight [out,in], Linear.bias, LayerNorm.weight, LayerNorm.bias;
 * then the output Linear), their gradients, AdamW moments, the bf16 inference copy
 * ("seqHalf", refreshed after every optimizer step) and the activation workspace for
 * up to cfg.max_rows rows.  Models: 0 = policy (actor), 1 = critic, 2 = the optional shared head
 * (cfg.n_shared_layers > 0; it comes last in the flat buffers so the policy / critic offsets do not
 * depend on it).  With a shared head every policy / critic entry point runs it first, as
 * PPOLearner::InferPolicyProbsFromModels / InferCritic / Learn do (PPOLearner.cpp:78-112,186-199,396-398).
 *
 * Arithmetic: training forward/backward in fp32 (cfg.train_gemm: the three-way bf16 split on
 * bf16 MFMA by default, or f32-input MFMA v_mfma_f32_32x32x2_f32), inference in bf16 on v_mfma_f32_32x32x16_bf16 with fp32 accumulation -- the reference's
 * precision split (Model::Forward: halfPrec only without grad).
 *
 * All d_ pointers are device pointers; every call is enqueued on `stream` (NULL = default)
 * without a host sync unless stated.  Return 0 or a negative rlgpu_status (rlgpu_core.h).
 */
#ifndef RLGPU_PPO_H
#define RLGPU_PPO_H

#include <stdint.h>
#include "rlgpu_core.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RLGPU_MAX_LAYERS 8

typedef struct {
    int32_t obs_size;                         /* 167 (AdvancedObs) */
    int32_t num_actions;                      /* 90 (DefaultAction) */
    int32_t policy_layers[RLGPU_MAX_LAYERS];  /* hidden sizes (1..2048), e.g. {512, 512} */
    int32_t n_policy_layers;
    int32_t critic_layers[RLGPU_MAX_LAYERS];
    int32_t n_critic_layers;
    int32_t layer_norm;                       /* ModelConfig::addLayerNorm (eps 1e-5, affine) */
    float leaky_slope;                        /* torch::nn::LeakyReLU default 0.01 */
    float policy_lr, critic_lr;               /* PPOLearnerConfig::policyLR / criticLR */
    float beta1, beta2, eps, weight_decay;    /* AdamW: 0.9, 0.999, 1e-8, 1e-2 */
    float clip_range;                         /* 0.2 */
    float entropy_scale;                      /* 0.035 (ExampleMain) */
    float max_grad_norm;                      /* 0.5 (PPOLearner.cpp:521-526) */
    int32_t max_rows;                         /* workspace rows: max(minibatch, inference chunk) */
    uint64_t seed;                            /* parameter init + action sampling (Philox) */
    int32_t train_gemm;                       /* training GEMM arithmetic: RLGPU_GEMM_F32X6 (0),
                                                 RLGPU_GEMM_F32 (1) or RLGPU_GEMM_F16X3 (2) -- see rlgpu_gemm */
    int32_t infer_fp16;                       /* inference precision (RLGPU_INFER_*): 0 = bf16 (the reference's
                                                 seqHalf), 1 = fp16 on v_mfma_f32_32x32x16_f16 (BASELINE config
                                                 C5), 2 = fp32 (PPOLearnerConfig::useHalfPrecision = false:
                                                 Model::Forward's fp32 branch, Models.cpp:36-68, on the training
                                                 forward; no old-version inference in this mode) */
    /* PPOLearnerConfig::sharedHead (PPOLearner.cpp:42-74): [Linear -> LayerNorm -> LeakyReLU] x k with
     * no output layer, run once on the obs; policy and critic then take its last activation as input
     * (ExampleMain: {512, 512} x scale, run_out.log:25-28 shows [384, 384]).  n_shared_layers = 0: no
     * shared head (policy and critic read the obs).  Model index 2; learning rate
     * min(policy_lr, critic_lr) (PPOLearner::SetLearningRates, PPOLearner.cpp:652-663). */
    int32_t shared_layers[RLGPU_MAX_LAYERS];
    int32_t n_shared_layers;
    /* global row number of this handle's row 0 for the sampler's Philox counter (row, step): rank r of a
     * data-parallel job passes r x its rows, so the ranks draw what one device holding every row draws */
    int64_t sample_row_offset;
} rlgpu_ppo_config;

/* fp32 GEMM arithmetic of the training path (libtorch fp32 Linear forward / backward in the
 * reference, Models.cpp:42-68):
 *   RLGPU_GEMM_F32X6  every f32 operand split exactly into three bf16 terms (h + m + l), the six
 *                     products above 2^-24 relative on v_mfma_f32_32x32x16_bf16, leading and
 *                     correction terms in separate f32 accumulators: f32-class accuracy at 8/3 x
 *                     the f32-MFMA rate (gfx950's f32-input MFMA runs at 1/16 of bf16);
 *   RLGPU_GEMM_F32    v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulate);
 *   RLGPU_GEMM_F16X3  every operand tensor scaled by a power of two (its max |x| into [2^14, 2^15))
 *                     and split exactly into two fp16 terms (h + l, 22 significant bits), the
 *                     three products h h + h l + l h on v_mfma_f32_32x32x16_f16, leading and
 *                     correction terms in separate f32 accumulators (the 3xTF32 scheme of fp32
 *                     emulation): half the MFMAs of F32X6, products within 2^-22 relative. */
enum { RLGPU_GEMM_F32X6 = 0, RLGPU_GEMM_F32 = 1, RLGPU_GEMM_F16X3 = 2 };
/* rlgpu_ppo_config.infer_fp16 values */
enum { RLGPU_INFER_BF16 = 0, RLGPU_INFER_F16 = 1, RLGPU_INFER_F32 = 2 };

typedef struct rlgpu_ppo rlgpu_ppo;

/* Metrics accumulated by rlgpu_ppo_minibatch (PPOLearner.cpp:283-296,399-475), one float each,
 * summed over minibatches; divide by the count (the reference's numAccumulated). */
enum {
    RLGPU_M_ENTROPY = 0, RLGPU_M_KL, RLGPU_M_POLICY_LOSS, RLGPU_M_CRITIC_LOSS, RLGPU_M_RATIO,
    RLGPU_M_CLIP_FRACTION, RLGPU_M_COUNT, RLGPU_M_GRAD_NORM_POLICY, RLGPU_M_GRAD_NORM_CRITIC,
    RLGPU_M_GRAD_NORM_SHARED, RLGPU_NUM_METRICS = 16
};

int rlgpu_ppo_create(const rlgpu_ppo_config* cfg, rlgpu_ppo** out);
int rlgpu_ppo_destroy(rlgpu_ppo* h);

/* Flat fp32 buffers of all models, contiguous (policy first, then critic, then the shared head). */
int rlgpu_ppo_buffers(rlgpu_ppo* h, float** d_params, float** d_grads, int64_t* num_params);
/* Offset / count of one model (0 policy, 1 critic, 2 shared head) inside the flat buffers; without a
 * shared head model 2 has count 0 (offset = the end of the buffers). */
int rlgpu_ppo_model_range(rlgpu_ppo* h, int32_t model, int64_t* offset, int64_t* count);
/* torch-default init (Linear: U(+-1/sqrt(fan_in)) weight and bias; LayerNorm 1 / 0), Philox. */
int rlgpu_ppo_init_params(rlgpu_ppo* h, uint64_t seed, void* stream);
/* Refresh the bf16 inference copy from the fp32 parameters (Model::Forward seqHalf) and mark the
 * training GEMMs' split weight planes stale.  Call it after writing d_params directly (checkpoint
 * load, broadcasts); the optimizer step does it itself. */
int rlgpu_ppo_refresh_half(rlgpu_ppo* h, void* stream);

/* Diagnostics: while d_buf != NULL, every fused inference launch writes 16 wall-clock (100 MHz)
 * phase marks per 64-row workgroup into d_buf (uint64 [workgroups * 16] within `capacity` entries;
 * a launch needing more fails with RLGPU_ERR_INVALID_ARG; tools/infer_trace.py). */
int rlgpu_debug_infer_trace(void* d_buf, int64_t capacity);
/* Diagnostics: learn-phase kernel timing.  While enabled, HIP events bracket every training GEMM
 * and LayerNorm launch on the stream it is launched on; rlgpu_kernel_timing_read sums, per slot
 * (0 forward / input-gradient GEMMs, 1 weight-gradient GEMMs, 2 LayerNorm forward, 3 LayerNorm
 * backward), the milliseconds, the work (flops for GEMMs, algorithmic bytes for the row kernels)
 * and the launch count since the last rlgpu_kernel_timing call (it waits for the events). */
int rlgpu_kernel_timing(int32_t enable);
int rlgpu_kernel_timing_read(double* ms, double* work, int64_t* count, int32_t nslots);

/* Plain forward of one model on n rows (n <= max_rows): precision 0 = fp32 (training path,
 * no activations kept), 1 = bf16 inference path.  d_out [n, out_size] fp32.  With a shared head,
 * models 0 / 1 are shared head -> policy / critic (Model::Forward chained as the reference does) and
 * model 2 is the shared head alone (out_size = its last width).
 * The 16-bit inference (this, rlgpu_ppo_infer_actions*, rlgpu_ppo_infer_critic) runs as one fused
 * kernel per call when every layer fits it (inputs / hidden widths <= 512, outputs <= 128); the
 * environment variable RLGPU_FUSED_INFER=0 selects the layer-by-layer kernels, same results. */
int rlgpu_ppo_forward(rlgpu_ppo* h, int32_t model, int32_t precision, const float* d_in, int32_t n,
                      float* d_out, void* stream);

/* InferActions: bf16 policy forward, logits + (-1e10)*!mask, softmax, clamp [1e-11, 1],
 * then argmax (deterministic) or a multinomial draw by inverse CDF on a Philox uniform
 * (key = cfg.seed, counter = (row, rng_step)).  d_actions int32 [n], d_logp [n] (may be NULL). */
int rlgpu_ppo_infer_actions(rlgpu_ppo* h, const float* d_obs, const uint8_t* d_masks, int32_t n,
                            int32_t deterministic, uint64_t rng_step, int32_t* d_actions, float* d_logp,
                            void* stream);
/* Self-play against an old policy version (LearnerConfig trainAgainstOldVersions,
 * Learner.cpp:587-627,733-767; versions kept by PolicyVersionManager, PolicyVersionManager.cpp:38-62).
 * set_version: bf16 inference copy of a policy given as its flat fp32 parameters (torch order,
 * the policy's rlgpu_ppo_model_range count), followed by the shared head's when there is one (the
 * reference versions GetPolicyModels() = every model but the critic, PPOLearner.cpp:665-674).  infer_actions_mixed: rows with d_old_rows[i] != 0
 * act with that version (no log-prob written), the others with the current policy (as
 * rlgpu_ppo_infer_actions). */
int rlgpu_ppo_set_version(rlgpu_ppo* h, const float* d_policy_params, void* stream);
int rlgpu_ppo_infer_actions_mixed(rlgpu_ppo* h, const float* d_obs, const uint8_t* d_masks, int32_t n,
                                  int32_t deterministic, uint64_t rng_step, const uint8_t* d_old_rows,
                                  int32_t* d_actions, float* d_logp, void* stream);
/* rlgpu_ppo_infer_actions (d_old_rows NULL) or _mixed over n rows that are rows [row0, row0 + n) of this rank's
 * players (the sampler's Philox row index is row0 + i; d_obs / d_masks / d_actions / d_logp / d_old_rows point
 * at those rows).  Calls on disjoint rows may run concurrently on different streams (the C++ Learner's arena
 * groups): only on the fused inference kernel, which keeps no per-handle row buffers -- otherwise
 * RLGPU_ERR_UNSUPPORTED (rlgpu_ppo_fused_infer tells beforehand). */
int rlgpu_ppo_infer_actions_rows(rlgpu_ppo* h, const float* d_obs, const uint8_t* d_masks, int32_t n, int64_t row0,
                                 int32_t deterministic, uint64_t rng_step, const uint8_t* d_old_rows,
                                 int32_t* d_actions, float* d_logp, void* stream);
/* 1 when model `model` (0 policy, 1 critic) runs on the fused inference kernel, else 0. */
int rlgpu_ppo_fused_infer(rlgpu_ppo* h, int32_t model);
/* InferCriticBatched: bf16 critic forward over n rows (any n; chunked by max_rows). */
int rlgpu_ppo_infer_critic(rlgpu_ppo* h, const float* d_obs, int64_t n, float* d_values, void* stream);

/* Mean and unbiased std of d_x[n] into d_out[2] (batch advantage normalisation,
 * PPOLearner.cpp:360-371). */
int rlgpu_mean_std(const float* d_x, int64_t n, float* d_out, void* stream);

/* One Learn minibatch: rows idx[start..start+n) of the batch (d_index may be NULL = identity)
 * (with a shared head: its forward once, policy and critic on its output, and its backward from the
 * sum of their input gradients -- PPOLearner.cpp:396-398,478-498)
 * gathered from d_obs [*, obs_size], d_masks [*, A], d_actions int32, d_old_logp, d_adv,
 * d_target.  Advantages are normalised with d_adv_stats = (mean, std) as (a - mean)/(std+1e-8).
 * loss = (policyLoss - entropy*entropy_scale)*n/batch_size + MSE(V, target)*n/batch_size;
 * gradients are ACCUMULATED into the grad buffer; metrics summed into d_metrics. */
int rlgpu_ppo_minibatch(rlgpu_ppo* h, const float* d_obs, const uint8_t* d_masks, const int32_t* d_actions,
                        const float* d_old_logp, const float* d_adv, const float* d_target,
                        const int32_t* d_index, int64_t start, int32_t n, int64_t batch_size,
                        const float* d_adv_stats, float* d_metrics, void* stream);

/* clip_grad_norm_(model, max_grad_norm) per model (policy, critic, shared head: PPOLearner.cpp:521-526),
 * AdamW step (libtorch semantics), zero grads, refresh the bf16 copy.  Grad norms written to
 * d_metrics (optional). */
int rlgpu_ppo_optimizer_step(rlgpu_ppo* h, float* d_metrics, void* stream);
int rlgpu_ppo_zero_grad(rlgpu_ppo* h, void* stream);
/* Optimizer state (step count + moments) for checkpointing; moments are device pointers. */
int rlgpu_ppo_optimizer_state(rlgpu_ppo* h, int64_t* step, float** d_exp_avg, float** d_exp_avg_sq);
/* Restore the AdamW step count (checkpoint resume; the moments are written through the pointers
 * rlgpu_ppo_optimizer_state returns). */
int rlgpu_ppo_set_optimizer_step(rlgpu_ppo* h, int64_t step);

/* Building block, exported for tests and microbenchmarks: C[I,J] = sum_k A(i,k) B(k,j) (+ bias[j])
 * in the fp32 arithmetic `mode` (RLGPU_GEMM_F32X6 / RLGPU_GEMM_F32 / RLGPU_GEMM_F16X3).  a_layout 0: A stored [I][lda] (k contiguous), 1: [K][lda] (i contiguous);
 * b_layout 0: B stored [J][ldb] (k contiguous), 1: [K][ldb] (j contiguous).  splits > 1 writes
 * per-split partials to C + s*I*ldc (caller reduces).  Supported pairs: (0,0), (0,1), (1,1). */
int rlgpu_gemm(int32_t mode, int32_t a_layout, int32_t b_layout, const float* d_A, int64_t lda, const float* d_B,
               int64_t ldb, float* d_C, int64_t ldc, const float* d_bias, int32_t I, int32_t J, int32_t K, int32_t splits,
               void* stream);
/* rlgpu_gemm with mode RLGPU_GEMM_F32. */
int rlgpu_gemm_f32(int32_t a_layout, int32_t b_layout, const float* d_A, int64_t lda, const float* d_B, int64_t ldb,
                   float* d_C, int64_t ldc, const float* d_bias, int32_t I, int32_t J, int32_t K, int32_t splits,
                   void* stream);

/* Random permutation of [0, n) (Philox keys + device radix sort): ExperienceBuffer shuffle. */
int rlgpu_permutation(int64_t n, uint64_t seed, uint64_t counter, int32_t* d_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif
