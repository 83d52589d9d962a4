// learner.hpp -- C++ host API of the MI355X rollout engine: the GigaLearnCPP Learner /
// ExperienceBuffer / WelfordStat and the RLGymCPP EnvSet surface over the rlgpu C ABI.
//
// This is the host code the reference's src/ExampleMain.cpp drops onto (host/example_main.cpp
// mirrors it).  Every C-ABI status is turned back into std::runtime_error, so the reference's
// try/catch (Learner.cpp:466-474, ExampleMain.cpp:603-612) keeps its behaviour.
//
// Reference map (GigaLearnCPP/RLGymCPP, paths as SURVEY.md):
//   RLGC::EnvSetGPU      RG/EnvSet/EnvSet.h:67-124        (EnvSet: StepFirstHalf / StepSecondHalf /
//                                                           Sync / Reset / ResetArena / state)
//   GGL::WelfordStat     GL/private/GigaLearnCPP/Util/WelfordStat.h:7-67
//   GGL::ExperienceBuffer GL/private/GigaLearnCPP/PPO/ExperienceBuffer.{h,cpp} ([T, P] in HBM)
//   GGL::PPOLearnerGPU   GL/private/GigaLearnCPP/PPO/PPOLearner.{h,cpp}
//   GGL::Learner         GL/public/GigaLearnCPP/Learner.{h,cpp}
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../include/rlgpu_env.h"
#include "../../include/rlgpu_gae.h"
#include "../../include/rlgpu_learner.h"
#include "../../include/rlgpu_ppo.h"

namespace RLGC {

inline void RlgpuCheck(int st, const char* what) {
    if (st != RLGPU_OK) throw std::runtime_error(std::string(what) + ": " + rlgpu_last_error());
}

// RLGC::EnvSet on the device (EnvSet.h:67-124): the ExampleMain plugin set built in.
class EnvSetGPU {
public:
    EnvSetGPU(const rlgpu_envset_config& cfg, hipStream_t stream);
    ~EnvSetGPU();
    EnvSetGPU(const EnvSetGPU&) = delete;
    EnvSetGPU& operator=(const EnvSetGPU&) = delete;

    void StepFirstHalf(bool async = true);                        // EnvSet.cpp:113-130
    void StepSecondHalf(const int32_t* d_actions, bool async);    // EnvSet.cpp:132-273
    void Step(const int32_t* d_actions, const rlgpu_step_outputs* out);  // fused + reset + append
    void Sync();                                                  // EnvSet.h:107
    void Reset();                                                 // EnvSet.cpp:331-354
    void ResetArenas(const uint8_t* d_mask);                      // EnvSet.cpp:275-329

    rlgpu_envset* handle() const { return h_; }
    const rlgpu_envset_buffers& state() const { return state_; }  // EnvSet::state (device views)

private:
    rlgpu_envset* h_ = nullptr;
    rlgpu_envset_buffers state_{};
    hipStream_t stream_;
};

}  // namespace RLGC

namespace GGL {

using RLGC::RlgpuCheck;

// WelfordStat.h:7-67: fp64 running mean / variance in the reference's update order.
struct WelfordStat {
    int64_t count = 0;
    double mean = 0, m2 = 0;
    void Increment(const float* xs, int64_t n);
    double GetMean() const { return count < 2 ? 0.0 : mean; }
    double GetSTD() const;
};

// (mean, unbiased std) from fp64 (sum, sum of squares, count): PPOLearner.cpp:360-371 over ranks
void MomentsMeanStd(const double* m3, float* out2);

// ExperienceBuffer::GetAllBatchesShuffled boundaries (ExperienceBuffer.cpp:117-162).
std::vector<std::pair<int64_t, int64_t>> BatchRanges(int64_t expSize, int64_t batchSize, bool overbatching);

// The rollout ([T, P] time-major) in HBM; every collected step is trained in the iteration that
// collected it (the unfinished tail bootstrapped from V(obs_T), DESIGN.md Deviations 5).
// In RLGPU_EXP_TRAJECTORIES the same arrays are a circular per-player step store of T rows (obs row r
// = the state the step at row r acted on) and the outputs (values, GAE, truncation rows) live in the
// combined batch instead (rollout_outputs = false).
struct ExperienceBuffer {
    int T = 0, P = 0, W = 0;  // W: obs row width (RLGPU_OBS x frames)
    rlgpu_rollout_view v{};
    std::vector<void*> allocs;
    void Allocate(int T, int P, int W, bool rollout_outputs = true);
    void Free();
};

// Device arrays that grow on demand (kept across iterations).
template <class T>
struct DevArray {
    T* p = nullptr;
    int64_t cap = 0;
    void Reserve(int64_t n, hipStream_t s, bool keep = false);
    void Free();
};

// RLGPU_EXP_TRAJECTORIES state: per-player trajectories, this iteration's records, truncation list and
// the combined batch (the reference's combinedTraj)
struct TrajectoryStore {
    int Tmax = 0, maxLen = 0;
    int64_t tsPerItr = 0;
    int64_t step = 0;           // global step counter (store row = step % Tmax)
    int64_t firstStep = 0;      // this iteration's first step
    int steps = 0;              // steps collected this iteration
    int lastOldTeam = -1;
    int32_t *start = nullptr, *len = nullptr, *trnew = nullptr;
    int64_t* counters = nullptr;      // device lk::kTcCount
    int64_t* hcounters = nullptr;     // pinned host copy
    DevArray<int32_t> rp, rstart, rlen, rcode, rtidx;
    DevArray<int64_t> roff;
    DevArray<float> truncObs, truncVals;
    DevArray<float> cObs, cLogp, cRews, cVals, cAdv, cTarget, cRet;
    DevArray<uint8_t> cMasks;
    DevArray<int32_t> cActs;
    DevArray<int8_t> cTerms;
    float* truncStage = nullptr;  // [P][W] stacked pre-reset rows (frame stacking)
    int64_t nrec = 0, ntrunc = 0, nrows = 0;
};

// PPOLearner (PPOLearner.h:41-59) over rlgpu_ppo.
class PPOLearnerGPU {
public:
    PPOLearnerGPU(const rlgpu_ppo_config& cfg, hipStream_t stream);
    ~PPOLearnerGPU();
    PPOLearnerGPU(const PPOLearnerGPU&) = delete;
    PPOLearnerGPU& operator=(const PPOLearnerGPU&) = delete;

    void InferActions(const float* d_obs, const uint8_t* d_masks, int n, bool deterministic, uint64_t step,
                      int32_t* d_actions, float* d_logp, const uint8_t* d_old_rows = nullptr);
    void InferCritic(const float* d_obs, int64_t n, float* d_values);
    void AdvantageStats(const float* d_adv, int64_t n);  // (mean, unbiased std) -> adv_stats
    void Minibatch(const float* d_obs, const uint8_t* d_masks, const int32_t* d_actions, const float* d_logp,
                   const float* d_adv, const float* d_target, const int32_t* d_index, int64_t start, int n,
                   int64_t batch);
    void OptimizerStep();
    int64_t minibatches = 0;  // summed into metrics() since the last reset

    rlgpu_ppo* handle() const { return h_; }
    float* grads() const { return grads_; }
    int64_t num_params() const { return nparams_; }
    float* adv_stats() const { return adv_stats_; }
    float* metrics() const { return metrics_; }

private:
    rlgpu_ppo* h_ = nullptr;
    hipStream_t stream_;
    float* grads_ = nullptr;
    int64_t nparams_ = 0;
    float* adv_stats_ = nullptr;  // device [2]
    float* metrics_ = nullptr;    // device [RLGPU_NUM_METRICS]
};

// GGL::Learner (Learner.h:11-45): one rank's training loop.
class Learner {
public:
    Learner(const rlgpu_learner_config& cfg, const rlgpu_collective* coll, hipStream_t stream);
    ~Learner();
    Learner(const Learner&) = delete;
    Learner& operator=(const Learner&) = delete;

    void Collect();           // Learner.cpp:669-861
    void Consume();           // Learner.cpp:863-990
    void Learn();             // PPOLearner::Learn, PPOLearner.cpp:278-581
    void FinishIteration();   // obs[0] <- obs[T], step counters
    rlgpu_learner_report Iterate();
    void Start(int64_t iterations);  // Learner::Start loop (Learner.cpp:482-1056), a fixed count

    void SetOldTeam(int team) { oldTeam_ = team; }
    void SetGradHook(rlgpu_grad_hook_fn fn, void* user) {
        gradHook_ = fn;
        gradHookUser_ = user;
    }
    void SetStepHook(rlgpu_step_hook_fn fn, void* user) {
        hook_ = fn;
        hookUser_ = user;
    }
    void SetEnvTiming(bool on) { envTiming_ = on; }

    const rlgpu_learner_config& config() const { return cfg_; }
    RLGC::EnvSetGPU& env() { return *env_; }
    PPOLearnerGPU& ppo() { return *ppo_; }
    ExperienceBuffer& exp() { return exp_; }
    rlgpu_learner_stats stats;
    WelfordStat returnStat;

private:
    void StepEnv(const int32_t* d_actions, const rlgpu_step_outputs& o);
    void AllReduceGrads(int epoch, int batch);
    void BatchAdvantageStats(const float* d_adv, const int32_t* d_idx, int64_t n);
    void CollectTrajectories();
    void ConsumeTrajectories();
    void FeedReturnStat(const float* d_ret, const std::vector<int64_t>& idx, int32_t m);
    bool trajMode() const { return cfg_.experience_mode == RLGPU_EXP_TRAJECTORIES; }
    hipStream_t s_;
    rlgpu_learner_config cfg_;
    rlgpu_collective coll_{};
    bool hasColl_ = false;
    RLGC::EnvSetGPU* env_ = nullptr;
    PPOLearnerGPU* ppo_ = nullptr;
    ExperienceBuffer exp_;
    int oldTeam_ = -1;
    bool envTiming_ = false;
    rlgpu_step_hook_fn hook_ = nullptr;  // host plugins / StepCallbackFn (rlgpu_learner_set_step_hook)
    void* hookUser_ = nullptr;
    rlgpu_grad_hook_fn gradHook_ = nullptr;
    void* gradHookUser_ = nullptr;
    int K_ = 1;                 // frames stacked (config C4)
    float* hist_ = nullptr;     // [K-1][P][OBS] frame history
    std::vector<hipEvent_t> ev_;
    // the rollout collection in arena groups (rlgpu_learner_config.collect_groups): one stream per group, joined
    // to s_ by events at the phase's start and end
    std::vector<hipStream_t> gs_;
    std::vector<hipEvent_t> gsEnd_;
    hipEvent_t gsStart_ = nullptr;
    int CollectGroups() const;
    int collectGroupsUsed_ = 1;
    void CollectGrouped(int G);
    // device scratch
    uint8_t* oldRows_[2] = {nullptr, nullptr};
    int32_t* trainRows_ = nullptr;
    int32_t* perm_ = nullptr;     // the shuffle, its row-selected form and the gathered batch advantages:
    int32_t* permRows_ = nullptr; // permCap_ rows each (T * P; grown to the combined batch in the
    float* badv_ = nullptr;       // trajectory mode, whose row count has no fixed bound)
    int64_t permCap_ = 0;
    void NeedLearnRows(int64_t n, const char* what) const;
    void ReserveLearnRows(int64_t M);
    int32_t* truncRows_ = nullptr;
    int32_t* truncCount_ = nullptr;
    void* selScratch_ = nullptr;
    size_t selBytes_ = 0;
    float* truncObsC_ = nullptr;
    float* truncValC_ = nullptr;
    int64_t truncCap_ = 0;
    int64_t* sampleIdx_ = nullptr;
    float* samples_ = nullptr;
    int32_t* ends_ = nullptr;          // [P] last trajectory end per column (return sampling)
    std::vector<int32_t> hostEnds_;
    double* mom_ = nullptr;   // [3] + scratch
    float* clipSums_ = nullptr;  // [2] GAE clip-portion partial sums
  public:
    TrajectoryStore traj;      // RLGPU_EXP_TRAJECTORIES
  private:
    std::vector<void*> allocs_;
    template <class T>
    T* Alloc(size_t count);
    void Release(void* p);
};

}  // namespace GGL
