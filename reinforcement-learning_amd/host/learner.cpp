// learner.cpp -- the C++ host Learner (host/learner.hpp) and its C ABI (include/rlgpu_learner.h).
//
// One rank's GigaLearnCPP training loop (Learner::Start, GL/public/GigaLearnCPP/Learner.cpp:482-1056)
// driving the HIP path through the rlgpu C ABI: bf16 policy inference + the fused env kernel with
// the experience append (collection), critic + GAE + return statistics (consumption), and
// PPOLearner::Learn (learning).  Nothing leaves HBM during an iteration except the handful of
// scalars the host needs (truncation count, 150 return samples, distributed moments).
#include "learner.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>

#include "../csrc/common.hpp"
#include "../csrc/learner_kernels.hpp"

namespace {
constexpr int OBS = RLGPU_OBS, ACT = RLGPU_ACTIONS;
using clk = std::chrono::steady_clock;
double secs(clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); }

inline void hipCheck(hipError_t e, const char* what) {
    if (e != hipSuccess) throw rlgpu::Error(RLGPU_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// splitmix64 (Steele et al.): the counter-based generator of rlgpu_sample_indices
inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
}  // namespace

// ------------------------------------------------------------------ RLGC::EnvSetGPU
namespace RLGC {

EnvSetGPU::EnvSetGPU(const rlgpu_envset_config& cfg, hipStream_t stream) : stream_(stream) {
    RlgpuCheck(rlgpu_envset_create(&cfg, &h_), "EnvSet");
    RlgpuCheck(rlgpu_envset_buffers_get(h_, &state_), "EnvSet buffers");
}
EnvSetGPU::~EnvSetGPU() {
    if (h_) rlgpu_envset_destroy(h_);
}
void EnvSetGPU::StepFirstHalf(bool) { RlgpuCheck(rlgpu_envset_step_first_half(h_, stream_), "StepFirstHalf"); }
void EnvSetGPU::StepSecondHalf(const int32_t* d_actions, bool async) {
    RlgpuCheck(rlgpu_envset_step_second_half(h_, d_actions, stream_), "StepSecondHalf");
    if (!async) Sync();
}
void EnvSetGPU::Step(const int32_t* d_actions, const rlgpu_step_outputs* out) {
    RlgpuCheck(rlgpu_envset_step(h_, d_actions, 1, out, stream_), "EnvSet step");
}
void EnvSetGPU::Sync() { RlgpuCheck(rlgpu_envset_sync(h_, stream_), "Sync"); }
void EnvSetGPU::Reset() { RlgpuCheck(rlgpu_envset_reset(h_, stream_), "Reset"); }
void EnvSetGPU::ResetArenas(const uint8_t* d_mask) {
    RlgpuCheck(rlgpu_envset_reset_arenas(h_, d_mask, stream_), "ResetArena");
}

}  // namespace RLGC

// ------------------------------------------------------------------ GGL
namespace GGL {

void WelfordStat::Increment(const float* xs, int64_t n) {
    for (int64_t i = 0; i < n; i++) {  // WelfordStat.h:25-35
        double delta = (double)xs[i] - mean;
        double deltaN = delta / (double)(count + 1);
        mean += deltaN;
        m2 += delta * deltaN * (double)count;
        count++;
    }
}
double WelfordStat::GetSTD() const {  // WelfordStat.h:41-50
    if (count < 2) return 1.0;
    double var = m2 / (double)(count - 1);
    if (var <= 0) var = 1.0;
    return std::sqrt(var);
}

void MomentsMeanStd(const double* m, float* out) {
    const double mean = m[0] / m[2];
    double var = (m[1] - m[0] * mean) / (m[2] - 1);
    if (!(var > 0)) var = 0;
    out[0] = (float)mean;
    out[1] = (float)std::sqrt(var);
}

std::vector<std::pair<int64_t, int64_t>> BatchRanges(int64_t expSize, int64_t batchSize, bool overbatching) {
    std::vector<std::pair<int64_t, int64_t>> out;
    if (expSize <= 0 || batchSize <= 0) return out;
    for (int64_t start = 0; start < expSize; start += batchSize) {  // ExperienceBuffer.cpp:117-162
        int64_t end = start + batchSize;
        if (end + batchSize > expSize && overbatching) end = expSize;
        if (end > expSize || end - start <= 0) break;
        out.emplace_back(start, end);
        if (end == expSize) break;
    }
    return out;
}

template <class T>
void DevArray<T>::Reserve(int64_t n, hipStream_t s, bool keep) {
    if (n <= cap) return;
    const int64_t ncap = std::max<int64_t>(n, cap + cap / 2);
    T* q = nullptr;
    hipCheck(hipMalloc((void**)&q, (size_t)ncap * sizeof(T) + 16), "DevArray alloc");
    if (keep && p && cap > 0) hipCheck(hipMemcpyAsync(q, p, (size_t)cap * sizeof(T), hipMemcpyDeviceToDevice, s), "DevArray copy");
    if (p) {
        hipCheck(hipStreamSynchronize(s), "sync");
        (void)hipFree(p);
    }
    p = q;
    cap = ncap;
}
template <class T>
void DevArray<T>::Free() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
}

void ExperienceBuffer::Allocate(int T_, int P_, int W_, bool rollout_outputs) {
    T = T_;
    P = P_;
    W = W_;
    auto A = [&](size_t bytes) {
        void* p = nullptr;
        hipCheck(hipMalloc(&p, bytes + 16), "ExperienceBuffer alloc");
        hipCheck(hipMemset(p, 0, bytes + 16), "ExperienceBuffer memset");
        allocs.push_back(p);
        return p;
    };
    const size_t TP = (size_t)T * P, T1P = (size_t)(T + 1) * P;
    const size_t OP = rollout_outputs ? TP : (size_t)P, O1P = rollout_outputs ? T1P : (size_t)P;
    v.obs = (float*)A(T1P * W * 4);
    v.masks = (uint8_t*)A(T1P * ACT);
    v.actions = (int32_t*)A(TP * 4);
    v.logp = (float*)A(TP * 4);
    v.rewards = (float*)A(TP * 4);
    v.terms = (int8_t*)A(TP);
    v.trunc_obs = (float*)A(OP * W * 4);
    v.values = (float*)A(O1P * 4);
    v.trunc_vals = (float*)A(OP * 4);
    v.adv = (float*)A(OP * 4);
    v.target = (float*)A(OP * 4);
    v.ret = (float*)A(OP * 4);
    v.T = T;
    v.P = P;
    v.obs_width = W;
}
void ExperienceBuffer::Free() {
    for (void* p : allocs) (void)hipFree(p);
    allocs.clear();
}

PPOLearnerGPU::PPOLearnerGPU(const rlgpu_ppo_config& cfg, hipStream_t stream) : stream_(stream) {
    RlgpuCheck(rlgpu_ppo_create(&cfg, &h_), "PPOLearner");
    float* params = nullptr;
    RlgpuCheck(rlgpu_ppo_buffers(h_, &params, &grads_, &nparams_), "PPOLearner buffers");
    hipCheck(hipMalloc((void**)&adv_stats_, 2 * sizeof(float)), "adv stats");
    hipCheck(hipMalloc((void**)&metrics_, RLGPU_NUM_METRICS * sizeof(float)), "metrics");
    hipCheck(hipMemset(metrics_, 0, RLGPU_NUM_METRICS * sizeof(float)), "metrics");
    RlgpuCheck(rlgpu_ppo_init_params(h_, cfg.seed, stream_), "init params");
}
PPOLearnerGPU::~PPOLearnerGPU() {
    if (adv_stats_) (void)hipFree(adv_stats_);
    if (metrics_) (void)hipFree(metrics_);
    if (h_) rlgpu_ppo_destroy(h_);
}
void PPOLearnerGPU::InferActions(const float* d_obs, const uint8_t* d_masks, int n, bool det, uint64_t step,
                                 int32_t* d_actions, float* d_logp, const uint8_t* d_old_rows) {
    if (d_old_rows)
        RlgpuCheck(rlgpu_ppo_infer_actions_mixed(h_, d_obs, d_masks, n, det, step, d_old_rows, d_actions, d_logp, stream_),
                   "InferActions (old version)");
    else
        RlgpuCheck(rlgpu_ppo_infer_actions(h_, d_obs, d_masks, n, det, step, d_actions, d_logp, stream_), "InferActions");
}
void PPOLearnerGPU::InferCritic(const float* d_obs, int64_t n, float* d_values) {
    RlgpuCheck(rlgpu_ppo_infer_critic(h_, d_obs, n, d_values, stream_), "InferCritic");
}
void PPOLearnerGPU::AdvantageStats(const float* d_adv, int64_t n) {
    RlgpuCheck(rlgpu_mean_std(d_adv, n, adv_stats_, stream_), "advantage stats");
}
void PPOLearnerGPU::Minibatch(const float* d_obs, const uint8_t* d_masks, const int32_t* d_actions, const float* d_logp,
                              const float* d_adv, const float* d_target, const int32_t* d_index, int64_t start, int n,
                              int64_t batch) {
    RlgpuCheck(rlgpu_ppo_minibatch(h_, d_obs, d_masks, d_actions, d_logp, d_adv, d_target, d_index, start, n, batch,
                                   adv_stats_, metrics_, stream_),
               "Learn minibatch");
    minibatches++;
}
void PPOLearnerGPU::OptimizerStep() { RlgpuCheck(rlgpu_ppo_optimizer_step(h_, metrics_, stream_), "optimizer step"); }

template <class T>
T* Learner::Alloc(size_t count) {
    void* p = nullptr;
    hipCheck(hipMalloc(&p, count * sizeof(T) + 16), "Learner alloc");
    allocs_.push_back(p);
    return (T*)p;
}
void Learner::Release(void* p) {  // an Alloc'd buffer, freed before the destructor
    for (auto& q : allocs_)
        if (q == p) {
            (void)hipFree(q);
            q = allocs_.back();
            allocs_.pop_back();
            return;
        }
}

Learner::Learner(const rlgpu_learner_config& cfg, const rlgpu_collective* coll, hipStream_t stream)
    : s_(stream), cfg_(cfg) {
    RLGPU_REQUIRE(cfg.num_arenas > 0 && cfg.rollout_len > 0 && cfg.epochs > 0 && cfg.mini_batch_size > 0,
                  "Learner: num_arenas, rollout_len, epochs and mini_batch_size must be > 0");
    RLGPU_REQUIRE(cfg.world >= 1 && cfg.rank >= 0 && cfg.rank < cfg.world, "Learner: bad rank / world");
    RLGPU_REQUIRE(cfg.world == 1 || (coll && coll->allreduce_sum_f32 && coll->allreduce_sum_f64 && coll->allgather_f32),
                  "Learner: world > 1 needs a complete rlgpu_collective");
    RLGPU_REQUIRE(cfg.return_samples >= 0, "Learner: return_samples must be >= 0");
    if (coll) {
        coll_ = *coll;
        hasColl_ = cfg.world > 1;
    }
    std::memset(&stats, 0, sizeof(stats));
    const int T = cfg.rollout_len, N = cfg.num_arenas, P = 4 * N;
    rlgpu_envset_config ec{};
    ec.num_arenas = N;
    ec.tick_skip = cfg.tick_skip;
    ec.action_delay = cfg.action_delay;
    // one arena stream space for the whole job: rank r's arenas are arenas [r N, (r + 1) N) of it
    ec.seed = cfg.seed * 1000003ull;
    ec.arena_offset = cfg.rank * N;
    ec.save_rewards = 1;
    ec.max_episode_steps = (int32_t)(cfg.max_episode_duration * (120.0f / (float)cfg.tick_skip));
    ec.mesh_tris = cfg.mesh_tris;
    ec.mesh_ntris = cfg.mesh_ntris;
    ec.mesh_objects = cfg.mesh_objects;
    ec.mesh_object_ntris = cfg.mesh_object_ntris;
    ec.rewards = cfg.rewards;
    ec.n_rewards = cfg.n_rewards;
    ec.terminals = cfg.terminals;
    ec.n_terminals = cfg.n_terminals;
    ec.arith = cfg.arith;
    env_ = new RLGC::EnvSetGPU(ec, s_);
    // ExampleMain registers its StepCallback (ExampleMain.cpp:233-283, 592): restated on the device
    RlgpuCheck(rlgpu_envset_enable_step_metrics(env_->handle(), 1), "step metrics");
    // the rollout rows are the only obs / masks the Learner reads after a fused step (the stacked-frame and
    // hooked steps pass no obs rows, so the set's own buffers still get theirs): one copy per env step
    RlgpuCheck(rlgpu_envset_set_output_only(env_->handle(), 1), "output-only rows");
    K_ = cfg.frame_stack > 1 ? cfg.frame_stack : 1;
    RLGPU_REQUIRE(K_ <= 16, "Learner: frame_stack must be <= 16");
    const int W = OBS * K_;
    rlgpu_ppo_config pc{};
    pc.obs_size = W;
    pc.num_actions = ACT;
    std::memcpy(pc.policy_layers, cfg.policy_layers, sizeof(pc.policy_layers));
    pc.n_policy_layers = cfg.n_policy_layers;
    std::memcpy(pc.critic_layers, cfg.critic_layers, sizeof(pc.critic_layers));
    pc.n_critic_layers = cfg.n_critic_layers;
    std::memcpy(pc.shared_layers, cfg.shared_layers, sizeof(pc.shared_layers));
    pc.n_shared_layers = cfg.n_shared_layers;
    RLGPU_REQUIRE(cfg.activation == RLGPU_ACT_LEAKY_RELU || cfg.activation == RLGPU_ACT_RELU,
                  "Learner: activation must be RLGPU_ACT_LEAKY_RELU or RLGPU_ACT_RELU");
    RLGPU_REQUIRE(cfg.optimizer == RLGPU_OPT_ADAMW || cfg.optimizer == RLGPU_OPT_ADAM,
                  "Learner: optimizer must be RLGPU_OPT_ADAMW or RLGPU_OPT_ADAM");
    pc.layer_norm = 1;
    pc.leaky_slope = cfg.activation == RLGPU_ACT_RELU ? 0.f : 0.01f;
    pc.policy_lr = cfg.policy_lr;
    pc.critic_lr = cfg.critic_lr;
    pc.beta1 = 0.9f;
    pc.beta2 = 0.999f;
    pc.eps = 1e-8f;
    pc.weight_decay = cfg.optimizer == RLGPU_OPT_ADAM ? 0.f : 1e-2f;  // Adam == AdamW without decoupled decay
    pc.clip_range = cfg.clip_range;
    pc.entropy_scale = cfg.entropy_scale;
    pc.max_grad_norm = 0.5f;
    const int64_t TP = (int64_t)T * P;
    // minibatch rows: the rollout's T * P caps them in mode 0; complete-trajectory batches can be larger
    const int64_t rowsCap = cfg.experience_mode == RLGPU_EXP_TRAJECTORIES ? (int64_t)cfg.mini_batch_size : TP;
    pc.max_rows = (int32_t)std::max<int64_t>(std::min<int64_t>(cfg.mini_batch_size, rowsCap), std::min<int64_t>(P, 65536));
    pc.seed = cfg.seed;
    pc.sample_row_offset = (int64_t)cfg.rank * P;  // rank r's players are players [r P, (r + 1) P) of the job
    pc.train_gemm = cfg.train_gemm;
    pc.infer_fp16 = cfg.infer_fp16;
    ppo_ = new PPOLearnerGPU(pc, s_);
    if (hasColl_) {  // identical initial weights on every rank: rank 0's (sum of zeros elsewhere)
        float* params = nullptr;
        float* g = nullptr;
        int64_t n = 0;
        RlgpuCheck(rlgpu_ppo_buffers(ppo_->handle(), &params, &g, &n), "buffers");
        if (cfg.rank != 0) hipCheck(hipMemsetAsync(params, 0, n * sizeof(float), s_), "broadcast");
        hipCheck(hipStreamSynchronize(s_), "sync");
        if (coll_.allreduce_sum_f32(coll_.user, params, n) != 0)
            throw rlgpu::Error(RLGPU_ERR_STATE, "Learner: parameter broadcast failed");
        RlgpuCheck(rlgpu_ppo_refresh_half(ppo_->handle(), s_), "refresh half");
    }
    if (trajMode()) {  // the reference's experience scheduling (RLGPU_EXP_TRAJECTORIES)
        RLGPU_REQUIRE(ec.max_episode_steps > 0, "Learner: experience_mode 1 needs max_episode_duration > 0");
        TrajectoryStore& J = traj;
        J.maxLen = ec.max_episode_steps;
        // every rank collects its share of the iteration's complete-trajectory steps
        const int64_t total = cfg.ts_per_itr > 0 ? cfg.ts_per_itr : (int64_t)T * P * cfg.world;
        J.tsPerItr = (total + cfg.world - 1) / cfg.world;
        const int64_t perStep = P;  // steps per env step (all players tracked at most)
        J.Tmax = cfg.experience_capacity > 0 ? cfg.experience_capacity
                                              : (int)(J.maxLen + 2 * ((J.tsPerItr + perStep - 1) / perStep) + 64);
        RLGPU_REQUIRE(J.Tmax > J.maxLen + 1, "Learner: experience_capacity must exceed the max episode length + 1");
        exp_.Allocate(J.Tmax, P, W, false);
        J.start = Alloc<int32_t>(P);
        J.len = Alloc<int32_t>(P);
        J.trnew = Alloc<int32_t>(P);
        J.counters = Alloc<int64_t>(lk::kTcCount);
        hipCheck(hipMemset(J.start, 0, (size_t)P * 4), "traj start");
        hipCheck(hipMemset(J.len, 0, (size_t)P * 4), "traj len");
        hipCheck(hipHostMalloc((void**)&J.hcounters, lk::kTcCount * sizeof(int64_t)), "pinned counters");
        if (K_ > 1) J.truncStage = Alloc<float>((size_t)P * W);
        const int64_t rc = 4 * (int64_t)P;
        for (auto* a : {&J.rp, &J.rstart, &J.rlen, &J.rcode, &J.rtidx}) a->Reserve(rc, s_);
        J.roff.Reserve(rc, s_);
        J.truncObs.Reserve(4 * (int64_t)P * W, s_);
    } else {
        exp_.Allocate(T, P, W);
    }
    // rollout row 0 = the env's initial obs (stacked: the first frame repeated) / masks
    const rlgpu_envset_buffers& st = env_->state();
    if (K_ > 1) {
        hist_ = Alloc<float>((size_t)(K_ - 1) * P * OBS);
        lk::stack_frames(st.obs, nullptr, nullptr, hist_, K_, P, OBS, exp_.v.obs, nullptr, s_);
    } else {
        hipCheck(hipMemcpyAsync(exp_.v.obs, st.obs, (size_t)P * OBS * 4, hipMemcpyDeviceToDevice, s_), "obs0");
    }
    hipCheck(hipMemcpyAsync(exp_.v.masks, st.action_masks, (size_t)P * ACT, hipMemcpyDeviceToDevice, s_), "masks0");
    // self-play team masks (team of player p is p % 2)
    std::vector<uint8_t> team(P);
    for (int k = 0; k < 2; k++) {
        oldRows_[k] = Alloc<uint8_t>(P);
        for (int p = 0; p < P; p++) team[p] = (uint8_t)(p % 2 == k);
        hipCheck(hipMemcpy(oldRows_[k], team.data(), P, hipMemcpyHostToDevice), "old rows");
    }
    trainRows_ = Alloc<int32_t>((size_t)TP / 2 + 1);
    perm_ = Alloc<int32_t>(TP);
    permRows_ = Alloc<int32_t>(TP);
    badv_ = Alloc<float>(TP);
    permCap_ = TP;
    truncRows_ = Alloc<int32_t>(TP);
    truncCount_ = Alloc<int32_t>(1);
    selBytes_ = lk::select_trunc_scratch_bytes(TP);
    selScratch_ = Alloc<char>(selBytes_);
    sampleIdx_ = Alloc<int64_t>((size_t)std::max(1, cfg.return_samples));
    samples_ = Alloc<float>((size_t)std::max(1, cfg.return_samples));
    ends_ = Alloc<int32_t>(P);
    hostEnds_.assign(P, -1);
    mom_ = (double*)Alloc<char>(4 * sizeof(double) + lk::moments_scratch_bytes());
    clipSums_ = Alloc<float>(2);
    hipCheck(hipStreamSynchronize(s_), "Learner init");
}

Learner::~Learner() {
    if (s_) (void)hipStreamSynchronize(s_);
    for (auto s : gs_) {
        (void)hipStreamSynchronize(s);
        (void)hipStreamDestroy(s);
    }
    for (auto e : gsEnd_) (void)hipEventDestroy(e);
    if (gsStart_) (void)hipEventDestroy(gsStart_);
    for (auto e : ev_) (void)hipEventDestroy(e);
    for (void* p : allocs_) (void)hipFree(p);
    if (truncObsC_) (void)hipFree(truncObsC_);
    if (truncValC_) (void)hipFree(truncValC_);
    if (traj.hcounters) (void)hipHostFree(traj.hcounters);
    for (auto* a : {&traj.rp, &traj.rstart, &traj.rlen, &traj.rcode, &traj.rtidx, &traj.cActs}) a->Free();
    traj.roff.Free();
    for (auto* a : {&traj.truncObs, &traj.truncVals, &traj.cObs, &traj.cLogp, &traj.cRews, &traj.cVals, &traj.cAdv,
                    &traj.cTarget, &traj.cRet})
        a->Free();
    traj.cMasks.Free();
    traj.cTerms.Free();
    exp_.Free();
    delete ppo_;
    delete env_;
}

// Arena groups for the rollout collection: a launch lasts as long as its slowest workgroup, so with the
// arenas split into groups stepped (and inferred) on their own streams, one group's launch tail could overlap
// the other groups' work (tools/env_streams.py, env steps alone: 0.84 -> 0.75 ms per step of 4,096 arenas with 4
// groups).  In the Learner, with the inference between the steps, it measured slower (collection 139 -> 152 ms
// with 2 groups, 260 ms with 4: profiles/r05y_collect_groups.txt), so the default stays one launch per step.
// Each arena's step and each player's draw are the same as in one launch (the arenas' Philox streams and the
// sampler's rows are global), so the rollout is bit-identical.  Only for the fused inference kernel (no
// per-handle row buffers), without a step hook or stacked frames, and for whole workgroups of arenas.
int Learner::CollectGroups() const {
    const int want = cfg_.collect_groups > 0 ? cfg_.collect_groups : 1;  // automatic = one group (see below)
    if (want <= 1 || hook_ || K_ > 1 || trajMode() || !rlgpu_ppo_fused_infer(ppo_->handle(), 0)) return 1;
    if (cfg_.num_arenas % (4 * want) != 0) return 1;
    return want;
}

void Learner::CollectGrouped(int G) {
    const int T = exp_.T, P = exp_.P, W = exp_.W;
    const rlgpu_rollout_view& v = exp_.v;
    const uint8_t* old = oldTeam_ >= 0 ? oldRows_[oldTeam_] : nullptr;
    const int Na = cfg_.num_arenas / G, Pg = 4 * Na;
    if ((int)gs_.size() != G) {
        for (auto s : gs_) (void)hipStreamDestroy(s);
        for (auto e : gsEnd_) (void)hipEventDestroy(e);
        gs_.assign(G, nullptr);
        gsEnd_.assign(G, nullptr);
        for (int g = 0; g < G; g++) {
            hipCheck(hipStreamCreateWithFlags(&gs_[g], hipStreamNonBlocking), "group stream");
            hipCheck(hipEventCreateWithFlags(&gsEnd_[g], hipEventDisableTiming), "group event");
        }
        if (!gsStart_) hipCheck(hipEventCreateWithFlags(&gsStart_, hipEventDisableTiming), "group event");
    }
    if (envTiming_ && ev_.size() < (size_t)2 * T * G) {
        for (auto e : ev_) (void)hipEventDestroy(e);
        ev_.assign((size_t)2 * T * G, nullptr);
        for (auto& e : ev_) hipCheck(hipEventCreate(&e), "event");
    }
    hipCheck(hipEventRecord(gsStart_, s_), "group start");
    for (int g = 0; g < G; g++) hipCheck(hipStreamWaitEvent(gs_[g], gsStart_, 0), "group wait");
    rlgpu_ppo* ph = ppo_->handle();
    rlgpu_envset* eh = env_->handle();
    for (int t = 0; t < T; t++) {
        const size_t r = (size_t)t * P;
        for (int g = 0; g < G; g++) {  // group 0 first: it advances the StepCallback cadence (rlgpu_envset_step_range)
            const size_t p0 = (size_t)g * Pg, a = r + p0;
            RlgpuCheck(rlgpu_ppo_infer_actions_rows(ph, v.obs + a * W, v.masks + a * ACT, Pg, (int64_t)p0,
                                                    cfg_.deterministic != 0, (uint64_t)stats.rng_step,
                                                    old ? old + p0 : nullptr, v.actions + a, v.logp + a, gs_[g]),
                       "InferActions (group)");
            rlgpu_step_outputs o{v.obs + (a + P) * OBS, v.masks + (a + P) * ACT, v.rewards + a, v.terms + a,
                                 v.trunc_obs + a * OBS};
            if (envTiming_) hipCheck(hipEventRecord(ev_[2 * ((size_t)t * G + g)], gs_[g]), "event");
            RlgpuCheck(rlgpu_envset_step_range(eh, g * Na, Na, v.actions + a, 1, &o, gs_[g]), "EnvSet step (group)");
            if (envTiming_) hipCheck(hipEventRecord(ev_[2 * ((size_t)t * G + g) + 1], gs_[g]), "event");
        }
        stats.rng_step++;
    }
    for (int g = 0; g < G; g++) {
        hipCheck(hipEventRecord(gsEnd_[g], gs_[g]), "group end");
        hipCheck(hipStreamWaitEvent(s_, gsEnd_[g], 0), "group join");
    }
}

void Learner::Collect() {
    if (trajMode()) {
        CollectTrajectories();
        return;
    }
    if (const int G = CollectGroups(); G > 1) {
        collectGroupsUsed_ = G;
        CollectGrouped(G);
        return;
    }
    collectGroupsUsed_ = 1;
    const int T = exp_.T, P = exp_.P;
    const rlgpu_rollout_view& v = exp_.v;
    const uint8_t* old = oldTeam_ >= 0 ? oldRows_[oldTeam_] : nullptr;
    if (envTiming_ && ev_.size() < (size_t)2 * T) {
        for (auto e : ev_) (void)hipEventDestroy(e);
        ev_.assign(2 * T, nullptr);
        for (auto& e : ev_) hipCheck(hipEventCreate(&e), "event");
    }
    const int W = exp_.W;
    const rlgpu_envset_buffers& st = env_->state();
    for (int t = 0; t < T; t++) {
        const size_t r = (size_t)t * P;
        ppo_->InferActions(v.obs + r * W, v.masks + r * ACT, P, cfg_.deterministic != 0, (uint64_t)stats.rng_step,
                           v.actions + r, v.logp + r, old);
        stats.rng_step++;
        // the fused step appends straight into the rollout; stacked obs are assembled from the env's
        // own obs / pre-reset rows after it
        rlgpu_step_outputs o{K_ > 1 ? nullptr : v.obs + (r + P) * OBS, v.masks + (r + P) * ACT, v.rewards + r,
                             v.terms + r, K_ > 1 ? nullptr : v.trunc_obs + r * OBS};
        if (envTiming_) hipCheck(hipEventRecord(ev_[2 * t], s_), "event");
        StepEnv(v.actions + r, o);
        if (envTiming_) hipCheck(hipEventRecord(ev_[2 * t + 1], s_), "event");
        if (K_ > 1)
            lk::stack_frames(st.obs, st.trunc_obs, v.terms + r, hist_, K_, P, OBS, v.obs + (r + P) * W, v.trunc_obs + r * W,
                             s_);
    }
}

// One env step with the experience append.  Without a hook: the fused kernel (step, reset of terminated
// arenas, append).  With one (host plugins / a StepCallbackFn): the step without its reset, then the hook
// (phase 0: the post-step GameStates; it may rewrite the env's rewards / terminals -- EnvSet::StepSecondHalf's
// host plugins and Learner.cpp:796-797's callback), the merged codes / rewards / truncation rows, the reset of
// the arenas whose merged terminal is set (EnvSet::Reset at the next step's start, Learner.cpp:676), the
// hook's phase 1 (the plugins' Reset on the new states), then the post-reset obs / masks appended.  With no
// host change this is bit-identical to the fused step (same kickoff draws, same builders).
void Learner::StepEnv(const int32_t* d_actions, const rlgpu_step_outputs& o) {
    if (!hook_) {
        env_->Step(d_actions, &o);
        return;
    }
    rlgpu_envset* e = env_->handle();
    const rlgpu_envset_buffers& st = env_->state();
    const int P = st.num_players;
    rlgpu_step_outputs pre{nullptr, nullptr, nullptr, o.terminals, nullptr};
    RlgpuCheck(rlgpu_envset_step(e, d_actions, 0, &pre, s_), "EnvSet step (hooked)");
    hipCheck(hipStreamSynchronize(s_), "sync");
    if (hook_(hookUser_, RLGPU_HOOK_AFTER_STEP) != 0)
        throw rlgpu::Error(RLGPU_ERR_STATE, std::string("Learner: step hook failed: ") + rlgpu_last_error());
    lk::host_step_finish(st.terminals, o.terminals, st.rewards, o.rewards, st.obs, st.trunc_obs, o.trunc_obs, P, OBS, s_);
    RlgpuCheck(rlgpu_envset_reset(e, s_), "EnvSet reset (hooked)");
    hipCheck(hipStreamSynchronize(s_), "sync");
    if (hook_(hookUser_, RLGPU_HOOK_AFTER_RESET) != 0)
        throw rlgpu::Error(RLGPU_ERR_STATE, std::string("Learner: step hook failed: ") + rlgpu_last_error());
    if (o.obs) hipCheck(hipMemcpyAsync(o.obs, st.obs, (size_t)P * OBS * 4, hipMemcpyDeviceToDevice, s_), "obs append");
    if (o.masks) hipCheck(hipMemcpyAsync(o.masks, st.action_masks, (size_t)P * ACT, hipMemcpyDeviceToDevice, s_), "mask append");
}

void Learner::Consume() {
    if (trajMode()) {
        ConsumeTrajectories();
        return;
    }
    const int T = exp_.T, P = exp_.P;
    const int64_t TP = (int64_t)T * P;
    const rlgpu_rollout_view& v = exp_.v;
    ppo_->InferCritic(v.obs, TP + P, v.values);  // InferCriticBatched over obs[0..T]
    // truncation values only where a trajectory was truncated (code 2): Learner.cpp:944
    lk::select_trunc(v.terms, TP, selScratch_, selBytes_, truncRows_, truncCount_, s_);
    int32_t ntr = 0;
    hipCheck(hipMemcpyAsync(&ntr, truncCount_, sizeof(int32_t), hipMemcpyDeviceToHost, s_), "trunc count");
    hipCheck(hipStreamSynchronize(s_), "sync");
    if (ntr > 0) {
        if (ntr > truncCap_) {
            if (truncObsC_) (void)hipFree(truncObsC_);
            if (truncValC_) (void)hipFree(truncValC_);
            truncCap_ = std::max<int64_t>(ntr, 2 * truncCap_);
            hipCheck(hipMalloc((void**)&truncObsC_, (size_t)truncCap_ * exp_.W * 4), "trunc obs");
            hipCheck(hipMalloc((void**)&truncValC_, (size_t)truncCap_ * 4), "trunc vals");
        }
        lk::gather_rows(v.trunc_obs, exp_.W, truncRows_, ntr, truncObsC_, s_);
        ppo_->InferCritic(truncObsC_, ntr, truncValC_);
        lk::scatter_f32(truncValC_, truncRows_, ntr, v.trunc_vals, s_);
    }
    const float std_ = (float)returnStat.GetSTD();
    RlgpuCheck(rlgpu_gae_rollout(v.rewards, v.terms, v.values, v.trunc_vals, v.values + TP, T, P, cfg_.gamma,
                                 cfg_.gae_lambda, std_, cfg_.reward_clip_range, v.adv, v.target, v.ret, nullptr, s_),
               "GAE");
    // return-std Welford over randomly sampled returns (Learner.cpp:959-967).  The reference samples
    // combinedTraj, i.e. steps of finished trajectories only, whose returns run to the trajectory's
    // end; here only rows (t, p) with t <= the column's last trajectory end qualify (an unfinished
    // tail's return would be cut at T).  In an old-version iteration only the current policy's
    // players have trajectories.
    const int k = cfg_.return_samples;
    if (k <= 0) return;
    lk::last_ends(v.terms, T, P, ends_, s_);
    hipCheck(hipMemcpyAsync(hostEnds_.data(), ends_, (size_t)P * sizeof(int32_t), hipMemcpyDeviceToHost, s_), "ends");
    hipCheck(hipStreamSynchronize(s_), "sync");
    if (oldTeam_ >= 0)
        for (int p = oldTeam_; p < P; p += 2) hostEnds_[p] = -1;  // team of player p is p % 2
    if (!hasColl_) {
        std::vector<int64_t> idx(k);
        int32_t m = 0;
        RlgpuCheck(rlgpu_sample_finished_rows(cfg_.seed, 0, stats.iteration, hostEnds_.data(), P, k, idx.data(), &m),
                   "return samples");
        FeedReturnStat(v.ret, idx, m);
        return;
    }
    // Several ranks: the draws are made over the job's rows -- every rank's columns in rank order, as one
    // device holding all of them would number them -- with one rank-independent generator, so a job of any
    // world size feeds the WelfordStat the same returns in the same order.  Each rank fills the draws that
    // fall in its own columns; an fp64 all-reduce of the draw vector (zeros elsewhere, exact) hands every
    // rank all of them.
    const int world = cfg_.world;
    std::vector<float> mine((size_t)P), all((size_t)P * world);
    for (int p = 0; p < P; p++) mine[p] = (float)hostEnds_[p];  // exact: ends < 2^24
    if (coll_.allgather_f32(coll_.user, mine.data(), P, all.data()) != 0)
        throw rlgpu::Error(RLGPU_ERR_STATE, "Learner: trajectory-end all-gather failed");
    std::vector<int32_t> gends((size_t)P * world);
    for (size_t i = 0; i < gends.size(); i++) gends[i] = (int32_t)all[i];
    const int64_t GP = (int64_t)P * world;
    std::vector<int64_t> gidx(k), idx;
    std::vector<int32_t> slot;
    int32_t m = 0;
    RlgpuCheck(rlgpu_sample_finished_rows(cfg_.seed, 0, stats.iteration, gends.data(), (int32_t)GP, k, gidx.data(), &m),
               "return samples");
    for (int32_t i = 0; i < m; i++) {  // global row t * GP + gp -> this rank's row t * P + (gp - rank P)
        const int64_t t = gidx[i] / GP, gp = gidx[i] % GP;
        if (gp / P == cfg_.rank) {
            idx.push_back(t * P + (gp - (int64_t)cfg_.rank * P));
            slot.push_back(i);
        }
    }
    std::vector<float> hs(std::max<size_t>(idx.size(), 1));
    if (!idx.empty()) {
        hipCheck(hipMemcpyAsync(sampleIdx_, idx.data(), idx.size() * sizeof(int64_t), hipMemcpyHostToDevice, s_),
                 "sample idx");
        lk::gather_samples(v.ret, sampleIdx_, (int32_t)idx.size(), samples_, s_);
        hipCheck(hipMemcpyAsync(hs.data(), samples_, idx.size() * sizeof(float), hipMemcpyDeviceToHost, s_), "samples");
        hipCheck(hipStreamSynchronize(s_), "sync");
    }
    std::vector<double> draw((size_t)std::max(m, 1), 0.0);
    for (size_t j = 0; j < idx.size(); j++) draw[slot[j]] = (double)hs[j];
    if (m > 0 && coll_.allreduce_sum_f64(coll_.user, draw.data(), m) != 0)
        throw rlgpu::Error(RLGPU_ERR_STATE, "Learner: return-sample all-reduce failed");
    std::vector<float> got((size_t)std::max(m, 1));
    for (int32_t i = 0; i < m; i++) got[i] = (float)draw[i];
    returnStat.Increment(got.data(), m);
}

// WelfordStat::Increment over the sampled returns (Learner.cpp:959-967); ranks may hold different
// sample counts, so the samples are all-gathered as (count, k padded samples) and every rank adds all
void Learner::FeedReturnStat(const float* d_ret, const std::vector<int64_t>& idx, int32_t m) {
    const int k = cfg_.return_samples;
    std::vector<float> hs((size_t)std::max(m, 1));
    if (m > 0) {
        hipCheck(hipMemcpyAsync(sampleIdx_, idx.data(), m * sizeof(int64_t), hipMemcpyHostToDevice, s_), "sample idx");
        lk::gather_samples(d_ret, sampleIdx_, m, samples_, s_);
        hipCheck(hipMemcpyAsync(hs.data(), samples_, m * sizeof(float), hipMemcpyDeviceToHost, s_), "samples");
        hipCheck(hipStreamSynchronize(s_), "sync");
    }
    if (hasColl_) {  // ranks may hold different sample counts: gather (count, k padded samples)
        std::vector<float> mine((size_t)k + 1, 0.f), all((size_t)(k + 1) * cfg_.world);
        mine[0] = (float)m;
        std::copy(hs.begin(), hs.begin() + m, mine.begin() + 1);
        if (coll_.allgather_f32(coll_.user, mine.data(), k + 1, all.data()) != 0)
            throw rlgpu::Error(RLGPU_ERR_STATE, "Learner: return-sample all-gather failed");
        for (int r = 0; r < cfg_.world; r++) {
            const float* blk = all.data() + (size_t)r * (k + 1);
            returnStat.Increment(blk + 1, (int64_t)blk[0]);
        }
    } else {
        returnStat.Increment(hs.data(), m);
    }
}

void Learner::AllReduceGrads(int epoch, int batch) {
    if (!hasColl_ && !gradHook_) return;
    hipCheck(hipStreamSynchronize(s_), "sync");
    if (hasColl_ && coll_.allreduce_sum_f32(coll_.user, ppo_->grads(), ppo_->num_params()) != 0)
        throw rlgpu::Error(RLGPU_ERR_STATE, "Learner: gradient all-reduce failed");
    if (gradHook_ && gradHook_(gradHookUser_, ppo_->grads(), ppo_->num_params(), epoch, batch) != 0)
        throw rlgpu::Error(RLGPU_ERR_STATE, "Learner: the gradient hook failed");
}

// batch advantage normalisation (PPOLearner.cpp:360-371): (mean, unbiased std) of the batch's
// advantages, global over ranks in fp64
void Learner::BatchAdvantageStats(const float* d_adv, const int32_t* d_idx, int64_t n) {
    if (!hasColl_) {
        if (d_idx) {
            NeedLearnRows(n, "the batch-advantage gather");
            lk::gather_f32(d_adv, d_idx, n, badv_, s_);
            ppo_->AdvantageStats(badv_, n);
        } else {
            ppo_->AdvantageStats(d_adv, n);
        }
        return;
    }
    lk::moments_f64(d_adv, d_idx, n, mom_ + 4, mom_, s_);
    double m[3];
    hipCheck(hipMemcpyAsync(m, mom_, sizeof(m), hipMemcpyDeviceToHost, s_), "moments");
    hipCheck(hipStreamSynchronize(s_), "sync");
    if (coll_.allreduce_sum_f64(coll_.user, m, 3) != 0)
        throw rlgpu::Error(RLGPU_ERR_STATE, "Learner: advantage-moment all-reduce failed");
    float st[2];
    MomentsMeanStd(m, st);
    hipCheck(hipMemcpyAsync(ppo_->adv_stats(), st, sizeof(st), hipMemcpyHostToDevice, s_), "adv stats");
    hipCheck(hipStreamSynchronize(s_), "sync");
}

// Every consumer of the per-row learn scratch checks its row count against the capacity first: an
// undersized buffer is an RLGPU_ERR_INVALID_ARG naming the consumer, never a device fault.
void Learner::NeedLearnRows(int64_t n, const char* what) const {
    if (n > permCap_)
        throw rlgpu::Error(RLGPU_ERR_INVALID_ARG, std::string("Learner: ") + what + " needs " + std::to_string(n) +
                                                      " rows of learn scratch, " + std::to_string(permCap_) + " reserved");
}

// the per-row learn scratch (shuffle, row selection, batch advantages) for M rows
void Learner::ReserveLearnRows(int64_t M) {
    if (M <= permCap_) return;
    const int64_t cap = std::max<int64_t>(M, permCap_ + permCap_ / 2);
    hipCheck(hipStreamSynchronize(s_), "sync");
    for (void* p : {(void*)perm_, (void*)permRows_, (void*)badv_}) Release(p);
    perm_ = Alloc<int32_t>(cap);
    permRows_ = Alloc<int32_t>(cap);
    badv_ = Alloc<float>(cap);
    permCap_ = cap;
}

void Learner::Learn() {
    const int T = exp_.T, P = exp_.P;
    rlgpu_rollout_view v = exp_.v;
    // the trajectory mode trains the combined batch (complete trajectories of the current policy's
    // players only, so no row selection)
    const bool rows = oldTeam_ >= 0 && !trajMode();
    int64_t M = rows ? (int64_t)T * (P / 2) : (int64_t)T * P;
    if (trajMode()) {
        M = traj.nrows;
        v.obs = traj.cObs.p;
        v.masks = traj.cMasks.p;
        v.actions = traj.cActs.p;
        v.logp = traj.cLogp.p;
        v.adv = traj.cAdv.p;
        v.target = traj.cTarget.p;
        if (M <= 0 && !hasColl_) return;  // with ranks, an empty one still joins every collective
    }
    ReserveLearnRows(M);
    int64_t globalM = M * cfg_.world;
    if (trajMode() && hasColl_) {  // ranks hold different complete-trajectory counts: the true total
        double m = (double)M;
        if (coll_.allreduce_sum_f64(coll_.user, &m, 1) != 0)
            throw rlgpu::Error(RLGPU_ERR_STATE, "Learner: batch-size all-reduce failed");
        globalM = (int64_t)m;
    }
    const int64_t batch = cfg_.batch_size > 0 ? cfg_.batch_size : globalM;
    const int64_t localBatch = cfg_.batch_size > 0 ? std::max<int64_t>(1, cfg_.batch_size / cfg_.world) : M;
    // with several ranks in the trajectory mode the ranks hold different row counts, yet every rank
    // must take the same optimizer steps (one all-reduce each): the batches are the reference's
    // GetAllBatchesShuffled split of the global combined batch (ExperienceBuffer.cpp:117-162), and
    // rank-local batch i is the same fraction [g0 / globalM, g1 / globalM) of this rank's rows
    std::vector<std::pair<int64_t, int64_t>> trajRanges;
    if (trajMode() && hasColl_) {
        for (auto [g0, g1] : BatchRanges(globalM, batch, cfg_.overbatching != 0))
            trajRanges.emplace_back(globalM ? g0 * M / globalM : 0, globalM ? g1 * M / globalM : 0);
        if (trajRanges.empty()) trajRanges.emplace_back(0, 0);
    }
    if (rows) lk::train_rows(T, P, 1 - oldTeam_, trainRows_, s_);
    for (int epoch = 0; epoch < cfg_.epochs; epoch++) {
        NeedLearnRows(M, "the shuffle");
        RlgpuCheck(rlgpu_permutation(M, cfg_.seed + (uint64_t)cfg_.rank, (uint64_t)(stats.iteration * cfg_.epochs + epoch),
                                     perm_, s_),
                   "shuffle");
        const int32_t* order = perm_;
        if (rows) {
            NeedLearnRows(M, "the team row selection");
            if (M > (int64_t)T * (P / 2)) throw rlgpu::Error(RLGPU_ERR_INVALID_ARG, "Learner: team rows exceed T * P / 2");
            lk::compose(trainRows_, perm_, M, permRows_, s_);
            order = permRows_;
        }
        const auto ranges = trajMode() && hasColl_ ? trajRanges : BatchRanges(M, localBatch, cfg_.overbatching != 0);
        int bi = 0;
        for (auto [b0, b1] : ranges) {
            const bool whole = !rows && b0 == 0 && b1 == M;
            BatchAdvantageStats(v.adv, whole ? nullptr : order + b0, b1 - b0);
            for (int64_t s0 = b0; s0 < b1; s0 += cfg_.mini_batch_size) {
                const int n = (int)std::min<int64_t>(cfg_.mini_batch_size, b1 - s0);
                ppo_->Minibatch(v.obs, v.masks, v.actions, v.logp, v.adv, v.target, order, s0, n, batch);
            }
            AllReduceGrads(epoch, bi++);  // RCCL over xGMI (via the collective), before clip_grad_norm_
            ppo_->OptimizerStep();
        }
    }
}

void Learner::FinishIteration() {
    const int T = exp_.T, P = exp_.P;
    const rlgpu_rollout_view& v = exp_.v;
    const size_t W = (size_t)exp_.W;
    const int64_t realPlayers = oldTeam_ < 0 ? P : P / 2;  // numRealPlayers (Learner.cpp:629)
    stats.iteration++;
    if (trajMode()) {  // stepsCollected (Learner.cpp:651): every step of the iteration, finished or not
        stats.total_steps += (int64_t)traj.steps * realPlayers * cfg_.world;
        return;
    }
    hipCheck(hipMemcpyAsync(v.obs, v.obs + (size_t)T * P * W, (size_t)P * W * 4, hipMemcpyDeviceToDevice, s_), "obs");
    hipCheck(hipMemcpyAsync(v.masks, v.masks + (size_t)T * P * ACT, (size_t)P * ACT, hipMemcpyDeviceToDevice, s_), "masks");
    stats.total_steps += (int64_t)T * realPlayers * cfg_.world;
}

// ---- RLGPU_EXP_TRAJECTORIES: the reference's trajectory loop (Learner.cpp:643-861)
void Learner::CollectTrajectories() {
    TrajectoryStore& J = traj;
    const int P = exp_.P, W = exp_.W, Tm = J.Tmax;
    const rlgpu_rollout_view& v = exp_.v;
    const rlgpu_envset_buffers& st = env_->state();
    // the players of the current policy; a team that acted with an old version last iteration starts
    // fresh trajectories (the reference freezes them and resumes them later across the gap)
    const uint8_t* track = oldTeam_ >= 0 ? oldRows_[1 - oldTeam_] : nullptr;
    if (J.lastOldTeam >= 0) lk::traj_restart(oldRows_[J.lastOldTeam], P, (int)(J.step % Tm), J.start, J.len, s_);
    J.lastOldTeam = oldTeam_;
    const uint8_t* old = oldTeam_ >= 0 ? oldRows_[oldTeam_] : nullptr;
    hipCheck(hipMemsetAsync(J.counters, 0, lk::kTcCount * sizeof(int64_t), s_), "traj counters");
    J.firstStep = J.step;
    J.steps = 0;
    J.nrec = J.ntrunc = J.nrows = 0;
    for (;;) {
        // room for this step's records and truncation rows (at most one per player)
        const int64_t need = std::max(J.nrec, J.ntrunc) + P;
        if (J.rp.cap < need) {
            for (auto* a : {&J.rp, &J.rstart, &J.rlen, &J.rcode, &J.rtidx}) a->Reserve(2 * need, s_, true);
            J.roff.Reserve(2 * need, s_, true);
        }
        J.truncObs.Reserve((J.ntrunc + P) * (int64_t)W, s_, true);
        const int r = (int)(J.step % Tm), rn = (int)((J.step + 1) % Tm);
        const size_t row = (size_t)r * P, rown = (size_t)rn * P;
        ppo_->InferActions(v.obs + row * W, v.masks + row * ACT, P, cfg_.deterministic != 0, (uint64_t)stats.rng_step,
                           v.actions + row, v.logp + row, old);
        stats.rng_step++;
        rlgpu_step_outputs o{K_ > 1 ? nullptr : v.obs + rown * OBS, v.masks + rown * ACT, v.rewards + row, v.terms + row,
                             nullptr};
        StepEnv(v.actions + row, o);
        if (K_ > 1)
            lk::stack_frames(st.obs, st.trunc_obs, v.terms + row, hist_, K_, P, OBS, v.obs + rown * W, J.truncStage, s_);
        lk::TrajRecs R{J.rp.p, J.rstart.p, J.rlen.p, J.rcode.p, J.rtidx.p, J.roff.p};
        lk::traj_step(v.terms + row, r, Tm, track, P, J.start, J.len, R, J.counters, J.trnew, s_);
        lk::traj_trunc_copy(K_ > 1 ? J.truncStage : st.trunc_obs, W, J.counters, J.trnew, J.truncObs.p, s_);
        J.step++;
        J.steps++;
        hipCheck(hipMemcpyAsync(J.hcounters, J.counters, lk::kTcCount * sizeof(int64_t), hipMemcpyDeviceToHost, s_),
                 "traj counters");
        hipCheck(hipStreamSynchronize(s_), "sync");
        J.nrec = J.hcounters[lk::kTcRecs];
        J.ntrunc = J.hcounters[lk::kTcTruncs];
        J.nrows = J.hcounters[lk::kTcSteps];
        if (J.nrows >= J.tsPerItr) break;  // combinedTraj.Length() >= tsPerItr (Learner.cpp:651)
        // the store holds maxLen steps of every live trajectory plus this iteration's: stop before the
        // next step could overwrite a live one
        if (J.steps + J.maxLen + 2 >= Tm) break;
    }
}

void Learner::ConsumeTrajectories() {
    TrajectoryStore& J = traj;
    const int P = exp_.P, W = exp_.W;
    const rlgpu_rollout_view& v = exp_.v;
    const int64_t M = J.nrows, K = J.nrec, ntr = J.ntrunc;
    J.cObs.Reserve(std::max<int64_t>(M, 1) * W, s_);
    J.cMasks.Reserve(std::max<int64_t>(M, 1) * ACT, s_);
    for (auto* a : {&J.cLogp, &J.cRews, &J.cVals, &J.cAdv, &J.cTarget, &J.cRet}) a->Reserve(std::max<int64_t>(M, 1), s_);
    J.cActs.Reserve(std::max<int64_t>(M, 1), s_);
    J.cTerms.Reserve(std::max<int64_t>(M, 1), s_);
    J.truncVals.Reserve(std::max<int64_t>(ntr, 1), s_);
    if (M == 0) {
        // a rank without finished rows still joins the return-sample all-gather the others make
        if (hasColl_ && cfg_.return_samples > 0) FeedReturnStat(J.cRet.p, {}, 0);
        return;
    }
    // combinedTraj -> tensors (Learner.cpp:863-912): the complete trajectories in the order they ended
    lk::TrajRecs R{J.rp.p, J.rstart.p, J.rlen.p, J.rcode.p, J.rtidx.p, J.roff.p};
    lk::traj_gather(R, K, J.Tmax, P, W, ACT, v.obs, v.masks, v.actions, v.logp, v.rewards, v.terms, J.cObs.p, J.cMasks.p,
                    J.cActs.p, J.cLogp.p, J.cRews.p, J.cTerms.p, s_);
    ppo_->InferCritic(J.cObs.p, M, J.cVals.p);  // InferCriticBatched (Learner.cpp:936)
    if (ntr > 0) ppo_->InferCritic(J.truncObs.p, ntr, J.truncVals.p);  // nextTruncStates (:939-941)
    const float std_ = (float)returnStat.GetSTD();
    hipCheck(hipMemsetAsync(clipSums_, 0, 2 * sizeof(float), s_), "clip sums");
    RlgpuCheck(rlgpu_gae_segments(J.cRews.p, J.cTerms.p, J.cVals.p, ntr > 0 ? J.truncVals.p : nullptr, J.roff.p, J.rlen.p,
                                  J.rtidx.p, K, cfg_.gamma, cfg_.gae_lambda, std_, cfg_.reward_clip_range, J.cAdv.p,
                                  J.cTarget.p, J.cRet.p, clipSums_, s_),
               "GAE");
    // return-std samples: torch::randint over every combined return (Learner.cpp:959-967)
    const int k = cfg_.return_samples;
    if (k <= 0) return;
    const int32_t m = (int32_t)std::min<int64_t>(k, M);
    std::vector<int64_t> idx((size_t)std::max(m, 1));
    if (m > 0) RlgpuCheck(rlgpu_sample_indices(cfg_.seed, cfg_.rank, stats.iteration, M, m, idx.data()), "return samples");
    FeedReturnStat(J.cRet.p, idx, m);
}

rlgpu_learner_report Learner::Iterate() {
    rlgpu_learner_report r{};
    auto t0 = clk::now();
    Collect();
    auto t0i = clk::now();
    hipCheck(hipStreamSynchronize(s_), "sync");
    auto t1 = clk::now();
    r.collect_issue_s = secs(t0, t0i);
    Consume();
    hipCheck(hipStreamSynchronize(s_), "sync");
    auto t2 = clk::now();
    Learn();
    FinishIteration();
    auto t2i = clk::now();
    hipCheck(hipStreamSynchronize(s_), "sync");
    auto t3 = clk::now();
    r.learn_issue_s = secs(t2, t2i);
    r.collect_s = secs(t0, t1);
    r.consume_s = secs(t1, t2);
    r.learn_s = secs(t2, t3);
    r.env_steps = (int64_t)(trajMode() ? traj.steps : exp_.T) * cfg_.num_arenas;
    r.env_launch_arenas = cfg_.num_arenas / std::max(1, collectGroupsUsed_);
    if (envTiming_ && !ev_.empty()) {
        double ms = 0;
        // per env launch: T per group (the trajectory mode records no per-step events)
        const int nt = trajMode() ? 0 : exp_.T * std::max(1, collectGroupsUsed_);
        std::vector<float> each(nt);
        for (int t = 0; t < nt; t++) {
            float x = 0;
            hipCheck(hipEventElapsedTime(&x, ev_[2 * t], ev_[2 * t + 1]), "elapsed");
            ms += x;
            each[t] = x;
        }
        r.env_kernel_ms = nt ? ms / nt : 0.0;
        if (nt) {
            std::sort(each.begin(), each.end());
            r.env_kernel_min_ms = each.front();
            r.env_kernel_max_ms = each.back();
            r.env_kernel_median_ms = (nt & 1) ? each[nt / 2] : 0.5 * ((double)each[nt / 2 - 1] + each[nt / 2]);
        }
    }
    return r;
}

void Learner::Start(int64_t iterations) {
    for (int64_t i = 0; i < iterations; i++) Iterate();
}

}  // namespace GGL

// ------------------------------------------------------------------ C ABI
struct rlgpu_learner {
    GGL::Learner* L = nullptr;
};

extern "C" int rlgpu_learner_default_config(rlgpu_learner_config* c) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(c, "null config");
        std::memset(c, 0, sizeof(*c));
        c->num_arenas = 4096;  // C2 (BASELINE.json configs[1])
        c->tick_skip = 8;      // ExampleMain.cpp:356-358
        c->action_delay = 7;
        c->seed = 123;
        c->max_episode_duration = 300.f;
        c->rollout_len = 128;
        c->epochs = 2;  // ExampleMain.cpp:404-430
        c->mini_batch_size = 50000;
        c->batch_size = 0;
        c->overbatching = 1;
        c->gamma = 0.99f;
        c->gae_lambda = 0.95f;
        c->clip_range = 0.2f;
        c->entropy_scale = 0.035f;
        c->policy_lr = 2.5e-4f;
        c->critic_lr = 2.5e-4f;
        c->reward_clip_range = 200.f;
        c->return_samples = 150;
        c->policy_layers[0] = c->policy_layers[1] = 512;
        c->n_policy_layers = 2;
        c->critic_layers[0] = c->critic_layers[1] = 512;
        c->n_critic_layers = 2;
        c->train_gemm = RLGPU_GEMM_F16X3;  // fp32-class training GEMMs at half the MFMAs of F32X6
        c->rank = 0;
        c->world = 1;
    });
}

extern "C" int rlgpu_learner_create(const rlgpu_learner_config* cfg, const rlgpu_collective* coll, void* stream,
                                    rlgpu_learner** out) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(cfg && out, "rlgpu_learner_create: null argument");
        auto* h = new rlgpu_learner();
        try {
            h->L = new GGL::Learner(*cfg, coll, rlgpu::as_stream(stream));
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
    });
}

extern "C" int rlgpu_learner_destroy(rlgpu_learner* h) {
    return rlgpu::guarded([&] {
        if (!h) return;
        delete h->L;
        delete h;
    });
}

#define RLGPU_LEARNER(h) RLGPU_REQUIRE((h) && (h)->L, "null learner handle")

extern "C" int rlgpu_learner_handles(rlgpu_learner* h, rlgpu_envset** env, rlgpu_ppo** ppo) {
    return rlgpu::guarded([&] {
        RLGPU_LEARNER(h);
        if (env) *env = h->L->env().handle();
        if (ppo) *ppo = h->L->ppo().handle();
    });
}
extern "C" int rlgpu_learner_rollout(rlgpu_learner* h, rlgpu_rollout_view* out) {
    return rlgpu::guarded([&] {
        RLGPU_LEARNER(h);
        RLGPU_REQUIRE(out, "null output");
        *out = h->L->exp().v;
    });
}
extern "C" int rlgpu_learner_batch(rlgpu_learner* h, rlgpu_batch_view* out) {
    return rlgpu::guarded([&] {
        RLGPU_LEARNER(h);
        RLGPU_REQUIRE(out, "null output");
        RLGPU_REQUIRE(h->L->config().experience_mode == RLGPU_EXP_TRAJECTORIES,
                      "rlgpu_learner_batch: the learner runs the rollout experience mode");
        const GGL::TrajectoryStore& J = h->L->traj;
        rlgpu_batch_view& b = *out;
        b.obs = J.cObs.p;
        b.masks = J.cMasks.p;
        b.actions = J.cActs.p;
        b.logp = J.cLogp.p;
        b.rewards = J.cRews.p;
        b.terms = J.cTerms.p;
        b.values = J.cVals.p;
        b.adv = J.cAdv.p;
        b.target = J.cTarget.p;
        b.ret = J.cRet.p;
        b.num_rows = J.nrows;
        b.trunc_obs = J.truncObs.p;
        b.trunc_vals = J.truncVals.p;
        b.num_truncs = J.ntrunc;
        b.seg_player = J.rp.p;
        b.seg_start = J.rstart.p;
        b.seg_len = J.rlen.p;
        b.seg_code = J.rcode.p;
        b.seg_tidx = J.rtidx.p;
        b.seg_off = J.roff.p;
        b.num_segments = J.nrec;
        b.store_rows = J.Tmax;
        b.steps = J.steps;
        b.first_step = J.firstStep;
    });
}

extern "C" int rlgpu_learner_iterate(rlgpu_learner* h, rlgpu_learner_report* rep) {
    return rlgpu::guarded([&] {
        RLGPU_LEARNER(h);
        rlgpu_learner_report r = h->L->Iterate();
        if (rep) *rep = r;
    });
}
extern "C" int rlgpu_learner_collect(rlgpu_learner* h) {
    return rlgpu::guarded([&] {
        RLGPU_LEARNER(h);
        h->L->Collect();
    });
}
extern "C" int rlgpu_learner_consume(rlgpu_learner* h) {
    return rlgpu::guarded([&] {
        RLGPU_LEARNER(h);
        h->L->Consume();
    });
}
extern "C" int rlgpu_learner_learn(rlgpu_learner* h) {
    return rlgpu::guarded([&] {
        RLGPU_LEARNER(h);
        h->L->Learn();
    });
}
extern "C" int rlgpu_learner_finish_iteration(rlgpu_learner* h) {
    return rlgpu::guarded([&] {
        RLGPU_LEARNER(h);
        h->L->FinishIteration();
    });
}
extern "C" int rlgpu_learner_set_old_team(rlgpu_learner* h, int32_t team) {
    return rlgpu::guarded([&] {
        RLGPU_LEARNER(h);
        RLGPU_REQUIRE(team >= -1 && team <= 1, "team must be -1, 0 or 1");
        h->L->SetOldTeam(team);
    });
}
extern "C" int rlgpu_learner_get_stats(rlgpu_learner* h, rlgpu_learner_stats* out) {
    return rlgpu::guarded([&] {
        RLGPU_LEARNER(h);
        RLGPU_REQUIRE(out, "null output");
        *out = h->L->stats;
        out->return_n = h->L->returnStat.count;
        out->return_mean = h->L->returnStat.mean;
        out->return_m2 = h->L->returnStat.m2;
    });
}
extern "C" int rlgpu_learner_set_stats(rlgpu_learner* h, const rlgpu_learner_stats* in) {
    return rlgpu::guarded([&] {
        RLGPU_LEARNER(h);
        RLGPU_REQUIRE(in && in->return_n >= 0 && in->iteration >= 0, "bad stats");
        h->L->stats = *in;
        h->L->returnStat.count = in->return_n;
        h->L->returnStat.mean = in->return_mean;
        h->L->returnStat.m2 = in->return_m2;
    });
}
extern "C" int rlgpu_learner_step_metrics(rlgpu_learner* h, double* h_total, uint64_t* h_count, int32_t reset) {
    return rlgpu::guarded([&] {
        RLGPU_LEARNER(h);
        RLGPU_CHECK_HIP(hipDeviceSynchronize());
        RLGC::RlgpuCheck(rlgpu_envset_step_metrics(h->L->env().handle(), h_total, h_count, reset, nullptr), "step metrics");
    });
}

extern "C" int rlgpu_learner_metrics(rlgpu_learner* h, float* h_out, int64_t* count, int32_t reset) {
    return rlgpu::guarded([&] {
        RLGPU_LEARNER(h);
        GGL::PPOLearnerGPU& p = h->L->ppo();
        hipStream_t s = nullptr;
        if (h_out) {
            RLGPU_CHECK_HIP(hipDeviceSynchronize());
            RLGPU_CHECK_HIP(hipMemcpy(h_out, p.metrics(), RLGPU_NUM_METRICS * sizeof(float), hipMemcpyDeviceToHost));
        }
        if (count) *count = p.minibatches;
        if (reset) {
            RLGPU_CHECK_HIP(hipMemsetAsync(p.metrics(), 0, RLGPU_NUM_METRICS * sizeof(float), s));
            RLGPU_CHECK_HIP(hipDeviceSynchronize());
            p.minibatches = 0;
        }
    });
}

extern "C" int rlgpu_moments_mean_std(const double* m3, float* out2) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(m3 && out2 && m3[2] > 1, "rlgpu_moments_mean_std: bad argument");
        GGL::MomentsMeanStd(m3, out2);
    });
}

extern "C" int rlgpu_learner_set_step_hook(rlgpu_learner* h, rlgpu_step_hook_fn fn, void* user) {
    return rlgpu::guarded([&] {
        RLGPU_LEARNER(h);
        h->L->SetStepHook(fn, user);
    });
}

extern "C" int rlgpu_learner_set_grad_hook(rlgpu_learner* h, rlgpu_grad_hook_fn fn, void* user) {
    return rlgpu::guarded([&] {
        RLGPU_LEARNER(h);
        h->L->SetGradHook(fn, user);
    });
}

extern "C" int rlgpu_learner_set_env_timing(rlgpu_learner* h, int32_t enable) {
    return rlgpu::guarded([&] {
        RLGPU_LEARNER(h);
        h->L->SetEnvTiming(enable != 0);
    });
}

extern "C" int64_t rlgpu_batch_ranges(int64_t exp_size, int64_t batch_size, int32_t overbatching, int64_t* out,
                                      int64_t max_ranges) {
    auto r = GGL::BatchRanges(exp_size, batch_size, overbatching != 0);
    for (int64_t i = 0; i < (int64_t)r.size() && i < max_ranges; i++) {
        out[2 * i] = r[i].first;
        out[2 * i + 1] = r[i].second;
    }
    return (int64_t)r.size();
}

extern "C" int rlgpu_welford_add(int64_t* count, double* mean, double* m2, const float* xs, int64_t n) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(count && mean && m2 && (xs || n == 0) && n >= 0, "rlgpu_welford_add: bad argument");
        GGL::WelfordStat w;
        w.count = *count;
        w.mean = *mean;
        w.m2 = *m2;
        w.Increment(xs, n);
        *count = w.count;
        *mean = w.mean;
        *m2 = w.m2;
    });
}

extern "C" double rlgpu_welford_std(int64_t count, double m2) {
    GGL::WelfordStat w;
    w.count = count;
    w.m2 = m2;
    return w.GetSTD();
}

extern "C" int rlgpu_sample_finished_rows(uint64_t seed, int32_t rank, int64_t iteration, const int32_t* ends,
                                          int32_t P, int32_t n, int64_t* out, int32_t* n_out) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(ends && out && n_out && n >= 0 && P > 0, "rlgpu_sample_finished_rows: bad argument");
        // cumulative eligible-row counts per column, then each draw j in [0, total) -> (column, t)
        std::vector<int64_t> cum((size_t)P + 1, 0);
        for (int32_t p = 0; p < P; p++) cum[p + 1] = cum[p] + (ends[p] >= 0 ? (int64_t)ends[p] + 1 : 0);
        const int64_t total = cum[P];
        const int32_t m = (int32_t)std::min<int64_t>(n, total);
        *n_out = m;
        if (m == 0) return;
        std::vector<int64_t> draws(m);
        RLGC::RlgpuCheck(rlgpu_sample_indices(seed, rank, iteration, total, m, draws.data()), "sample indices");
        for (int32_t i = 0; i < m; i++) {
            const int64_t j = draws[i];
            const int32_t p = (int32_t)(std::upper_bound(cum.begin(), cum.end(), j) - cum.begin()) - 1;
            out[i] = (j - cum[p]) * (int64_t)P + p;
        }
    });
}

extern "C" int rlgpu_sample_indices(uint64_t seed, int32_t rank, int64_t iteration, int64_t range, int32_t n,
                                    int64_t* out) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(out && n >= 0 && range > 0, "rlgpu_sample_indices: bad argument");
        const uint64_t key = splitmix64(seed ^ splitmix64(((uint64_t)(uint32_t)rank << 40) ^ (uint64_t)iteration));
        for (int32_t i = 0; i < n; i++) {
            const uint64_t x = splitmix64(key + (uint64_t)i);
            out[i] = (int64_t)(((unsigned __int128)x * (unsigned __int128)(uint64_t)range) >> 64);
        }
    });
}

extern "C" double rlgpu_host_uniform(uint64_t seed, uint64_t stream, uint64_t counter) {
    const uint64_t x = splitmix64(seed ^ splitmix64((stream << 48) ^ splitmix64(counter)));
    return (double)(x >> 11) * (1.0 / 9007199254740992.0);  // 53 bits
}
