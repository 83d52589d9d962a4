// example_main.cpp -- rlgpu_train: the reference's src/ExampleMain.cpp setup on the MI355X engine, written
// against the trainer facade (facade/GigaLearn.hpp: GGL::Learner(EnvCreateFn, LearnerConfig, StepCallbackFn),
// Start / Save / Load) with every plugin a device-registry class, plus the command-line knobs of a benchmark /
// multi-rank launcher.  It stands in for the reference's own ExampleMain.cpp, which is written against the same
// facade surface but is not compiled here (building against the reference's sources was
// refused by the environment).
//
// ExampleMain.cpp:128-226: the 2v2 arena, AdvancedObs, DefaultAction, the 13 weighted rewards, NoTouch(8) +
// ScoreLimit(3), KickoffState; :340-430: the LearnerConfig / PPOLearnerConfig.  The model topology is the one
// its log prints (run_out.log:25-28: shared head [384, 384], policy and critic [384] x 3); --c2-model selects
// BASELINE config C2's [512, 512] actor / critic without a shared head.  The StepCallback's metrics are the
// device's (rlgpu_learner_step_metrics), printed per iteration, so no GameState leaves the GPU.
//
// Checkpoints: --checkpoint-folder DIR makes the Learner Load the newest numbered checkpoint at start and Save
// at the end (and every --ts-per-save timesteps); --resave-to DIR2 loads DIR's newest checkpoint, saves it into
// DIR2 without training and exits (a lossless round trip: tests/test_trainer_facade.py).
//
// Multi-GPU: one process per GPU (--rank r --world N --rccl-id FILE): rank 0 writes RCCL's unique id to FILE,
// the other ranks read it, every rank trains its own arenas and the Learner's exchanges run over the native RCCL
// communicator (host/rccl_collective.cpp).
//
//   rlgpu_train [--iterations N] [--arenas A] [--rollout T] [--trajectories] [--f32-gemm] [--c2-model] [--seed S]
//               [--checkpoint-folder DIR [--ts-per-save N] [--resave-to DIR2]] [--self-play] [--fp32-inference]
//               [--rank r --world N --rccl-id FILE [--rccl-nonce STR]]
#include <execinfo.h>
#include <signal.h>

#include <chrono>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <fstream>
#include <string>
#include <thread>

#include "../facade/GigaLearn.hpp"

using namespace GGL;
using namespace RLGC;

// src/ExampleMain.cpp:128-226 with registry classes only
static EnvCreateResult EnvCreateFunc(int) {
    std::vector<WeightedReward> rewards = {
        {new AirReward(), 0.25f},
        {new WavedashReward(), 0.12f},
        {new KickoffProximityReward2v2Enhanced(), 5.f},
        {new VelocityPlayerToBallReward(), 4.f},
        {new StrongTouchReward(20, 120), 60},
        {new TouchAccelReward(), 6.f},
        {new ZeroSumReward(new VelocityBallToGoalReward(), 1), 8.0f},
        {new PickupBoostReward(), 0.1f},
        {new SaveBoostReward(), 0.010f},
        {new ZeroSumReward(new BumpReward(), 0.5f), 20},
        {new ZeroSumReward(new DemoReward(), 0.5f), 80},
        {new ZeroSumReward(new GoalReward(), 1), 150},
        {new LosingPenaltyReward(0.02f), 1.0f},
    };
    EnvCreateResult r{};
    r.rewards = rewards;
    r.terminalConditions = {new NoTouchCondition(8), new ScoreLimitCondition(3)};
    r.arena = Arena::Create(GameMode::SOCCAR);
    for (int i = 0; i < 2; i++) {
        r.arena->AddCar(Team::BLUE);
        r.arena->AddCar(Team::ORANGE);
    }
    r.actionParser = new DefaultAction();
    r.obsBuilder = new AdvancedObs();
    r.stateSetter = new KickoffState();
    return r;
}

static void ReadOrWriteRcclId(int rank, const std::string& idFile, std::string nonce, uint8_t* id) {
    // The file carries the launch's nonce (--rccl-nonce, else $RLGPU_RUN_ID, else $TORCHELASTIC_RUN_ID) before the
    // id: a reader accepts only a file of its own launch, so an id left over from an earlier run is never taken.
    if (nonce.empty())
        for (const char* e : {"RLGPU_RUN_ID", "TORCHELASTIC_RUN_ID"})
            if (const char* v = std::getenv(e); v && *v) {
                nonce = v;
                break;
            }
    const std::string header = "RLGPUID1:" + nonce + "\n";
    if (rank == 0) {  // remove, write, check, rename: readers never see a partial or stale id
        std::remove(idFile.c_str());
        RlgpuCheck(rlgpu_rccl_unique_id(id, RLGPU_RCCL_ID_BYTES), "RCCL unique id");
        const std::string tmp = idFile + ".tmp";
        {
            std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
            f.write(header.data(), (std::streamsize)header.size());
            f.write((const char*)id, RLGPU_RCCL_ID_BYTES);
            f.close();
            if (!f) throw std::runtime_error("cannot write " + tmp);
        }
        if (std::rename(tmp.c_str(), idFile.c_str()) != 0) throw std::runtime_error("cannot write " + idFile);
        return;
    }
    for (int tries = 0;; tries++) {
        std::ifstream f(idFile, std::ios::binary);
        std::string h(header.size(), '\0');
        if (f && f.read(h.data(), (std::streamsize)h.size()) && h == header && f.read((char*)id, RLGPU_RCCL_ID_BYTES) &&
            f.gcount() == (std::streamsize)RLGPU_RCCL_ID_BYTES)
            return;
        if (tries > 6000) throw std::runtime_error("timed out waiting for " + idFile + " of this launch");
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
}

// a crash prints the host backtrace to stderr before the default action (diagnostics for a test run)
static void OnCrash(int sig) {
    void* frames[64];
    const int n = backtrace(frames, 64);
    const char msg[] = "rlgpu_train: fatal signal, host backtrace:\n";
    (void)!write(2, msg, sizeof msg - 1);
    backtrace_symbols_fd(frames, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

int main(int argc, char** argv) {
    std::setvbuf(stdout, nullptr, _IOLBF, 0);
    signal(SIGSEGV, OnCrash);
    signal(SIGABRT, OnCrash);
    LearnerConfig cfg = {};
    LearnerGPUOptions opt;
    opt.experienceMode = RLGPU_EXP_ROLLOUT;  // the engine's fixed [T, P] rollout (the bench's); --trajectories: the reference's
    opt.rolloutLen = 128;
    opt.maxIterations = 3;
    opt.quitKeyThread = false;
    opt.displayReport = false;
    cfg.numGames = 4096;  // BASELINE config C2 per GPU
    cfg.tickSkip = 8;     // ExampleMain.cpp:356-430
    cfg.actionDelay = 7;
    cfg.randomSeed = 123;
    cfg.ppo.miniBatchSize = 50'000;
    cfg.ppo.maxEpisodeDuration = 300.0;
    cfg.ppo.epochs = 2;
    cfg.ppo.entropyScale = 0.035f;
    cfg.ppo.gaeGamma = 0.99f;
    cfg.ppo.policyLR = 2.5e-4f;
    cfg.ppo.criticLR = 2.5e-4f;
    cfg.ppo.sharedHead.layerSizes = {384, 384};
    cfg.ppo.policy.layerSizes = {384, 384, 384};
    cfg.ppo.critic.layerSizes = {384, 384, 384};
    for (PartialModelConfig* m : {&cfg.ppo.policy, &cfg.ppo.critic, &cfg.ppo.sharedHead}) {
        m->optimType = ModelOptimType::ADAMW;
        m->activationType = ModelActivationType::LEAKY_RELU;
        m->addLayerNorm = true;
    }
    cfg.checkpointFolder.clear();  // no checkpoints unless asked
    cfg.trainAgainstOldVersions = false;
    cfg.sendMetrics = false;
    std::string idFile, nonce, resaveTo;
    for (int i = 1; i < argc; i++) {
        auto next = [&]() -> const char* {
            if (i + 1 >= argc) throw std::invalid_argument(std::string("missing value after ") + argv[i]);
            return argv[++i];
        };
        try {
            if (!std::strcmp(argv[i], "--iterations")) opt.maxIterations = std::atol(next());
            else if (!std::strcmp(argv[i], "--arenas")) cfg.numGames = std::atoi(next());
            else if (!std::strcmp(argv[i], "--rollout")) opt.rolloutLen = std::atoi(next());
            else if (!std::strcmp(argv[i], "--trajectories")) opt.experienceMode = RLGPU_EXP_TRAJECTORIES;
            else if (!std::strcmp(argv[i], "--f32-gemm")) opt.trainGemm = RLGPU_GEMM_F32;
            else if (!std::strcmp(argv[i], "--seed")) cfg.randomSeed = std::atoll(next());
            else if (!std::strcmp(argv[i], "--checkpoint-folder")) cfg.checkpointFolder = next();
            else if (!std::strcmp(argv[i], "--ts-per-save")) cfg.tsPerSave = std::atoll(next());
            else if (!std::strcmp(argv[i], "--resave-to")) resaveTo = next();
            else if (!std::strcmp(argv[i], "--self-play")) cfg.trainAgainstOldVersions = true;
            else if (!std::strcmp(argv[i], "--fp32-inference")) cfg.ppo.useHalfPrecision = false;
            else if (!std::strcmp(argv[i], "--rank")) opt.rank = std::atoi(next());
            else if (!std::strcmp(argv[i], "--world")) opt.world = std::atoi(next());
            else if (!std::strcmp(argv[i], "--rccl-id")) idFile = next();
            else if (!std::strcmp(argv[i], "--rccl-nonce")) nonce = next();
            else if (!std::strcmp(argv[i], "--c2-model")) {
                cfg.ppo.sharedHead.layerSizes.clear();
                cfg.ppo.policy.layerSizes = cfg.ppo.critic.layerSizes = {512, 512};
            } else {
                throw std::invalid_argument(std::string("unknown argument ") + argv[i]);
            }
        } catch (const std::exception& e) {
            std::fprintf(stderr, "%s\nusage: %s [--iterations N] [--arenas A] [--rollout T] [--trajectories] [--f32-gemm] "
                                 "[--c2-model] [--seed S] [--checkpoint-folder DIR [--ts-per-save N] [--resave-to DIR2]] "
                                 "[--self-play] [--fp32-inference] [--rank r --world N --rccl-id FILE]\n", e.what(), argv[0]);
            return 2;
        }
    }
    const int players = 4 * cfg.numGames;
    cfg.ppo.tsPerItr = (int64_t)opt.rolloutLen * players;  // one rollout per iteration (or that many trajectory steps)
    cfg.ppo.batchSize = cfg.ppo.tsPerItr;
    if (cfg.ppo.miniBatchSize > cfg.ppo.batchSize) cfg.ppo.miniBatchSize = cfg.ppo.batchSize;
    if (!resaveTo.empty() && cfg.checkpointFolder.empty()) {
        std::fprintf(stderr, "--resave-to needs --checkpoint-folder\n");
        return 2;
    }
    try {
        rlgpu_collective coll{};
        hipStream_t stream = nullptr;
        if (opt.world > 1) {  // one GPU per rank (local rank = rank on one node)
            int ndev = 0;
            if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) throw std::runtime_error("no GPU");
            if (hipSetDevice(opt.rank % ndev) != hipSuccess) throw std::runtime_error("hipSetDevice failed");
            if (idFile.empty()) throw std::runtime_error("--world > 1 needs --rccl-id FILE");
            uint8_t id[RLGPU_RCCL_ID_BYTES];
            ReadOrWriteRcclId(opt.rank, idFile, nonce, id);
            // the gradient all-reduce is enqueued on the Learner's own stream
            if (hipStreamCreate(&stream) != hipSuccess) throw std::runtime_error("hipStreamCreate failed");
            RlgpuCheck(rlgpu_rccl_collective_create(id, opt.rank, opt.world, stream, &coll), "RCCL communicator");
            opt.collective = &coll;
            opt.stream = stream;
        }
        {
            Learner learner(EnvCreateFunc, cfg, nullptr, opt);
            if (!resaveTo.empty()) {  // the loaded checkpoint, saved again elsewhere without training
                learner.config.checkpointFolder = resaveTo;
                learner.Save();
            } else {
                for (int64_t it = 0; it < opt.maxIterations; it++) {
                    Report report;
                    const int64_t prev = learner.Iterate(report);
                    const bool last = it + 1 == opt.maxIterations;
                    if (!cfg.checkpointFolder.empty() && opt.rank == 0 &&
                        (last || (int64_t)learner.totalTimesteps / learner.config.tsPerSave > prev / learner.config.tsPerSave))
                        learner.Save();
                    const double t = report["Collection Time"] + report["Consumption Time"];
                    const double envSteps = report["Collected Timesteps"] / 4.0;
                    std::printf("iteration %lld: Steps/Second %.0f (agent), env-steps/s %.0f, Collection Time %.3f s, "
                                "Consumption Time %.3f s, PPO Learn Time %.3f s, Total Timesteps %llu\n",
                                (long long)it + 1, report["Collected Timesteps"] / t, envSteps / t, report["Collection Time"],
                                report["Consumption Time"] - report["PPO Learn Time"], report["PPO Learn Time"],
                                (unsigned long long)learner.totalTimesteps);
                    // the StepCallback's report (ExampleMain.cpp:233-283) over this iteration, from the device
                    double tot[RLGPU_NUM_STEP_METRICS];
                    uint64_t cnt[RLGPU_NUM_STEP_METRICS];
                    RlgpuCheck(rlgpu_learner_step_metrics(learner.handle(), tot, cnt, 1), "step metrics");
                    for (int k = 0; k < RLGPU_NUM_STEP_METRICS; k++)
                        if (cnt[k]) std::printf("  %s: %.4g\n", rlgpu_step_metric_name(k), tot[k] / (double)cnt[k]);
                }
            }
        }
        if (opt.world > 1) {
            RlgpuCheck(rlgpu_rccl_collective_destroy(&coll), "RCCL communicator");
            (void)hipStreamDestroy(stream);
        }
    } catch (const std::exception& e) {  // ExampleMain.cpp:603-612
        std::fprintf(stderr, "Exception thrown: %s\n", e.what());
        return 1;
    }
    return 0;
}
