// example_main.cpp -- the reference's src/ExampleMain.cpp on the MI355X engine (one GPU rank).
//
// ExampleMain builds the 2v2 EnvSet (AdvancedObs, DefaultAction, the 13 weighted rewards,
// NoTouch(8) + ScoreLimit(3), KickoffState; ExampleMain.cpp:128-226), sets the LearnerConfig /
// PPOLearnerConfig of ExampleMain.cpp:340-430 and calls Learner::Start.  Here the plugin set is
// the one built into the env kernel and the config is rlgpu_learner_default_config with
// ExampleMain's model topology: shared head [384, 384], policy and critic [384] x 3 (the sizes its
// log prints, run_out.log:25-28; ExampleMain.cpp:478-522); --c2-model selects BASELINE config C2's
// [512, 512] actor / critic without a shared head.  The loop is GGL::Learner::Start over a fixed
// number of iterations, printing the reference's report keys.
//
// Multi-GPU: one process per GPU (--rank r --world N --rccl-id FILE): rank 0 writes RCCL's unique id
// to FILE, the other ranks read it, every rank trains its own arenas and the Learner's exchanges run
// over the native RCCL communicator (host/rccl_collective.cpp).
//
//   rlgpu_train [--iterations N] [--arenas A] [--rollout T] [--f32-gemm] [--c2-model]
//               [--rank r --world N --rccl-id FILE [--rccl-nonce STR]]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <fstream>
#include <string>
#include <thread>

#include "learner.hpp"

int main(int argc, char** argv) {
    rlgpu_learner_config cfg;
    rlgpu_learner_default_config(&cfg);
    long iterations = 3;
    std::string idFile, nonce;
    cfg.n_shared_layers = 2;
    cfg.shared_layers[0] = cfg.shared_layers[1] = 384;
    cfg.n_policy_layers = cfg.n_critic_layers = 3;
    for (int l = 0; l < 3; l++) cfg.policy_layers[l] = cfg.critic_layers[l] = 384;
    for (int i = 1; i < argc; i++) {
        if (!std::strcmp(argv[i], "--iterations") && i + 1 < argc) iterations = std::atol(argv[++i]);
        else if (!std::strcmp(argv[i], "--arenas") && i + 1 < argc) cfg.num_arenas = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--rollout") && i + 1 < argc) cfg.rollout_len = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--f32-gemm")) cfg.train_gemm = RLGPU_GEMM_F32;
        else if (!std::strcmp(argv[i], "--rank") && i + 1 < argc) cfg.rank = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--world") && i + 1 < argc) cfg.world = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--rccl-id") && i + 1 < argc) idFile = argv[++i];
        else if (!std::strcmp(argv[i], "--rccl-nonce") && i + 1 < argc) nonce = argv[++i];
        else if (!std::strcmp(argv[i], "--c2-model")) {
            cfg.n_shared_layers = 0;
            cfg.n_policy_layers = cfg.n_critic_layers = 2;
            for (int l = 0; l < 2; l++) cfg.policy_layers[l] = cfg.critic_layers[l] = 512;
        } else {
            std::fprintf(stderr, "usage: %s [--iterations N] [--arenas A] [--rollout T] [--f32-gemm] [--c2-model]\n", argv[0]);
            return 2;
        }
    }
    try {
        if (cfg.world > 1) {  // one GPU per rank (local rank = rank on one node)
            int ndev = 0;
            if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) throw std::runtime_error("no GPU");
            if (hipSetDevice(cfg.rank % ndev) != hipSuccess) throw std::runtime_error("hipSetDevice failed");
        }
        hipStream_t s = nullptr;
        if (hipStreamCreate(&s) != hipSuccess) throw std::runtime_error("hipStreamCreate failed");
        rlgpu_collective coll{};
        if (cfg.world > 1) {
            if (idFile.empty()) throw std::runtime_error("--world > 1 needs --rccl-id FILE");
            // The file carries the launch's nonce (--rccl-nonce, else $RLGPU_RUN_ID, else
            // $TORCHELASTIC_RUN_ID) before the id: a reader accepts only a file of its own launch, so an
            // id left over from an earlier run is never taken.
            if (nonce.empty())
                for (const char* e : {"RLGPU_RUN_ID", "TORCHELASTIC_RUN_ID"})
                    if (const char* v = std::getenv(e); v && *v) {
                        nonce = v;
                        break;
                    }
            const std::string header = "RLGPUID1:" + nonce + "\n";
            uint8_t id[RLGPU_RCCL_ID_BYTES];
            if (cfg.rank == 0) {  // remove, write, check, rename: readers never see a partial or stale id
                std::remove(idFile.c_str());
                RLGC::RlgpuCheck(rlgpu_rccl_unique_id(id, sizeof id), "RCCL unique id");
                const std::string tmp = idFile + ".tmp";
                {
                    std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
                    f.write(header.data(), (std::streamsize)header.size());
                    f.write((const char*)id, sizeof id);
                    f.close();
                    if (!f) throw std::runtime_error("cannot write " + tmp);
                }
                if (std::rename(tmp.c_str(), idFile.c_str()) != 0) throw std::runtime_error("cannot write " + idFile);
            } else {
                for (int tries = 0;; tries++) {
                    std::ifstream f(idFile, std::ios::binary);
                    std::string h(header.size(), '\0');
                    if (f && f.read(h.data(), (std::streamsize)h.size()) && h == header && f.read((char*)id, sizeof id) &&
                        f.gcount() == (std::streamsize)sizeof id)
                        break;
                    if (tries > 6000) throw std::runtime_error("timed out waiting for " + idFile + " of this launch");
                    std::this_thread::sleep_for(std::chrono::milliseconds(10));
                }
            }
            RLGC::RlgpuCheck(rlgpu_rccl_collective_create(id, cfg.rank, cfg.world, s, &coll), "RCCL communicator");
        }
        GGL::Learner learner(cfg, cfg.world > 1 ? &coll : nullptr, s);
        {  // "Model parameter counts:" (PPOLearner.cpp:24-33; ModelSet order: critic, policy, shared_head)
            int64_t cnt[3] = {0, 0, 0}, total = 0;
            for (int m = 0; m < 3; m++) RLGC::RlgpuCheck(rlgpu_ppo_model_range(learner.ppo().handle(), m, nullptr, &cnt[m]), "model range");
            std::printf("Model parameter counts:\n");
            const int order[3] = {1, 0, 2};
            const char* names[3] = {"policy", "critic", "shared_head"};
            for (int m : order)
                if (cnt[m]) {
                    std::printf("\t\"%s\": %lld\n", names[m], (long long)cnt[m]);
                    total += cnt[m];
                }
            std::printf("\t[Total]: %lld\n", (long long)total);
        }
        for (long it = 0; it < iterations; it++) {
            rlgpu_learner_report r = learner.Iterate();
            const double total = r.collect_s + r.consume_s + r.learn_s;
            const double agentSteps = 4.0 * (double)r.env_steps;
            std::printf("iteration %ld: Steps/Second %.0f (agent), env-steps/s %.0f, Collection Time %.3f s, "
                        "Consumption Time %.3f s, PPO Learn Time %.3f s, Total Timesteps %lld\n",
                        it + 1, agentSteps / total, (double)r.env_steps / total, r.collect_s, r.consume_s, r.learn_s,
                        (long long)learner.stats.total_steps);
            // the StepCallback's report (ExampleMain.cpp:233-283), averaged over this iteration
            double tot[RLGPU_NUM_STEP_METRICS];
            uint64_t cnt[RLGPU_NUM_STEP_METRICS];
            RLGC::RlgpuCheck(rlgpu_envset_step_metrics(learner.env().handle(), tot, cnt, 1, s), "step metrics");
            for (int k = 0; k < RLGPU_NUM_STEP_METRICS; k++)
                if (cnt[k]) std::printf("  %s: %.4g\n", rlgpu_step_metric_name(k), tot[k] / (double)cnt[k]);
        }
        if (cfg.world > 1) RLGC::RlgpuCheck(rlgpu_rccl_collective_destroy(&coll), "RCCL communicator");
        (void)hipStreamDestroy(s);
    } catch (const std::exception& e) {  // ExampleMain.cpp:603-612
        std::fprintf(stderr, "Exception thrown: %s\n", e.what());
        return 1;
    }
    return 0;
}
