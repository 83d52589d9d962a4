// GigaLearn.hpp -- GigaLearnCPP's trainer surface over the rlgpu C ABI: the GGL::Learner a user's main constructs
// with an EnvCreateFn, a LearnerConfig and a StepCallbackFn, then Start()s (GL/public/GigaLearnCPP/Learner.h:11-57,
// src/ExampleMain.cpp:592-598), with Save / Load / SaveStats / LoadStats in the reference's checkpoint layout, old
// policy versions for self-play and the ELO skill matches.
//
//   reference                                           here
//   LearnerConfig / PPOLearnerConfig / SkillTrackerConfig / PartialModelConfig
//     (LearnerConfig.h:14-71, PPOLearnerConfig.h:9-67,  restated with the same fields and defaults; the fields the
//      SkillTrackerConfig.h, Util/ModelConfig.h)        engine cannot honour are refused by name (ValidateConfig)
//   Report (Util/Report.h:6-110)                        Report: data / AddAvg / Finish / Display
//   Learner::Learner (Learner.cpp:26-160)               envs from the EnvCreateFn (the arena checked, the plugins
//                                                       translated by EnvSetGPU.hpp), rlgpu_learner_create, the host
//                                                       fallback attached, versions, Load of the latest checkpoint
//   Learner::Start (Learner.cpp:482-1056)               Iterate(): the old-version draw, rlgpu_learner_iterate with
//                                                       the step hook (host plugins + StepCallbackFn after every env
//                                                       step, rlgpu_learner_set_step_hook), report, OnIteration,
//                                                       tsPerSave; Start() loops until 'Q' (stdin) or maxIterations
//   Save / Load / SaveStats / LoadStats (:164-279)      <checkpointFolder>/<timesteps>/RUNNING_STATS.json, POLICY.lt,
//                                                       CRITIC.lt, SHARED_HEAD.lt, <NAME>_OPTIM.lt (libtorch archives
//                                                       written / read by rlgpu/rlgpu_optim_lt), RLGPU_OPTIM.safetensors
//   PolicyVersionManager (PolicyVersionManager.cpp)     PolicyVersionManager: AddVersion / OnIteration / Save / Load
//                                                       Versions, RunSkillMatches on a FuzzedKickoffState env set
//
// One process drives one GPU (the caller selects it with hipSetDevice).  LearnerGPUOptions carries what the
// reference has no field for: rank / world and the collective of a data-parallel job, the arithmetic of the
// reference build to follow, the training GEMM mode, the experience scheduling, and an iteration cap for Start.
// Everything runs through the C ABI (include/*.h); no C++ type crosses the library boundary.
#pragma once
#include <dlfcn.h>
#include <spawn.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cinttypes>
#include <map>
#include <set>
#include <sstream>
#include <thread>
#include <unordered_map>

#include "../../include/rlgpu_learner.h"
#include "../../include/rlgpu_mesh.h"
#include "../../include/rlgpu_ppo.h"
#include "EnvSetGPU.hpp"

extern char** environ;

namespace GGL {

using RLGC::FList;
using RLGC::IList;

// ---------------------------------------------------------------------------------------------------------
// Configuration (LearnerConfig.h, PPO/PPOLearnerConfig.h, SkillTrackerConfig.h, Util/ModelConfig.h)
// ---------------------------------------------------------------------------------------------------------
enum class LearnerDeviceType { AUTO, CPU, GPU_CUDA };
enum class ModelOptimType { ADAM, ADAMW, ADAGRAD, RMSPROP, MAGSGD };
enum class ModelActivationType { RELU, LEAKY_RELU, SIGMOID, TANH };

struct PartialModelConfig {
    std::vector<int> layerSizes = {};
    ModelActivationType activationType = ModelActivationType::RELU;
    ModelOptimType optimType = ModelOptimType::ADAM;
    bool addLayerNorm = true;
    bool addOutputLayer = true;
    bool IsValid() const { return !layerSizes.empty(); }
};

struct PPOLearnerConfig {
    int64_t tsPerItr = 50'000;
    int64_t batchSize = 50'000;
    int64_t miniBatchSize = 0;  // 0: batchSize
    bool overbatching = true;
    double maxEpisodeDuration = 120;
    bool deterministic = false;
    bool useHalfPrecision = true;
    PartialModelConfig policy, critic, sharedHead;
    int epochs = 2;
    float policyLR = 3e-4f;
    float criticLR = 3e-4f;
    float entropyScale = 0.018f;
    bool maskEntropy = false;
    float clipRange = 0.2f;
    float policyTemperature = 1;
    float gaeLambda = 0.95f;
    float gaeGamma = 0.99f;
    float rewardClipRange = 200;
    bool useGuidingPolicy = false;
    std::filesystem::path guidingPolicyPath = "guiding_policy/";
    float guidingStrength = 0.03f;
    PPOLearnerConfig() {
        policy.layerSizes = {256, 256, 256};
        critic.layerSizes = {256, 256, 256};
        sharedHead.layerSizes = {256};
        sharedHead.addOutputLayer = false;
    }
};

// PPO/TransferLearnConfig.h: the fields of Learner::StartTransferLearn's configuration (distilling an old policy
// with its own obs builder / action parser into the current one, Learner.cpp:290-470, PPOLearner.cpp:583-637).
// Restated so a caller's source compiles; the engine does not run that mode (StartTransferLearn says so).
using MakeObsFn = std::function<RLGC::ObsBuilder*()>;
using MakeActFn = std::function<RLGC::ActionParser*()>;
struct TransferLearnConfig {
    MakeObsFn makeOldObsFn;
    MakeActFn makeOldActFn;
    std::function<std::vector<int>(const RLGC::Player&, const RLGC::GameState&)> mapActsFn = nullptr;
    PartialModelConfig oldPolicyConfig;
    PartialModelConfig oldSharedHeadConfig;
    std::filesystem::path oldModelsPath;
    float lr = 3e-4f;
    int batchSize = 50'000;
    int epochs = 5;
    bool useKLDiv = false;
    float lossScale = 500.f;
    float lossExponent = 1.f;
};

struct SkillTrackerConfig {
    bool enabled = false;
    int numArenas = 16;
    float simTime = 45;
    float maxSimTime = 240;
    int updateInterval = 16;
    float ratingInc = 5;
    float initialRating = 0;
    bool deterministic = false;
};

struct LearnerConfig {
    int numGames = 300;
    int tickSkip = 8;
    int actionDelay = 7;
    bool renderMode = false;
    float renderTimeScale = 1.0f;
    PPOLearnerConfig ppo = {};
    std::filesystem::path checkpointFolder = "C:\\Giga\\GigaLearnCPP-Leak\\checkpoints";
    int64_t tsPerSave = 10'000'000;
    int64_t randomSeed = -1;
    int checkpointsToKeep = 8;
    LearnerDeviceType deviceType = LearnerDeviceType::AUTO;
    bool standardizeObs = false;
    float minObsSTD = 1 / 10.f;
    float maxObsMeanRange = 3;
    int maxObsSamples = 100;
    bool standardizeReturns = true;
    int maxReturnSamples = 150;
    bool addRewardsToMetrics = true;
    int maxRewardSamples = 50;
    int rewardSampleRandInterval = 8;
    bool sendMetrics = true;
    std::string metricsProjectName = "Reinforcement Learning";
    std::string metricsGroupName = "Rocket League";
    std::string metricsRunName = "gigalearncpp-run";
    bool savePolicyVersions = false;
    int64_t tsPerVersion = 25'000'000;
    int maxOldVersions = 32;
    bool trainAgainstOldVersions = true;
    float trainAgainstOldChance = 0.15f;
    SkillTrackerConfig skillTracker = {};
};

// Engine options the reference has no field for.
struct LearnerGPUOptions {
    int rank = 0, world = 1;                       // data-parallel job: this rank's numGames arenas
    const rlgpu_collective* collective = nullptr;  // world > 1: rlgpu_rccl_collective_create's, or any other
    int32_t arith = RLGPU_ARITH_MSVC_X64;          // the reference build's Bullet arithmetic (include/rlgpu_arith.h)
    int32_t trainGemm = RLGPU_GEMM_F16X3;          // fp32-class training GEMMs (include/rlgpu_ppo.h)
    int32_t experienceMode = RLGPU_EXP_TRAJECTORIES;  // the reference's complete trajectories; RLGPU_EXP_ROLLOUT:
    int32_t rolloutLen = 0;                        //   a fixed [rolloutLen, players] rollout (0: tsPerItr / players)
    int64_t maxIterations = -1;                    // Start() saves and returns after this many (-1: until 'Q';
                                                   // the environment variable RLGPU_MAX_ITERATIONS sets it too)
    bool quitKeyThread = true;                     // read 'Q' from a terminal stdin (StartQuitKeyThread)
    bool displayReport = true;                     // Report::Display every iteration
    hipStream_t stream = nullptr;                  // the Learner's HIP stream (null: its own); a native RCCL
                                                   // collective enqueues the gradient all-reduce on the same one
};

// ---------------------------------------------------------------------------------------------------------
// Report (Util/Report.h:6-110)
// ---------------------------------------------------------------------------------------------------------
struct Report {
    typedef double Val;
    std::unordered_map<std::string, Val> data;
    struct Avg {
        Val total = 0;
        uint64_t count = 0;
    };
    std::unordered_map<std::string, Avg> avgs;

    Val& operator[](const std::string& key) { return data[key]; }
    Val operator[](const std::string& key) const { return data.at(key); }
    bool Has(const std::string& key) const { return data.find(key) != data.end(); }
    void Add(const std::string& key, Val val) { data[key] += val; }
    void AddAvg(const std::string& key, Val val) {
        auto& a = avgs[key];
        a.total += val;
        a.count++;
    }
    void FinishAvg(const std::string& key) {
        auto it = avgs.find(key);
        if (it == avgs.end()) throw std::runtime_error("Cannot call Report::FinishAvg() on non-existent average \"" + key + "\"!");
        data[key] = it->second.total / (Val)it->second.count;
        avgs.erase(it);
    }
    void Finish() {
        for (auto& p : avgs) data[p.first] = p.second.total / (Val)p.second.count;
        avgs.clear();
    }
    void Clear() { *this = Report(); }
    std::string SingleToString(const std::string& key, bool = false) const {
        std::ostringstream o;
        o << key << ": " << (*this)[key];
        return o.str();
    }
    std::string ToString(bool digitCommas = false, const std::string& prefix = {}) const {
        std::ostringstream o;
        for (auto& p : data) o << prefix << SingleToString(p.first, digitCommas) << "\n";
        return o.str();
    }
    void Display(const std::vector<std::string>& keyRows) const {  // Report.cpp:5-40
        std::ostringstream o;
        o << "\n" << std::string(40, '=') << "\n";
        for (std::string row : keyRows) {
            if (row.empty()) {
                o << "\n";
                continue;
            }
            int indent = 0;
            while (!row.empty() && row[0] == '-') {
                indent++;
                row.erase(row.begin());
            }
            if (!Has(row)) continue;
            if (indent > 0) o << std::string((indent - 1) * 3, ' ') << " - ";
            o << SingleToString(row, true) << "\n";
        }
        std::cout << o.str() << std::flush;
    }
};

class Learner;
typedef std::function<void(Learner*, const std::vector<RLGC::GameState>& states, Report& report)> StepCallbackFn;

// ---------------------------------------------------------------------------------------------------------
// File helpers: a small JSON reader / writer for RUNNING_STATS.json / STATS.json, safetensors, the libtorch helper
// ---------------------------------------------------------------------------------------------------------
namespace detail {

struct Json {
    enum Kind { NUL, NUM, STR, OBJ, ARR, BOOL } kind = NUL;
    std::string text;  // NUM: the token (integers stay exact); STR: the string
    bool b = false;
    std::map<std::string, Json> obj;
    std::vector<Json> arr;
    bool Has(const std::string& k) const { return kind == OBJ && obj.count(k); }
    const Json& operator[](const std::string& k) const {
        auto it = obj.find(k);
        if (kind != OBJ || it == obj.end()) throw std::runtime_error("JSON: no key \"" + k + "\"");
        return it->second;
    }
    double Num() const {
        if (kind != NUM) throw std::runtime_error("JSON: not a number");
        return std::stod(text);
    }
    int64_t Int() const {
        if (kind != NUM) throw std::runtime_error("JSON: not a number");
        return text.find_first_of(".eE") == std::string::npos ? (int64_t)std::stoll(text) : (int64_t)std::stod(text);
    }
};

struct JsonParser {
    const std::string& s;
    size_t i = 0;
    void Ws() {
        while (i < s.size() && std::isspace((unsigned char)s[i])) i++;
    }
    [[noreturn]] void Fail(const char* what) { throw std::runtime_error(std::string("JSON parse error: ") + what); }
    std::string Str() {
        if (s[i] != '"') Fail("expected a string");
        std::string out;
        for (i++; i < s.size() && s[i] != '"'; i++) {
            if (s[i] == '\\' && i + 1 < s.size()) {
                char c = s[++i];
                out += c == 'n' ? '\n' : c == 't' ? '\t' : c;
            } else {
                out += s[i];
            }
        }
        if (i >= s.size()) Fail("unterminated string");
        i++;
        return out;
    }
    Json Value() {
        Ws();
        if (i >= s.size()) Fail("unexpected end");
        Json v;
        char c = s[i];
        if (c == '{') {
            v.kind = Json::OBJ;
            i++;
            Ws();
            if (s[i] == '}') {
                i++;
                return v;
            }
            for (;;) {
                Ws();
                std::string k = Str();
                Ws();
                if (s[i] != ':') Fail("expected ':'");
                i++;
                v.obj[k] = Value();
                Ws();
                if (s[i] == ',') {
                    i++;
                    continue;
                }
                if (s[i] == '}') {
                    i++;
                    return v;
                }
                Fail("expected ',' or '}'");
            }
        }
        if (c == '[') {
            v.kind = Json::ARR;
            i++;
            Ws();
            if (s[i] == ']') {
                i++;
                return v;
            }
            for (;;) {
                v.arr.push_back(Value());
                Ws();
                if (s[i] == ',') {
                    i++;
                    continue;
                }
                if (s[i] == ']') {
                    i++;
                    return v;
                }
                Fail("expected ',' or ']'");
            }
        }
        if (c == '"') {
            v.kind = Json::STR;
            v.text = Str();
            return v;
        }
        if (!s.compare(i, 4, "true") || !s.compare(i, 5, "false")) {
            v.kind = Json::BOOL;
            v.b = s[i] == 't';
            i += v.b ? 4 : 5;
            return v;
        }
        if (!s.compare(i, 4, "null")) {
            i += 4;
            return v;
        }
        size_t j = i;
        while (j < s.size() && (std::isdigit((unsigned char)s[j]) || std::strchr("+-.eE", s[j]))) j++;
        if (j == i) Fail("unexpected character");
        v.kind = Json::NUM;
        v.text = s.substr(i, j - i);
        i = j;
        return v;
    }
};

inline Json ParseJson(const std::string& text) {
    JsonParser p{text};
    return p.Value();
}

inline std::string ReadFile(const std::filesystem::path& p) {
    std::ifstream f(p, std::ios::binary);
    if (!f.good()) throw std::runtime_error("Can't open file at " + p.string());
    std::ostringstream o;
    o << f.rdbuf();
    return o.str();
}

inline void WriteFile(const std::filesystem::path& p, const void* data, size_t bytes) {
    std::ofstream f(p, std::ios::binary | std::ios::trunc);
    f.write((const char*)data, (std::streamsize)bytes);
    if (!f.good()) throw std::runtime_error("Can't write file at " + p.string());
}

inline std::string Num(double v) {  // shortest text that reads back as the same double
    char b[64];
    std::snprintf(b, sizeof b, "%.17g", v);
    return b;
}

// Utils::FindNumberedDirs (Util/Utils.cpp:3-27)
inline std::set<int64_t> NumberedDirs(const std::filesystem::path& base) {
    std::set<int64_t> out;
    std::error_code ec;
    if (!std::filesystem::is_directory(base, ec)) return out;
    for (auto& e : std::filesystem::directory_iterator(base)) {
        const std::string n = e.path().filename().string();
        if (e.is_directory() && !n.empty() && n.find_first_not_of("0123456789") == std::string::npos) out.insert(std::stoll(n));
    }
    return out;
}

// safetensors (the exact optimizer state kept beside the libtorch archives, rlgpu/checkpoint.py OPTIM_FILE)
struct Tensor {
    std::string dtype;  // "F32" / "I64"
    std::vector<int64_t> shape;
    std::vector<char> bytes;
};
inline void WriteSafetensors(const std::filesystem::path& p, const std::map<std::string, Tensor>& ts) {
    std::string h = "{";
    size_t off = 0;
    for (auto& [name, t] : ts) {
        if (h.size() > 1) h += ",";
        h += "\"" + name + "\":{\"dtype\":\"" + t.dtype + "\",\"shape\":[";
        for (size_t k = 0; k < t.shape.size(); k++) h += (k ? "," : "") + std::to_string(t.shape[k]);
        h += "],\"data_offsets\":[" + std::to_string(off) + "," + std::to_string(off + t.bytes.size()) + "]}";
        off += t.bytes.size();
    }
    h += "}";
    while (h.size() % 8) h += ' ';
    std::string out(8, '\0');
    const uint64_t n = h.size();
    std::memcpy(out.data(), &n, 8);
    out += h;
    for (auto& kv : ts) out.append(kv.second.bytes.data(), kv.second.bytes.size());
    WriteFile(p, out.data(), out.size());
}
inline std::map<std::string, Tensor> ReadSafetensors(const std::filesystem::path& p) {
    const std::string raw = ReadFile(p);
    if (raw.size() < 8) throw std::runtime_error(p.string() + ": not a safetensors file");
    uint64_t n = 0;
    std::memcpy(&n, raw.data(), 8);
    if (8 + n > raw.size()) throw std::runtime_error(p.string() + ": truncated header");
    const Json h = ParseJson(raw.substr(8, n));
    std::map<std::string, Tensor> out;
    for (auto& [name, v] : h.obj) {
        if (name == "__metadata__") continue;
        Tensor t;
        t.dtype = v["dtype"].text;
        for (auto& d : v["shape"].arr) t.shape.push_back(d.Int());
        const int64_t a = v["data_offsets"].arr.at(0).Int(), b = v["data_offsets"].arr.at(1).Int();
        if (a < 0 || b < a || 8 + n + (uint64_t)b > raw.size()) throw std::runtime_error(p.string() + ": bad offsets");
        t.bytes.assign(raw.data() + 8 + n + a, raw.data() + 8 + n + b);
        out[name] = std::move(t);
    }
    return out;
}

// the directory of librlgpu.so (its libtorch helper rlgpu_optim_lt sits next to it)
inline std::filesystem::path LibraryDir() {
    Dl_info info{};
    if (!dladdr((const void*)&rlgpu_learner_create, &info) || !info.dli_fname)
        throw std::runtime_error("cannot locate librlgpu.so");
    return std::filesystem::absolute(info.dli_fname).parent_path();
}

// runs the libtorch helper as a child process (posix_spawn: no exec of this process) and waits for it
inline void RunHelper(const std::vector<std::string>& args) {
    const std::string tool = (LibraryDir() / "rlgpu_optim_lt").string();
    if (!std::filesystem::exists(tool))
        throw std::runtime_error(tool + " is not built (__graft_entry__.build / make optim): no libtorch archives");
    std::vector<std::string> all{tool};
    all.insert(all.end(), args.begin(), args.end());
    std::vector<char*> argv;
    for (auto& a : all) argv.push_back(const_cast<char*>(a.c_str()));
    argv.push_back(nullptr);
    pid_t pid = 0;
    if (posix_spawn(&pid, tool.c_str(), nullptr, nullptr, argv.data(), environ) != 0)
        throw std::runtime_error("cannot start " + tool);
    int st = 0;
    if (waitpid(pid, &st, 0) != pid || !WIFEXITED(st) || WEXITSTATUS(st) != 0) {
        std::string cmd;
        for (auto& a : all) cmd += a + " ";
        throw std::runtime_error("libtorch archive helper failed (exit " + std::to_string(WIFEXITED(st) ? WEXITSTATUS(st) : -1) +
                                 "): " + cmd);
    }
}

inline std::filesystem::path TempFile(const char* tag) {
    static std::atomic<int> k{0};
    return std::filesystem::temp_directory_path() /
           ("rlgpu_" + std::to_string((long)getpid()) + "_" + std::to_string(k++) + "_" + tag);
}

inline void HipOk(hipError_t e, const char* what) { RLGC::RlgpuCheckHip(e, what); }

}  // namespace detail

// ---------------------------------------------------------------------------------------------------------
// Models of the PPO handle: names, shapes and file layout (PPOLearner.cpp:42-74, Models.h:114-128)
// ---------------------------------------------------------------------------------------------------------
struct ModelSpec {
    int index;          // rlgpu_ppo model index: 0 policy, 1 critic, 2 shared head
    const char* name;   // Model::modelName
    int inputs, outputs;
    std::vector<int> layers;
    std::string FileName(const char* suffix = "") const {  // GetSuffixedSavePath: upper-cased name + suffix + .lt
        std::string n = name;
        for (auto& c : n) c = (char)std::toupper((unsigned char)c);
        return n + suffix + ".lt";
    }
    std::vector<std::string> HelperShape() const {
        std::vector<std::string> a{std::to_string(inputs), std::to_string(outputs)};
        for (int h : layers) a.push_back(std::to_string(h));
        return a;
    }
    // parameter shapes in parameters() order (Linear weight [out, in], bias, LayerNorm weight, bias; output Linear)
    std::vector<std::string> ParamShapes() const {
        std::vector<std::string> s;
        int last = inputs;
        for (int h : layers) {
            s.push_back(std::to_string(h) + "x" + std::to_string(last));
            s.push_back(std::to_string(h));
            s.push_back(std::to_string(h));
            s.push_back(std::to_string(h));
            last = h;
        }
        if (outputs > 0) {
            s.push_back(std::to_string(outputs) + "x" + std::to_string(last));
            s.push_back(std::to_string(outputs));
        }
        return s;
    }
};

// ---------------------------------------------------------------------------------------------------------
// Skill ratings and old policy versions (PolicyVersionManager.h:12-52, PolicyVersionManager.cpp)
// ---------------------------------------------------------------------------------------------------------
struct SkillRating {
    std::map<std::string, float> data;
    float& GetRating(const std::string& mode, float initial) {  // inserts the initial rating for a new mode
        auto it = data.find(mode);
        if (it == data.end()) it = data.emplace(mode, initial).first;
        return it->second;
    }
    std::string ToJSON() const {
        std::string s = "{";
        for (auto& [k, v] : data) s += (s.size() > 1 ? ", " : "") + std::string("\"") + k + "\": " + detail::Num((double)v);
        return s + "}";
    }
    void ReadFromJSON(const detail::Json& j) {
        data.clear();
        for (auto& [k, v] : j.obj) data[k] = (float)v.Num();
    }
    // GetModeName: "<smaller team>v<larger team>"
    static std::string ModeName(const std::vector<RLGC::Player>& players) {
        int n[2] = {0, 0};
        for (auto& p : players) n[(int)p.team]++;
        return std::to_string(std::min(n[0], n[1])) + "v" + std::to_string(std::max(n[0], n[1]));
    }
};

struct PolicyVersion {
    int64_t timesteps = 0;
    float* params = nullptr;  // device: the policy's flat parameters, then the shared head's (rlgpu_ppo_set_version)
    SkillRating ratings;
};

class Learner;

class PolicyVersionManager {
  public:
    std::filesystem::path saveFolder;
    int maxVersions;
    int64_t tsPerVersion;
    SkillTrackerConfig skillConfig;
    std::vector<PolicyVersion> versions;
    SkillRating curRatings;

    PolicyVersionManager(Learner* learner, std::filesystem::path folder, int maxVersions, int64_t tsPerVersion,
                         const SkillTrackerConfig& skill);
    ~PolicyVersionManager();
    PolicyVersionManager(const PolicyVersionManager&) = delete;
    PolicyVersionManager& operator=(const PolicyVersionManager&) = delete;

    PolicyVersion& AddVersion(int64_t timesteps, const float* dParams = nullptr);
    void OnIteration(Report& report, int64_t totalTimesteps, int64_t prevTimesteps);
    void SaveVersions();
    void LoadVersions(int64_t curTimesteps);
    void RunSkillMatches(Report& report);
    void AddRunningStatsToJSON(std::string& j) const {
        if (skillConfig.enabled) j += ",\n    \"skill_ratings\": " + curRatings.ToJSON();
    }
    void LoadRunningStatsFromJSON(const detail::Json& j) {
        if (skillConfig.enabled && j.Has("skill_ratings")) curRatings.ReadFromJSON(j["skill_ratings"]);
    }

  private:
    Learner* L;
    int64_t versionSize = 0;
    // RunSkillMatches state (PolicyVersionManager.cpp:156-300)
    rlgpu_envset* skillEnv = nullptr;
    int32_t* dSkillActs = nullptr;
    uint8_t* dOldRows = nullptr;
    int curGoals = 0, skillRuns = 0, iterationsSinceRan = 0;
    bool doContinuation = false;
    int prevOldVersionIndex = 0, prevNewTeam = 0;
    float prevSimTime = 0;
    uint64_t skillSteps = 0;
};

// ---------------------------------------------------------------------------------------------------------
// Learner
// ---------------------------------------------------------------------------------------------------------
class Learner {
  public:
    LearnerConfig config;
    RLGC::EnvSetGPU* envSet = nullptr;
    PolicyVersionManager* versionMgr = nullptr;
    RLGC::EnvCreateFn envCreateFn;
    int obsSize = RLGPU_OBS;
    int numActions = RLGPU_ACTIONS;
    std::string runID = {};
    uint64_t totalTimesteps = 0, totalIterations = 0;
    StepCallbackFn stepCallback = nullptr;
    LearnerGPUOptions options;
    std::vector<ModelSpec> models;  // the PPO handle's models (policy, critic[, shared head])

    Learner(RLGC::EnvCreateFn envCreateFunc, LearnerConfig cfg, StepCallbackFn cb = nullptr)
        : Learner(std::move(envCreateFunc), std::move(cfg), std::move(cb), LearnerGPUOptions{}) {}
    Learner(RLGC::EnvCreateFn envCreateFunc, LearnerConfig cfg, StepCallbackFn cb, const LearnerGPUOptions& opt);
    ~Learner();
    Learner(const Learner&) = delete;
    Learner& operator=(const Learner&) = delete;

    void Start();
    // Learner::StartTransferLearn (Learner.h:45): not part of the engine's path; refused by name
    [[noreturn]] void StartTransferLearn(const TransferLearnConfig&) {
        throw std::runtime_error("GGL::Learner::StartTransferLearn: transfer learning (PPOLearner::TransferLearn) is not "
                                 "implemented by the rlgpu engine");
    }
    // one Start() loop body (collection, consumption, learning, versions) into `report`; returns the timesteps
    // before it (engine extension: Start() without the loop)
    int64_t Iterate(Report& report);
    void Save();
    void Load();
    void SaveStats(const std::filesystem::path& path);
    void LoadStats(const std::filesystem::path& path);

    rlgpu_learner* handle() const { return h_; }
    rlgpu_ppo* ppoHandle() const { return ppo_; }
    hipStream_t stream() const { return stream_; }
    int oldTeam() const { return oldTeam_; }
    // the model's flat parameters / AdamW state in torch parameters() order, on the host
    std::vector<float> ModelParams(int model) const;

    static void ValidateConfig(const LearnerConfig& c);

  private:
    rlgpu_learner* h_ = nullptr;
    rlgpu_ppo* ppo_ = nullptr;
    hipStream_t stream_ = nullptr;
    std::vector<float> meshTris_;
    std::vector<int32_t> meshObjects_;
    Report* curReport_ = nullptr;
    std::string hookError_;
    int oldTeam_ = -1;
    std::atomic<bool> quitPressed_{false};

    static int HookThunk(void* user, int32_t phase);
    void SyncStats();
    void PushStats();
    void LoadMeshes();
    void SaveModels(const std::filesystem::path& folder, bool saveOptim, const float* flatParams,
                    const std::vector<int>& which) const;
    friend class PolicyVersionManager;
};

// ---- config checks: what the engine computes is the reference's, or the field is refused by name -------------
inline void Learner::ValidateConfig(const LearnerConfig& c) {
    auto bad = [](const std::string& what) { throw std::invalid_argument("LearnerConfig: " + what); };
    if (c.renderMode) bad("renderMode is not supported (the RLBot render path is out of this engine's scope)");
    if (c.deviceType == LearnerDeviceType::CPU) bad("deviceType CPU: this engine runs on the GPU only");
    if (c.numGames <= 0) bad("numGames must be positive");
    if (c.standardizeObs) bad("standardizeObs is not supported (obs standardisation is not on the device path)");
    if (c.ppo.policyTemperature != 1) bad("ppo.policyTemperature must be 1");
    if (c.ppo.maskEntropy) bad("ppo.maskEntropy is not supported");
    if (c.ppo.useGuidingPolicy) bad("ppo.useGuidingPolicy is not supported");
    if (!c.ppo.useHalfPrecision && (c.trainAgainstOldVersions || c.skillTracker.enabled))
        bad("ppo.useHalfPrecision = false with trainAgainstOldVersions or skillTracker: old policy versions run on "
            "16-bit inference copies only (set useHalfPrecision = true, or turn self-play / skill matches off)");
    if (c.ppo.epochs <= 0 || c.ppo.tsPerItr <= 0 || c.ppo.batchSize <= 0) bad("ppo.epochs / tsPerItr / batchSize must be positive");
    const PartialModelConfig* ms[3] = {&c.ppo.policy, &c.ppo.critic, &c.ppo.sharedHead};
    const char* names[3] = {"policy", "critic", "sharedHead"};
    for (int k = 0; k < 3; k++) {
        const PartialModelConfig& m = *ms[k];
        if (k == 2 && !m.IsValid()) continue;
        if (!m.IsValid()) bad(std::string("ppo.") + names[k] + " has no layers");
        if ((int)m.layerSizes.size() > RLGPU_MAX_LAYERS) bad(std::string("ppo.") + names[k] + ": more than 8 layers");
        if (!m.addLayerNorm) bad(std::string("ppo.") + names[k] + ".addLayerNorm = false is not supported");
        if (m.activationType != ModelActivationType::LEAKY_RELU && m.activationType != ModelActivationType::RELU)
            bad(std::string("ppo.") + names[k] + ".activationType must be LEAKY_RELU or RELU");
        if (m.activationType != c.ppo.policy.activationType) bad("every model must use the same activationType");
        if (m.optimType != ModelOptimType::ADAMW && m.optimType != ModelOptimType::ADAM)
            bad(std::string("ppo.") + names[k] + ".optimType must be ADAMW or ADAM");
        if (m.optimType != c.ppo.policy.optimType) bad("every model must use the same optimType");
        if (k < 2 && !m.addOutputLayer) bad(std::string("ppo.") + names[k] + ".addOutputLayer must be true");
        if (k == 2 && m.addOutputLayer) bad("ppo.sharedHead.addOutputLayer must be false (PPOLearner.cpp:57)");
    }
}

inline Learner::Learner(RLGC::EnvCreateFn envCreateFunc, LearnerConfig cfg, StepCallbackFn cb, const LearnerGPUOptions& opt)
    : config(std::move(cfg)), envCreateFn(std::move(envCreateFunc)), stepCallback(std::move(cb)), options(opt) {
    ValidateConfig(config);
    if (const char* v = std::getenv("RLGPU_MAX_ITERATIONS"); v && *v) options.maxIterations = std::atoll(v);
    if (config.tsPerSave == 0) config.tsPerSave = config.ppo.tsPerItr;
    if (config.randomSeed == -1)
        config.randomSeed = std::chrono::duration_cast<std::chrono::milliseconds>(
                                std::chrono::system_clock::now().time_since_epoch()).count();
    std::printf("Learner::Learner():\n\tCheckpoint Save/Load Dir: %s\n", config.checkpointFolder.string().c_str());
    if (config.sendMetrics) std::printf("\t(metrics are printed; the Python metrics receiver is not part of this engine)\n");
    if (options.stream) stream_ = options.stream;
    else detail::HipOk(hipStreamCreate(&stream_), "stream");
    LoadMeshes();

    // envs: the EnvCreateFn per arena, the arena checked, the plugins translated (EnvSet ctor, EnvSet.cpp:46-111)
    RLGC::EnvSetConfig esc{envCreateFn, config.numGames, config.tickSkip, config.actionDelay, config.addRewardsToMetrics};
    std::vector<RLGC::EnvCreateResult> results;
    const RLGC::PluginPlan plan = RLGC::EnvSetGPU::CreateEnvs(esc, results);

    rlgpu_learner_config c;
    RLGC::RlgpuCheck(rlgpu_learner_default_config(&c), "default config");
    const int players = 4 * config.numGames;
    c.num_arenas = config.numGames;
    c.tick_skip = config.tickSkip;
    c.action_delay = config.actionDelay;
    c.seed = (uint64_t)config.randomSeed;
    c.max_episode_duration = (float)config.ppo.maxEpisodeDuration;
    c.experience_mode = options.experienceMode;
    c.ts_per_itr = config.ppo.tsPerItr;
    c.rollout_len = options.rolloutLen > 0 ? options.rolloutLen
                                            : (int32_t)std::max<int64_t>(1, (config.ppo.tsPerItr + players - 1) / players);
    c.epochs = config.ppo.epochs;
    c.mini_batch_size = (int32_t)(config.ppo.miniBatchSize > 0 ? config.ppo.miniBatchSize : config.ppo.batchSize);
    c.batch_size = config.ppo.batchSize;
    c.overbatching = config.ppo.overbatching;
    c.gamma = config.ppo.gaeGamma;
    c.gae_lambda = config.ppo.gaeLambda;
    c.clip_range = config.ppo.clipRange;
    c.entropy_scale = config.ppo.entropyScale;
    c.policy_lr = config.ppo.policyLR;
    c.critic_lr = config.ppo.criticLR;
    c.reward_clip_range = config.ppo.rewardClipRange;
    c.return_samples = config.standardizeReturns ? config.maxReturnSamples : 0;  // no samples: std stays 1
    auto layers = [](const PartialModelConfig& m, int32_t* dst, int32_t& n) {
        n = (int32_t)m.layerSizes.size();
        for (int i = 0; i < n; i++) dst[i] = m.layerSizes[i];
    };
    layers(config.ppo.policy, c.policy_layers, c.n_policy_layers);
    layers(config.ppo.critic, c.critic_layers, c.n_critic_layers);
    c.n_shared_layers = 0;
    if (config.ppo.sharedHead.IsValid()) layers(config.ppo.sharedHead, c.shared_layers, c.n_shared_layers);
    c.deterministic = config.ppo.deterministic;
    // PPOLearnerConfig::useHalfPrecision (PPOLearnerConfig.h:31): Model::Forward's half branch (bf16 inference,
    // the reference's seqHalf) or its fp32 branch (Models.cpp:36-68) -- the training forward's arithmetic
    c.infer_fp16 = config.ppo.useHalfPrecision ? RLGPU_INFER_BF16 : RLGPU_INFER_F32;
    c.train_gemm = options.trainGemm;
    c.arith = options.arith;
    c.activation = config.ppo.policy.activationType == ModelActivationType::RELU ? RLGPU_ACT_RELU : RLGPU_ACT_LEAKY_RELU;
    c.optimizer = config.ppo.policy.optimType == ModelOptimType::ADAM ? RLGPU_OPT_ADAM : RLGPU_OPT_ADAMW;
    c.rank = options.rank;
    c.world = options.world;
    static const rlgpu_reward_spec kNoRewards{};
    static const rlgpu_terminal_spec kNoTerminals{};
    c.rewards = plan.deviceRewards.empty() ? &kNoRewards : plan.deviceRewards.data();  // empty list, not ExampleMain's
    c.n_rewards = (int32_t)plan.deviceRewards.size();
    c.terminals = plan.deviceTerminals.empty() ? &kNoTerminals : plan.deviceTerminals.data();
    c.n_terminals = (int32_t)plan.deviceTerminals.size();
    if (!meshTris_.empty()) {
        c.mesh_tris = meshTris_.data();
        c.mesh_ntris = (int32_t)(meshTris_.size() / 9);
        c.mesh_objects = (int32_t)meshObjects_.size();
        c.mesh_object_ntris = meshObjects_.data();
    }
    if (plan.stateSetter != RLGPU_SS_KICKOFF)
        throw std::invalid_argument("Learner: the training env set resets to KickoffState (FuzzedKickoffState is the skill tracker's)");
    RLGC::RlgpuCheck(rlgpu_learner_create(&c, options.world > 1 ? options.collective : nullptr, stream_, &h_), "Learner");
    rlgpu_envset* env = nullptr;
    RLGC::RlgpuCheck(rlgpu_learner_handles(h_, &env, &ppo_), "Learner handles");
    envSet = new RLGC::EnvSetGPU(esc, std::move(results), plan, env, stream_);
    if (plan.HasHost() || stepCallback) RLGC::RlgpuCheck(rlgpu_learner_set_step_hook(h_, &Learner::HookThunk, this), "step hook");

    // the PPO handle's models (PPOLearner::MakeModels): shared head feeds policy and critic
    const int feat = c.n_shared_layers ? config.ppo.sharedHead.layerSizes.back() : RLGPU_OBS;
    models.push_back({0, "policy", feat, RLGPU_ACTIONS, config.ppo.policy.layerSizes});
    models.push_back({1, "critic", feat, 1, config.ppo.critic.layerSizes});
    if (c.n_shared_layers) models.push_back({2, "shared_head", RLGPU_OBS, 0, config.ppo.sharedHead.layerSizes});
    std::printf("Model parameter counts:\n");
    int64_t total = 0;
    for (int m : {0, 1, 2}) {
        int64_t off = 0, cnt = 0;
        RLGC::RlgpuCheck(rlgpu_ppo_model_range(ppo_, m, &off, &cnt), "model range");
        if (cnt) std::printf("\t\"%s\": %" PRId64 "\n", m == 0 ? "policy" : m == 1 ? "critic" : "shared_head", cnt);
        total += cnt;
    }
    std::printf("\t[Total]: %" PRId64 "\n", total);

    if (config.skillTracker.enabled || config.trainAgainstOldVersions) config.savePolicyVersions = true;  // :131-132
    if (config.savePolicyVersions) {
        if (config.checkpointFolder.empty())
            throw std::invalid_argument("Cannot save/load old policy versions with no checkpoint save folder");
        versionMgr = new PolicyVersionManager(this, config.checkpointFolder / "policy_versions", config.maxOldVersions,
                                              config.tsPerVersion, config.skillTracker);
    }
    if (!config.checkpointFolder.empty()) Load();
    if (versionMgr) versionMgr->LoadVersions((int64_t)totalTimesteps);
}

inline Learner::~Learner() {
    if (stream_) (void)hipStreamSynchronize(stream_);
    delete versionMgr;
    delete envSet;
    if (h_) rlgpu_learner_destroy(h_);
    if (stream_ && !options.stream) (void)hipStreamDestroy(stream_);
}

// RocketSim::Init's folder (RocketSim.cpp:100-170: <folder>/soccar/*.cmf, one collision object per file, sorted
// by name here); the reference's Learner initialises "collision_meshes" itself when the user did not
inline void Learner::LoadMeshes() {
    std::string folder = RocketSim::MeshFolder();
    if (folder.empty()) folder = "collision_meshes";
    const std::filesystem::path sub = std::filesystem::path(folder) / "soccar";
    std::error_code ec;
    if (!std::filesystem::is_directory(sub, ec)) return;
    std::vector<std::filesystem::path> files;
    for (auto& e : std::filesystem::directory_iterator(sub))
        if (e.path().extension() == ".cmf") files.push_back(e.path());
    std::sort(files.begin(), files.end());
    for (auto& f : files) {
        const std::string img = detail::ReadFile(f);
        int32_t nt = 0;
        RLGC::RlgpuCheck(rlgpu_cmf_parse(img.data(), (int64_t)img.size(), nullptr, 0, &nt, nullptr, nullptr), f.string().c_str());
        const size_t at = meshTris_.size();
        meshTris_.resize(at + (size_t)nt * 9);
        RLGC::RlgpuCheck(rlgpu_cmf_parse(img.data(), (int64_t)img.size(), meshTris_.data() + at, nt, &nt, nullptr, nullptr),
                         f.string().c_str());
        meshObjects_.push_back(nt);
    }
    if (!files.empty()) std::printf("\tLoaded %zu collision meshes from %s\n", files.size(), sub.string().c_str());
}

inline void Learner::SyncStats() {
    rlgpu_learner_stats st{};
    RLGC::RlgpuCheck(rlgpu_learner_get_stats(h_, &st), "stats");
    totalTimesteps = (uint64_t)st.total_steps;
    totalIterations = (uint64_t)st.iteration;
}
inline void Learner::PushStats() {
    rlgpu_learner_stats st{};
    RLGC::RlgpuCheck(rlgpu_learner_get_stats(h_, &st), "stats");
    st.total_steps = (int64_t)totalTimesteps;
    st.iteration = (int64_t)totalIterations;
    RLGC::RlgpuCheck(rlgpu_learner_set_stats(h_, &st), "stats");
}

// the step hook (rlgpu_learner_set_step_hook): host plugins + the StepCallbackFn after every env step
// (EnvSet.cpp:163-255, Learner.cpp:796-797), the plugins' Reset after the arenas reset
inline int Learner::HookThunk(void* user, int32_t phase) {
    auto* L = static_cast<Learner*>(user);
    try {
        if (phase == RLGPU_HOOK_AFTER_STEP) {
            L->envSet->HostAfterStep();
            if (L->stepCallback) {
                static Report scratch;  // a StepCallbackFn outside Start()/Iterate() reports into a scratch report
                L->stepCallback(L, L->envSet->GetGameStates(), L->curReport_ ? *L->curReport_ : scratch);
            }
        } else {
            L->envSet->HostAfterReset();
        }
        return 0;
    } catch (const std::exception& e) {
        L->hookError_ = e.what();
        return 1;
    }
}

inline int64_t Learner::Iterate(Report& report) {
    SyncStats();
    const int64_t prev = (int64_t)totalTimesteps;
    const uint64_t seed = (uint64_t)config.randomSeed;
    // Learner.cpp:587-627: train against an old version with trainAgainstOldChance (picks: rlgpu_host_uniform)
    oldTeam_ = -1;
    if (config.trainAgainstOldVersions && versionMgr && !versionMgr->versions.empty()) {
        const uint64_t it = totalIterations;
        if (rlgpu_host_uniform(seed, 1, 3 * it) < config.trainAgainstOldChance) {
            const int n = (int)versionMgr->versions.size();
            const int v = std::min(n - 1, (int)(rlgpu_host_uniform(seed, 1, 3 * it + 1) * n));
            oldTeam_ = std::min(1, (int)(rlgpu_host_uniform(seed, 1, 3 * it + 2) * 2));
            RLGC::RlgpuCheck(rlgpu_ppo_set_version(ppo_, versionMgr->versions[v].params, stream_), "set old version");
            report["Old Version Timesteps"] = (double)versionMgr->versions[v].timesteps;
        }
    }
    RLGC::RlgpuCheck(rlgpu_learner_set_old_team(h_, oldTeam_), "old team");
    curReport_ = &report;
    hookError_.clear();
    rlgpu_learner_report rep{};
    const int st = rlgpu_learner_iterate(h_, &rep);
    curReport_ = nullptr;
    if (st != RLGPU_OK) {
        if (!hookError_.empty()) throw std::runtime_error("step hook: " + hookError_);
        RLGC::RlgpuCheck(st, "Learner iteration");
    }
    SyncStats();
    // PPOLearner::Learn's report (PPOLearner.cpp:537-566): metric sums over the minibatches
    float m[RLGPU_NUM_METRICS];
    int64_t cnt = 0;
    RLGC::RlgpuCheck(rlgpu_learner_metrics(h_, m, &cnt, 1), "metrics");
    if (cnt > 0) {
        report["Policy Entropy"] = m[RLGPU_M_ENTROPY] / cnt;
        report["Mean KL Divergence"] = m[RLGPU_M_KL] / cnt;
        report["Policy Loss"] = m[RLGPU_M_POLICY_LOSS] / cnt;
        report["Critic Loss"] = m[RLGPU_M_CRITIC_LOSS] / cnt;
        report["SB3 Clip Fraction"] = m[RLGPU_M_CLIP_FRACTION] / cnt;
    }
    const double steps = (double)((int64_t)totalTimesteps - prev);
    report["Collected Timesteps"] = steps;
    report["Collection Time"] = rep.collect_s;
    report["Consumption Time"] = rep.consume_s + rep.learn_s;
    report["-PPO Learn Time"] = rep.learn_s;
    report["PPO Learn Time"] = rep.learn_s;
    report["Collection Steps/Second"] = steps / std::max(rep.collect_s, 1e-9);
    report["Consumption Steps/Second"] = steps / std::max(rep.consume_s + rep.learn_s, 1e-9);
    report["Overall Steps/Second"] = steps / std::max(rep.collect_s + rep.consume_s + rep.learn_s, 1e-9);
    report["Total Timesteps"] = (double)totalTimesteps;
    report["Total Iterations"] = (double)totalIterations;
    if (versionMgr) versionMgr->OnIteration(report, (int64_t)totalTimesteps, prev);
    return prev;
}

inline void Learner::Start() {
    std::printf("Learner::Start():\n\tObs size: %d\n\tAction amount: %d\n", obsSize, numActions);
    if (options.quitKeyThread && isatty(0)) {  // StartQuitKeyThread (Learner.cpp:281-300)
        std::printf("Press 'Q' to save and quit!\n");
        std::thread([this] {
            for (int c; (c = std::getchar()) != EOF;)
                if (std::toupper(c) == 'Q') {
                    std::printf("Save queued, will save and exit next iteration.\n");
                    quitPressed_ = true;
                }
        }).detach();
    }
    for (int64_t n = 0;; n++) {
        Report report;
        const int64_t prev = Iterate(report);
        const bool quit = quitPressed_ || (options.maxIterations >= 0 && n + 1 >= options.maxIterations);
        if (quit) {  // saveQueued: save and leave (Learner.cpp:1007-1010)
            if (!config.checkpointFolder.empty()) Save();
            return;
        }
        if (!config.checkpointFolder.empty() && (int64_t)totalTimesteps / config.tsPerSave > prev / config.tsPerSave) Save();
        report.Finish();
        if (options.displayReport)
            report.Display({"Average Step Reward", "Policy Entropy", "Mean KL Divergence", "SB3 Clip Fraction", "",
                            "Policy Update Magnitude", "Critic Update Magnitude", "", "Collection Steps/Second",
                            "Consumption Steps/Second", "Overall Steps/Second", "", "Collection Time", "Consumption Time",
                            "-PPO Learn Time", "", "Collected Timesteps", "Total Timesteps", "Total Iterations"});
    }
}

inline std::vector<float> Learner::ModelParams(int model) const {
    float* params = nullptr;
    float* grads = nullptr;
    int64_t n = 0, off = 0, cnt = 0;
    RLGC::RlgpuCheck(rlgpu_ppo_buffers(ppo_, &params, &grads, &n), "buffers");
    RLGC::RlgpuCheck(rlgpu_ppo_model_range(ppo_, model, &off, &cnt), "model range");
    std::vector<float> out((size_t)cnt);
    detail::HipOk(hipStreamSynchronize(stream_), "sync");
    if (cnt) detail::HipOk(hipMemcpy(out.data(), params + off, (size_t)cnt * 4, hipMemcpyDeviceToHost), "params");
    return out;
}

// ---- checkpoints (Learner.cpp:164-279, Models.cpp:116-195) ------------------------------------------------
inline void Learner::SaveStats(const std::filesystem::path& path) {
    rlgpu_learner_stats st{};
    RLGC::RlgpuCheck(rlgpu_learner_get_stats(h_, &st), "stats");
    std::string j = "{\n    \"total_timesteps\": " + std::to_string(totalTimesteps) + ",\n    \"total_iterations\": " +
                    std::to_string(totalIterations);
    if (!runID.empty()) j += ",\n    \"run_id\": \"" + runID + "\"";
    if (config.standardizeReturns)  // WelfordStat::ToJSON
        j += ",\n    \"return_stat\": {\"mean\": " + detail::Num(st.return_mean) + ", \"var\": " + detail::Num(st.return_m2) +
             ", \"count\": " + std::to_string(st.return_n) + "}";
    if (versionMgr) versionMgr->AddRunningStatsToJSON(j);
    j += "\n}\n";
    detail::WriteFile(path, j.data(), j.size());
}

inline void Learner::LoadStats(const std::filesystem::path& path) {
    const detail::Json j = detail::ParseJson(detail::ReadFile(path));
    totalTimesteps = (uint64_t)j["total_timesteps"].Int();
    totalIterations = (uint64_t)j["total_iterations"].Int();
    if (j.Has("run_id")) runID = j["run_id"].text;
    rlgpu_learner_stats st{};
    RLGC::RlgpuCheck(rlgpu_learner_get_stats(h_, &st), "stats");
    st.total_steps = (int64_t)totalTimesteps;
    st.iteration = (int64_t)totalIterations;
    if (config.standardizeReturns && j.Has("return_stat")) {
        const detail::Json& r = j["return_stat"];
        st.return_mean = r["mean"].Num();
        st.return_m2 = r["var"].Num();
        st.return_n = r["count"].Int();
    }
    RLGC::RlgpuCheck(rlgpu_learner_set_stats(h_, &st), "stats");
    if (versionMgr) versionMgr->LoadRunningStatsFromJSON(j);
}

// <NAME>.lt of every model in `which` from flatParams (the PPO handle's flat buffer, or a version's policy +
// shared head), and with saveOptim the optimizer archives and the exact state
inline void Learner::SaveModels(const std::filesystem::path& folder, bool saveOptim, const float* flatParams,
                                const std::vector<int>& which) const {
    std::vector<float> host;
    for (const ModelSpec& m : models) {
        if (std::find(which.begin(), which.end(), m.index) == which.end()) continue;
        int64_t off = 0, cnt = 0;
        RLGC::RlgpuCheck(rlgpu_ppo_model_range(ppo_, m.index, &off, &cnt), "model range");
        if (flatParams == nullptr) {
            host = ModelParams(m.index);
        } else {  // a version: policy first, then the shared head (rlgpu_ppo_set_version's layout)
            int64_t poff = 0, pcnt = 0;
            RLGC::RlgpuCheck(rlgpu_ppo_model_range(ppo_, 0, &poff, &pcnt), "model range");
            const int64_t at = m.index == 0 ? 0 : pcnt;
            host.assign((size_t)cnt, 0.f);
            detail::HipOk(hipMemcpy(host.data(), flatParams + at, (size_t)cnt * 4, hipMemcpyDeviceToHost), "version params");
        }
        const auto tmp = detail::TempFile("params.f32");
        detail::WriteFile(tmp, host.data(), host.size() * 4);
        std::vector<std::string> a{"model-save", (folder / m.FileName()).string(), tmp.string()};
        for (auto& s : m.HelperShape()) a.push_back(s);
        try {
            detail::RunHelper(a);
        } catch (...) {
            std::filesystem::remove(tmp);
            throw;
        }
        std::filesystem::remove(tmp);
    }
    if (!saveOptim) return;
    int64_t step = 0;
    float *dm = nullptr, *dv = nullptr;
    RLGC::RlgpuCheck(rlgpu_ppo_optimizer_state(ppo_, &step, &dm, &dv), "optimizer state");
    std::map<std::string, detail::Tensor> ts;
    detail::Tensor tstep{"I64", {1}, std::vector<char>(8)};
    std::memcpy(tstep.bytes.data(), &step, 8);
    ts["step"] = tstep;
    const float lrs[3] = {config.ppo.policyLR, config.ppo.criticLR, std::min(config.ppo.policyLR, config.ppo.criticLR)};
    const bool adam = config.ppo.policy.optimType == ModelOptimType::ADAM;
    for (const ModelSpec& m : models) {
        int64_t off = 0, cnt = 0;
        RLGC::RlgpuCheck(rlgpu_ppo_model_range(ppo_, m.index, &off, &cnt), "model range");
        std::vector<float> mv((size_t)cnt * 2);
        detail::HipOk(hipMemcpy(mv.data(), dm + off, (size_t)cnt * 4, hipMemcpyDeviceToHost), "exp_avg");
        detail::HipOk(hipMemcpy(mv.data() + cnt, dv + off, (size_t)cnt * 4, hipMemcpyDeviceToHost), "exp_avg_sq");
        for (int k = 0; k < 2; k++) {
            detail::Tensor t{"F32", {cnt}, std::vector<char>((size_t)cnt * 4)};
            std::memcpy(t.bytes.data(), mv.data() + (size_t)k * cnt, (size_t)cnt * 4);
            ts[std::string(m.name) + (k ? ".exp_avg_sq" : ".exp_avg")] = std::move(t);
        }
        // <NAME>_OPTIM.lt: libtorch's own AdamW::save (Models.cpp:122-125)
        const auto tmp = detail::TempFile("optim.f32");
        detail::WriteFile(tmp, mv.data(), mv.size() * 4);
        char lr[32], wd[32];
        std::snprintf(lr, sizeof lr, "%.9g", (double)lrs[m.index]);
        std::snprintf(wd, sizeof wd, "%.9g", adam ? 0.0 : 1e-2);
        std::vector<std::string> a{"save", (folder / m.FileName("_OPTIM")).string(), tmp.string(), std::to_string(step), lr,
                                   "0.9", "0.999", "1e-08", wd};
        for (auto& s : m.ParamShapes()) a.push_back(s);
        try {
            detail::RunHelper(a);
        } catch (...) {
            std::filesystem::remove(tmp);
            throw;
        }
        std::filesystem::remove(tmp);
    }
    detail::WriteSafetensors(folder / "RLGPU_OPTIM.safetensors", ts);
}

inline void Learner::Save() {
    if (config.checkpointFolder.empty())
        throw std::runtime_error("Learner::Save(): Cannot save because config.checkpointSaveFolder is not set");
    SyncStats();
    const std::filesystem::path folder = config.checkpointFolder / std::to_string(totalTimesteps);
    std::filesystem::create_directories(folder);
    std::printf("Saving to folder %s...\n", folder.string().c_str());
    SaveStats(folder / "RUNNING_STATS.json");
    std::vector<int> all;
    for (auto& m : models) all.push_back(m.index);
    SaveModels(folder, true, nullptr, all);
    if (config.checkpointsToKeep != -1) {  // Learner.cpp:236-252
        std::set<int64_t> saved = detail::NumberedDirs(config.checkpointFolder);
        while ((int)saved.size() > config.checkpointsToKeep) {
            const int64_t low = *saved.begin();
            std::filesystem::remove_all(config.checkpointFolder / std::to_string(low));
            saved.erase(low);
        }
    }
    if (versionMgr) versionMgr->SaveVersions();
    std::printf(" > Done.\n");
}

inline void Learner::Load() {
    if (config.checkpointFolder.empty())
        throw std::runtime_error("Learner::Load(): Cannot load because config.checkpointLoadFolder is not set");
    std::printf("Loading most recent checkpoint in %s...\n", config.checkpointFolder.string().c_str());
    const std::set<int64_t> saved = detail::NumberedDirs(config.checkpointFolder);
    if (saved.empty()) {
        std::printf(" > No checkpoints found, starting new model.\n");
        return;
    }
    const std::filesystem::path folder = config.checkpointFolder / std::to_string(*saved.rbegin());
    std::printf(" > Loading checkpoint %s...\n", folder.string().c_str());
    LoadStats(folder / "RUNNING_STATS.json");
    float* params = nullptr;
    float* grads = nullptr;
    int64_t n = 0;
    RLGC::RlgpuCheck(rlgpu_ppo_buffers(ppo_, &params, &grads, &n), "buffers");
    detail::HipOk(hipStreamSynchronize(stream_), "sync");
    for (const ModelSpec& m : models) {  // Model::Load (Models.cpp:130-166), allowNotExist
        const std::filesystem::path p = folder / m.FileName();
        if (!std::filesystem::exists(p)) {
            std::printf("Warning: Model \"%s\" does not exist in %s and will be reset\n", m.name, folder.string().c_str());
            continue;
        }
        int64_t off = 0, cnt = 0;
        RLGC::RlgpuCheck(rlgpu_ppo_model_range(ppo_, m.index, &off, &cnt), "model range");
        const auto tmp = detail::TempFile("load.f32");
        std::vector<std::string> a{"model-load", p.string(), tmp.string()};
        for (auto& s : m.HelperShape()) a.push_back(s);
        detail::RunHelper(a);
        const std::string raw = detail::ReadFile(tmp);
        std::filesystem::remove(tmp);
        if ((int64_t)raw.size() != cnt * 4) throw std::runtime_error("Saved model has different size than current model: " + p.string());
        detail::HipOk(hipMemcpy(params + off, raw.data(), raw.size(), hipMemcpyHostToDevice), "load params");
    }
    RLGC::RlgpuCheck(rlgpu_ppo_refresh_half(ppo_, stream_), "refresh half");
    int64_t step = 0;
    float *dm = nullptr, *dv = nullptr;
    RLGC::RlgpuCheck(rlgpu_ppo_optimizer_state(ppo_, &step, &dm, &dv), "optimizer state");
    const std::filesystem::path st = folder / "RLGPU_OPTIM.safetensors";
    if (std::filesystem::exists(st)) {
        auto ts = detail::ReadSafetensors(st);
        for (const ModelSpec& m : models) {
            int64_t off = 0, cnt = 0;
            RLGC::RlgpuCheck(rlgpu_ppo_model_range(ppo_, m.index, &off, &cnt), "model range");
            for (int k = 0; k < 2; k++) {
                const std::string key = std::string(m.name) + (k ? ".exp_avg_sq" : ".exp_avg");
                if (!ts.count(key) || (int64_t)ts[key].bytes.size() != cnt * 4)
                    throw std::runtime_error("optimizer state in " + st.string() + " does not match the model sizes");
                detail::HipOk(hipMemcpy((k ? dv : dm) + off, ts[key].bytes.data(), (size_t)cnt * 4, hipMemcpyHostToDevice),
                              "optimizer state");
            }
        }
        int64_t s = 0;
        std::memcpy(&s, ts.at("step").bytes.data(), 8);
        RLGC::RlgpuCheck(rlgpu_ppo_set_optimizer_step(ppo_, s), "optimizer step");
    } else {  // the reference's <NAME>_OPTIM.lt archives (Models.cpp:168-186); a model without one is reset
        int64_t s = 0;
        for (const ModelSpec& m : models) {
            int64_t off = 0, cnt = 0;
            RLGC::RlgpuCheck(rlgpu_ppo_model_range(ppo_, m.index, &off, &cnt), "model range");
            const std::filesystem::path p = folder / m.FileName("_OPTIM");
            std::error_code ec;
            if (!std::filesystem::exists(p) || std::filesystem::file_size(p, ec) == 0) {
                std::printf("WARNING: No optimizer found at %s, optimizer will be reset\n", p.string().c_str());
                detail::HipOk(hipMemset(dm + off, 0, (size_t)cnt * 4), "reset");
                detail::HipOk(hipMemset(dv + off, 0, (size_t)cnt * 4), "reset");
                continue;
            }
            const auto tmp = detail::TempFile("optim.bin");
            std::vector<std::string> a{"load", p.string(), tmp.string()};
            for (auto& x : m.ParamShapes()) a.push_back(x);
            detail::RunHelper(a);
            const std::string raw = detail::ReadFile(tmp);
            std::filesystem::remove(tmp);
            if ((int64_t)raw.size() != 8 + 2 * cnt * 4) throw std::runtime_error("optimizer archive " + p.string() + " has other sizes");
            std::memcpy(&s, raw.data(), 8);
            detail::HipOk(hipMemcpy(dm + off, raw.data() + 8, (size_t)cnt * 4, hipMemcpyHostToDevice), "exp_avg");
            detail::HipOk(hipMemcpy(dv + off, raw.data() + 8 + cnt * 4, (size_t)cnt * 4, hipMemcpyHostToDevice), "exp_avg_sq");
        }
        RLGC::RlgpuCheck(rlgpu_ppo_set_optimizer_step(ppo_, s), "optimizer step");
    }
    std::printf(" > Done.\n");
}

// ---- PolicyVersionManager (PolicyVersionManager.cpp) ------------------------------------------------------
inline PolicyVersionManager::PolicyVersionManager(Learner* learner, std::filesystem::path folder, int maxV, int64_t tsPerV,
                                                  const SkillTrackerConfig& skill)
    : saveFolder(std::move(folder)), maxVersions(maxV), tsPerVersion(tsPerV), skillConfig(skill), L(learner) {
    int64_t off = 0, pc = 0, sc = 0;
    RLGC::RlgpuCheck(rlgpu_ppo_model_range(L->ppo_, 0, &off, &pc), "model range");
    RLGC::RlgpuCheck(rlgpu_ppo_model_range(L->ppo_, 2, &off, &sc), "model range");
    versionSize = pc + sc;
    if (!saveFolder.empty()) std::filesystem::create_directories(saveFolder);
    if (skillConfig.enabled && L->options.rank == 0) {  // the skill env set (PolicyVersionManager.cpp:24-31)
        rlgpu_envset_config ec{};
        ec.num_arenas = skillConfig.numArenas;
        ec.tick_skip = L->config.tickSkip;
        ec.action_delay = L->config.actionDelay;
        ec.seed = (uint64_t)L->config.randomSeed + 7919;
        static const rlgpu_reward_spec kNone{};
        static const rlgpu_terminal_spec kGoal{RLGPU_TC_GOAL_SCORE, 0.f};
        ec.rewards = &kNone;
        ec.n_rewards = 0;
        ec.terminals = &kGoal;
        ec.n_terminals = 1;
        ec.arith = L->options.arith;
        ec.state_setter = RLGPU_SS_FUZZED_KICKOFF;
        if (!L->meshTris_.empty()) {
            ec.mesh_tris = L->meshTris_.data();
            ec.mesh_ntris = (int32_t)(L->meshTris_.size() / 9);
            ec.mesh_objects = (int32_t)L->meshObjects_.size();
            ec.mesh_object_ntris = L->meshObjects_.data();
        }
        RLGC::RlgpuCheck(rlgpu_envset_create(&ec, &skillEnv), "skill env set");
        const int P = 4 * skillConfig.numArenas;
        detail::HipOk(hipMalloc(&dSkillActs, (size_t)P * 4), "skill actions");
        detail::HipOk(hipMalloc(&dOldRows, (size_t)P), "skill rows");
    }
}

inline PolicyVersionManager::~PolicyVersionManager() {
    for (auto& v : versions) (void)hipFree(v.params);
    if (skillEnv) rlgpu_envset_destroy(skillEnv);
    if (dSkillActs) (void)hipFree(dSkillActs);
    if (dOldRows) (void)hipFree(dOldRows);
}

// AddVersion (PolicyVersionManager.cpp:38-62): a copy of the current policy (+ shared head) or of dParams, the
// current ratings copied, sorted by timesteps, the oldest dropped beyond maxVersions
inline PolicyVersion& PolicyVersionManager::AddVersion(int64_t timesteps, const float* dParams) {
    PolicyVersion v;
    v.timesteps = timesteps;
    v.ratings = curRatings;
    detail::HipOk(hipMalloc(&v.params, (size_t)versionSize * 4), "version");
    if (dParams) {
        detail::HipOk(hipMemcpy(v.params, dParams, (size_t)versionSize * 4, hipMemcpyDefault), "version");
    } else {
        float* params = nullptr;
        float* grads = nullptr;
        int64_t n = 0, off = 0, pc = 0, soff = 0, sc = 0;
        RLGC::RlgpuCheck(rlgpu_ppo_buffers(L->ppo_, &params, &grads, &n), "buffers");
        RLGC::RlgpuCheck(rlgpu_ppo_model_range(L->ppo_, 0, &off, &pc), "model range");
        RLGC::RlgpuCheck(rlgpu_ppo_model_range(L->ppo_, 2, &soff, &sc), "model range");
        detail::HipOk(hipStreamSynchronize(L->stream_), "sync");
        detail::HipOk(hipMemcpy(v.params, params + off, (size_t)pc * 4, hipMemcpyDeviceToDevice), "version");
        if (sc) detail::HipOk(hipMemcpy(v.params + pc, params + soff, (size_t)sc * 4, hipMemcpyDeviceToDevice), "version");
    }
    const int64_t ts = v.timesteps;
    versions.push_back(std::move(v));
    std::stable_sort(versions.begin(), versions.end(), [](const PolicyVersion& a, const PolicyVersion& b) { return a.timesteps < b.timesteps; });
    while ((int)versions.size() > maxVersions) {
        (void)hipFree(versions.front().params);
        versions.erase(versions.begin());
    }
    for (auto& x : versions)
        if (x.timesteps == ts) return x;
    return versions.back();
}

// OnIteration (PolicyVersionManager.cpp:302-315): a version every tsPerVersion timesteps and after the first
// iteration, then the skill matches every updateInterval iterations once a version exists
inline void PolicyVersionManager::OnIteration(Report& report, int64_t total, int64_t prev) {
    if (total / tsPerVersion > prev / tsPerVersion || prev == 0) AddVersion(total);
    if (skillEnv) {
        iterationsSinceRan++;
        if (iterationsSinceRan >= skillConfig.updateInterval && !versions.empty()) {
            iterationsSinceRan = 0;
            RunSkillMatches(report);
        }
    }
}

// SaveVersions (PolicyVersionManager.cpp:64-104): <folder>/<timesteps>/POLICY.lt (+ SHARED_HEAD.lt), STATS.json;
// folders of dropped versions removed
inline void PolicyVersionManager::SaveVersions() {
    if (saveFolder.empty()) return;
    std::set<int64_t> keep;
    for (auto& v : versions) keep.insert(v.timesteps);
    const std::set<int64_t> saved = detail::NumberedDirs(saveFolder);
    for (int64_t ts : saved)
        if (!keep.count(ts)) std::filesystem::remove_all(saveFolder / std::to_string(ts));
    for (auto& v : versions) {
        if (saved.count(v.timesteps)) continue;
        const std::filesystem::path d = saveFolder / std::to_string(v.timesteps);
        std::filesystem::create_directories(d);
        L->SaveModels(d, false, v.params, {0, 2});
        const std::string j = "{\n    \"skill_ratings\": " + v.ratings.ToJSON() + "\n}\n";
        detail::WriteFile(d / "STATS.json", j.data(), j.size());
    }
}

// LoadVersions (PolicyVersionManager.cpp:106-144): refuses versions newer than the current model
inline void PolicyVersionManager::LoadVersions(int64_t cur) {
    for (auto& v : versions) (void)hipFree(v.params);
    versions.clear();
    if (saveFolder.empty()) return;
    int64_t poff = 0, pc = 0;
    RLGC::RlgpuCheck(rlgpu_ppo_model_range(L->ppo_, 0, &poff, &pc), "model range");
    for (int64_t ts : detail::NumberedDirs(saveFolder)) {
        if (ts > cur)
            throw std::runtime_error("Tried to load saved policy version that is newer than our current model (" +
                                     std::to_string(ts) + " > " + std::to_string(cur) + ")");
        const std::filesystem::path d = saveFolder / std::to_string(ts);
        std::vector<float> flat((size_t)versionSize);
        for (const ModelSpec& m : L->models) {
            if (m.index == 1) continue;
            const auto tmp = detail::TempFile("version.f32");
            std::vector<std::string> a{"model-load", (d / m.FileName()).string(), tmp.string()};
            for (auto& s : m.HelperShape()) a.push_back(s);
            detail::RunHelper(a);
            const std::string raw = detail::ReadFile(tmp);
            std::filesystem::remove(tmp);
            const size_t at = m.index == 0 ? 0 : (size_t)pc;
            if (at * 4 + raw.size() > flat.size() * 4) throw std::runtime_error("saved policy version in " + d.string() + " has another size");
            std::memcpy(flat.data() + at, raw.data(), raw.size());
        }
        PolicyVersion& v = AddVersion(ts, flat.data());
        if (std::filesystem::exists(d / "STATS.json")) {
            const detail::Json j = detail::ParseJson(detail::ReadFile(d / "STATS.json"));
            if (j.Has("skill_ratings")) v.ratings.ReadFromJSON(j["skill_ratings"]);
        }
    }
}

// RunSkillMatches (PolicyVersionManager.cpp:156-300): the current policy against a random old version on the
// skill env set (FuzzedKickoffState, GoalScoreCondition), ELO per goal in arena order in fp32, continuation of
// the same pairing while a run ends with fewer goals than arenas
inline void PolicyVersionManager::RunSkillMatches(Report& report) {
    const SkillTrackerConfig& cfg = skillConfig;
    const uint64_t seed = (uint64_t)L->config.randomSeed;
    int oldIndex, newTeam;
    float total;
    if (doContinuation) {
        oldIndex = std::min(prevOldVersionIndex, (int)versions.size() - 1);
        newTeam = prevNewTeam;
        total = prevSimTime;
    } else {
        const int n = (int)versions.size();
        oldIndex = std::min(n - 1, (int)(rlgpu_host_uniform(seed, 2, 2 * (uint64_t)skillRuns) * n));
        newTeam = std::min(1, (int)(rlgpu_host_uniform(seed, 2, 2 * (uint64_t)skillRuns + 1) * 2));
        total = 0;
        RLGC::RlgpuCheck(rlgpu_envset_reset(skillEnv, L->stream_), "skill reset");  // skill.envSet->Reset()
    }
    skillRuns++;
    doContinuation = false;
    PolicyVersion& old = versions[oldIndex];
    RLGC::RlgpuCheck(rlgpu_ppo_set_version(L->ppo_, old.params, L->stream_), "skill version");
    const int A = cfg.numArenas, P = 4 * A;
    std::vector<uint8_t> rows((size_t)P);
    for (int p = 0; p < P; p++) rows[p] = (uint8_t)(p % 2 != newTeam);  // the other team acts with the old version
    detail::HipOk(hipMemcpy(dOldRows, rows.data(), rows.size(), hipMemcpyHostToDevice), "skill rows");
    rlgpu_envset_buffers b{};
    RLGC::RlgpuCheck(rlgpu_envset_buffers_get(skillEnv, &b), "skill buffers");
    const float stepTime = (float)L->config.tickSkip * (1.0f / 120.0f);
    std::vector<rlgpu_gamestate> gs((size_t)A);
    auto elo = [&](SkillRating& winner, SkillRating& loser, const std::string& mode) {  // PolicyVersionManager.cpp:159-169
        float& w = winner.GetRating(mode, cfg.initialRating);
        float& l = loser.GetRating(mode, cfg.initialRating);
        const float expDelta = (l - w) / 400.f;
        const float expected = 1.f / (powf(10.f, expDelta) + 1.f);
        w += cfg.ratingInc * (1.f - expected);
        l += cfg.ratingInc * (expected - 1.f);  // a reference: sees the winner's update when both are the same
    };
    for (float t = 0; t < cfg.simTime && total < cfg.maxSimTime && curGoals < A; t += stepTime, total += stepTime) {
        RLGC::RlgpuCheck(rlgpu_envset_reset(skillEnv, L->stream_), "skill reset");
        RLGC::RlgpuCheck(rlgpu_envset_step_first_half(skillEnv, L->stream_), "skill step");
        RLGC::RlgpuCheck(rlgpu_ppo_infer_actions_mixed(L->ppo_, b.obs, b.action_masks, P, cfg.deterministic,
                                                       (1ull << 40) + skillSteps++, dOldRows, dSkillActs, nullptr, L->stream_),
                         "skill inference");
        RLGC::RlgpuCheck(rlgpu_envset_step_second_half(skillEnv, dSkillActs, L->stream_), "skill step");
        RLGC::RlgpuCheck(rlgpu_envset_download_gamestates(skillEnv, 0, A, gs.data(), L->stream_), "skill states");
        for (int a = 0; a < A; a++) {
            if (!gs[a].goal_scored) continue;
            std::vector<RLGC::Player> players(RLGPU_CARS);
            for (int i = 0; i < RLGPU_CARS; i++) players[i].team = (RLGC::Team)gs[a].players[i].team;
            const std::string mode = SkillRating::ModeName(players);
            const int ballTeam = gs[a].ball.pos[1] < 0 ? 0 : 1;  // RS_TEAM_FROM_Y
            if (ballTeam != newTeam) elo(curRatings, old.ratings, mode);
            else elo(old.ratings, curRatings, mode);
            curGoals++;
        }
    }
    for (auto& [mode, r] : curRatings.data) report["Rating/" + mode] = r;
    if (curGoals < A && total < cfg.maxSimTime) {
        doContinuation = true;
        prevOldVersionIndex = oldIndex;
        prevNewTeam = newTeam;
        prevSimTime = total;
    } else {
        curGoals = 0;
    }
}

}  // namespace GGL
