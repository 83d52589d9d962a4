// facade_test.cpp -- checks of EnvSetGPU.hpp's plugin translation and host fallback (tests/test_facade.py).
//
//   facade_test translate   (CPU) ExampleMain's EnvCreateFunc (src/ExampleMain.cpp:128-226) written against
//                           RLGC.hpp translates to exactly rlgpu_envset_default_plugins' registry lists; user
//                           classes, subclasses of registry classes and ZeroSumReward over a user class go to
//                           the host; fields the registry cannot hold and foreign builders are refused.
//   facade_test learner     (GPU) two trainer-facade GGL::Learners (GigaLearn.hpp) on the same seed: one whose
//                           EnvCreateFn gives registry classes (the fused env step), one with the user classes
//                           on the host plus a StepCallbackFn (the hooked step): the same parameters bit for bit
//                           after every iteration, and the callback saw every step's GameStates.
//   facade_test fallback    (GPU) two env sets in lockstep on the same seed and actions: one whose plugins are
//                           all registry classes, one where user classes restating the same rewards and
//                           conditions run on the host.  Rewards, terminals and obs must agree bit for bit over
//                           every step, resets included; a reward reading isFinal sees the merged terminal.
#include <cstdio>
#include <cstring>
#include <random>

#include "GigaLearn.hpp"

using namespace RLGC;

static int g_fail = 0;
#define CHECK(c, ...)                                        \
    do {                                                     \
        if (!(c)) {                                          \
            std::printf("FAIL %s:%d: ", __FILE__, __LINE__); \
            std::printf(__VA_ARGS__);                        \
            std::printf("\n");                               \
            g_fail++;                                        \
        }                                                    \
    } while (0)

// ---- user plugins (what a GigaLearnCPP user writes) ----
class MySpeedReward : public Reward {  // SpeedReward's body (CommonRewards.h:100-105), a user class
  public:
    float GetReward(const Player& player, const GameState&, bool) override { return player.vel.Length() / 2300.f; }
};
class MyTouchBallReward : public Reward {
  public:
    int resets = 0;
    void Reset(const GameState&) override { resets++; }
    float GetReward(const Player& player, const GameState&, bool) override { return player.ballTouchedStep; }
};
class MyAirReward : public AirReward {  // a subclass of a registry class is the user's own: host
  public:
    float GetReward(const Player& player, const GameState&, bool) override { return !player.isOnGround; }
};
class FinalFlagReward : public Reward {
  public:
    float GetReward(const Player&, const GameState&, bool isFinal) override { return isFinal ? 1.f : 0.f; }
};
class MyNoTouchCondition : public TerminalCondition {  // NoTouchCondition.h's body
  public:
    float timeSinceTouch = 0, maxTime;
    explicit MyNoTouchCondition(float t) : maxTime(t) {}
    void Reset(const GameState&) override { timeSinceTouch = 0; }
    bool IsTerminal(const GameState& s) override {
        for (auto& p : s.players)
            if (p.ballTouchedStep) {
                timeSinceTouch = 0;
                return false;
            }
        timeSinceTouch += s.deltaTime;
        return timeSinceTouch >= maxTime;
    }
    bool IsTruncation() override { return true; }
};
class MyGoalCondition : public TerminalCondition {
  public:
    bool IsTerminal(const GameState& s) override { return s.goalScored; }
    bool IsTruncation() override { return false; }
};
class MyObs : public ObsBuilder {};

// src/ExampleMain.cpp:128-226 against RLGC.hpp
static EnvCreateResult ExampleMainEnv(int) {
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
    EnvCreateResult r;
    r.rewards = rewards;
    r.terminalConditions = {new NoTouchCondition(8), new ScoreLimitCondition(3)};
    r.actionParser = new DefaultAction();
    r.obsBuilder = new AdvancedObs();
    r.stateSetter = new KickoffState();
    return r;
}

static void FreeResult(EnvCreateResult& r) {
    for (auto& w : r.rewards) delete w.reward;
    for (auto* t : r.terminalConditions) delete t;
    delete r.obsBuilder;
    delete r.actionParser;
    delete r.stateSetter;
}

static bool SameSpec(const rlgpu_reward_spec& a, const rlgpu_reward_spec& b) {
    return std::memcmp(&a, &b, sizeof a) == 0;
}

static int Translate() {
    // ExampleMain == the registry's default lists, byte for byte
    EnvCreateResult ex = ExampleMainEnv(0);
    PluginPlan p = TranslatePlugins(ex);
    rlgpu_reward_spec rw[RLGPU_MAX_REWARDS];
    rlgpu_terminal_spec tc[RLGPU_MAX_TERMINALS];
    std::memset(rw, 0, sizeof rw);
    std::memset(tc, 0, sizeof tc);
    int32_t nr = 0, nt = 0;
    RlgpuCheck(rlgpu_envset_default_plugins(rw, &nr, tc, &nt), "default plugins");
    CHECK(!p.HasHost(), "ExampleMain has a host plugin");
    CHECK((int)p.deviceRewards.size() == nr, "%zu rewards vs %d", p.deviceRewards.size(), nr);
    for (int i = 0; i < nr && i < (int)p.deviceRewards.size(); i++) {
        const auto& a = p.deviceRewards[i];
        CHECK(SameSpec(a, rw[i]), "reward %d: type %d/%d weight %g/%g params %g,%g,%g / %g,%g,%g zs %d/%d ts %g/%g os %g/%g", i,
              a.type, rw[i].type, a.weight, rw[i].weight, a.params[0], a.params[1], a.params[2], rw[i].params[0],
              rw[i].params[1], rw[i].params[2], a.zero_sum, rw[i].zero_sum, a.zero_sum_team_spirit,
              rw[i].zero_sum_team_spirit, a.zero_sum_opponent_scale, rw[i].zero_sum_opponent_scale);
    }
    CHECK((int)p.deviceTerminals.size() == nt, "%zu terminals vs %d", p.deviceTerminals.size(), nt);
    for (int i = 0; i < nt && i < (int)p.deviceTerminals.size(); i++)
        CHECK(p.deviceTerminals[i].type == tc[i].type && p.deviceTerminals[i].param == tc[i].param, "terminal %d", i);
    for (int i = 0; i < (int)p.rewardSlot.size(); i++) CHECK(p.rewardSlot[i] == i, "slot %d", i);
    FreeResult(ex);

    // every registry class with non-default fields
    {
        EnvCreateResult r;
        r.rewards = {{new VelocityReward(true), 1.f},        {new VelocityBallToGoalReward(true), 2.f},
                     {new SaveBoostReward(0.25f), 3.f},      {new GoalReward(-0.5f), 4.f},
                     {new BumpedPenalty(), 5.f},             {new DemoedPenalty(), 6.f},
                     {new FaceBallReward(), 7.f},            {new TouchBallReward(), 8.f},
                     {new SpeedReward(), 9.f},               {new StrongTouchReward(13.7f, 171.3f), 10.f},
                     {new ZeroSumReward(new SpeedReward(), 0.3f, 0.7f), 11.f}};
        r.terminalConditions = {new GoalScoreCondition(), new NoTouchCondition(2.5f), new ScoreLimitCondition(5)};
        PluginPlan q = TranslatePlugins(r);
        const int want[] = {RLGPU_RW_VELOCITY, RLGPU_RW_VELOCITY_BALL_TO_GOAL, RLGPU_RW_SAVE_BOOST, RLGPU_RW_GOAL,
                            RLGPU_RW_BUMPED_PENALTY, RLGPU_RW_DEMOED_PENALTY, RLGPU_RW_FACE_BALL, RLGPU_RW_TOUCH_BALL,
                            RLGPU_RW_SPEED, RLGPU_RW_STRONG_TOUCH, RLGPU_RW_SPEED};
        CHECK(q.deviceRewards.size() == 11 && !q.HasHost(), "registry classes");
        for (int i = 0; i < 11 && i < (int)q.deviceRewards.size(); i++) {
            CHECK(q.deviceRewards[i].type == want[i], "type %d", i);
            CHECK(q.deviceRewards[i].weight == (float)(i + 1), "weight %d", i);
        }
        if (q.deviceRewards.size() == 11) {
            CHECK(q.deviceRewards[0].params[0] == 1.f && q.deviceRewards[1].params[0] == 1.f, "bool params");
            CHECK(q.deviceRewards[2].params[0] == 0.25f && q.deviceRewards[3].params[0] == -0.5f, "float params");
            // the device multiplies the kph back by 250/9: the stored speeds must come back exactly
            CHECK(q.deviceRewards[9].params[0] * (250.f / 9.f) == Math::KPHToVel(13.7f) &&
                      q.deviceRewards[9].params[1] * (250.f / 9.f) == Math::KPHToVel(171.3f), "strong touch speeds");
            CHECK(q.deviceRewards[10].zero_sum == 1 && q.deviceRewards[10].zero_sum_team_spirit == 0.3f &&
                      q.deviceRewards[10].zero_sum_opponent_scale == 0.7f, "zero sum");
        }
        CHECK(q.deviceTerminals.size() == 3 && q.deviceTerminals[0].type == RLGPU_TC_GOAL_SCORE &&
                  q.deviceTerminals[1].param == 2.5f && q.deviceTerminals[2].param == 5.f, "terminals");
        FreeResult(r);
    }
    // every kph whose KPHToVel a StrongTouchReward stores comes back through the registry exactly
    {
        std::mt19937 rng(3);
        std::uniform_real_distribution<float> U(0.f, 400.f);
        int bad = 0;
        for (int i = 0; i < 200000; i++) {
            float k = U(rng);
            float v = Math::KPHToVel(k);
            if (detail::KphFromVel(v, "x") * (250.f / 9.f) != v) bad++;
        }
        CHECK(bad == 0, "%d kph values do not round trip", bad);
    }
    // user classes go to the host, in place in the list
    {
        EnvCreateResult r;
        r.rewards = {{new AirReward(), 1.f}, {new MySpeedReward(), 2.f}, {new MyAirReward(), 3.f},
                     {new ZeroSumReward(new MySpeedReward(), 1), 4.f}, {new ZeroSumReward(new AirReward(), 1), 5.f}};
        r.terminalConditions = {new MyNoTouchCondition(3), new GoalScoreCondition(), new MyGoalCondition()};
        PluginPlan q = TranslatePlugins(r);
        CHECK((q.rewardSlot == std::vector<int>{0, -1, -1, -1, 1}), "reward slots");
        CHECK(q.NumHostRewards() == 3 && q.deviceRewards.size() == 2, "host rewards");
        CHECK((q.hostTerminals == std::vector<int>{0, 2}) && q.deviceTerminals.size() == 1, "host terminals");
        CHECK(q.hostNames.size() == 5, "names");
        FreeResult(r);
    }
    // KickoffProximityReward2v2Enhanced's tunables are device parameters (goerReward, rotationPrepWeight)
    {
        EnvCreateResult r;
        auto* k = new KickoffProximityReward2v2Enhanced();
        k->goerReward = 2.f;
        k->rotationPrepWeight = 0.35f;
        r.rewards = {{k, 1.f}, {new KickoffProximityReward2v2Enhanced(), 2.f}};
        PluginPlan q = TranslatePlugins(r);
        CHECK(!q.HasHost() && q.deviceRewards.size() == 2, "kickoff tunables");
        if (q.deviceRewards.size() == 2) {
            CHECK(q.deviceRewards[0].params[0] == 2.f && q.deviceRewards[0].params[1] == 0.35f &&
                      q.deviceRewards[0].params[2] == 1.f, "kickoff tunables in params");
            CHECK(q.deviceRewards[1].params[2] == 0.f, "default kickoff tunables are the registry's zero params");
        }
        FreeResult(r);
    }
    // the arena an EnvCreateFn builds must be the device's: 2v2 SOCCAR, Octanes added blue, orange, blue, orange
    {
        auto arena = [](GameMode mode, std::vector<Team> teams, const CarConfig& car = CAR_CONFIG_OCTANE) {
            Arena* a = Arena::Create(mode);
            for (Team t : teams) a->AddCar(t, car);
            return a;
        };
        const std::vector<Team> ok2v2 = {Team::BLUE, Team::ORANGE, Team::BLUE, Team::ORANGE};
        struct Case {
            Arena* a;
            const char* why;
        } bad[] = {{arena(GameMode::SOCCAR, {Team::BLUE, Team::ORANGE}), "1v1"},
                   {arena(GameMode::HOOPS, ok2v2), "HOOPS"},
                   {arena(GameMode::SOCCAR, {Team::BLUE, Team::BLUE, Team::ORANGE, Team::ORANGE}), "team order"},
                   {arena(GameMode::SOCCAR, ok2v2, CAR_CONFIG_DOMINUS), "Dominus"},
                   {Arena::Create(GameMode::SOCCAR, {}, 60), "60 Hz"}};
        for (auto& c : bad) {
            bool threw = false;
            try {
                RequireDeviceArena(c.a, 3);
            } catch (const std::invalid_argument& e) {
                threw = std::string(e.what()).find("EnvCreateFn(3)") != std::string::npos;
            }
            CHECK(threw, "arena accepted: %s", c.why);
            delete c.a;
        }
        Arena* good = arena(GameMode::SOCCAR, ok2v2);
        bool threw = false;
        try {
            RequireDeviceArena(good, 0);
        } catch (const std::exception&) {
            threw = true;
        }
        CHECK(!threw, "ExampleMain's 2v2 arena refused");
        delete good;
    }
    // refused: foreign builders, differing arenas
    {
        bool threw = false;
        EnvCreateResult o;
        o.obsBuilder = new MyObs();
        threw = false;
        try {
            TranslatePlugins(o);
        } catch (const std::invalid_argument&) {
            threw = true;
        }
        CHECK(threw, "foreign obs builder accepted");
        FreeResult(o);
        EnvCreateResult a = ExampleMainEnv(0), b = ExampleMainEnv(1);
        static_cast<GoalReward*>(static_cast<ZeroSumReward*>(b.rewards[11].reward)->child)->concedeScale = -2;
        threw = false;
        try {
            RequireSamePlan(TranslatePlugins(a), TranslatePlugins(b), 1);
        } catch (const std::invalid_argument&) {
            threw = true;
        }
        CHECK(threw, "differing arenas accepted");
        FreeResult(a);
        FreeResult(b);
    }
    std::printf("translate: %s\n", g_fail ? "FAILED" : "ok");
    return g_fail ? 1 : 0;
}

// ---- GPU: registry plugins vs the same plugins as user classes on the host ----
static EnvCreateResult DeviceEnv(int) {
    EnvCreateResult r;
    r.rewards = {{new SpeedReward(), 2.f}, {new AirReward(), 0.5f}, {new TouchBallReward(), 3.f},
                 {new ZeroSumReward(new GoalReward(), 1), 150.f}};
    r.terminalConditions = {new NoTouchCondition(3.0f), new GoalScoreCondition()};
    return r;
}
static EnvCreateResult HostEnv(int) {
    EnvCreateResult r;
    r.rewards = {{new MySpeedReward(), 2.f}, {new AirReward(), 0.5f}, {new MyTouchBallReward(), 3.f},
                 {new ZeroSumReward(new GoalReward(), 1), 150.f}};
    r.terminalConditions = {new MyNoTouchCondition(3.0f), new MyGoalCondition()};
    return r;
}
static EnvCreateResult FinalEnv(int) {
    EnvCreateResult r;
    r.rewards = {{new FinalFlagReward(), 1.f}};
    r.terminalConditions = {new NoTouchCondition(0.75f)};
    return r;
}

static int Fallback(int arenas, int steps) {
    EnvSetConfig ca{DeviceEnv, arenas, 8, 7, false};
    EnvSetConfig cb{HostEnv, arenas, 8, 7, false};
    EnvSetConfig cf{FinalEnv, arenas, 8, 7, false};
    EnvSetGPUOptions opt;
    opt.seed = 99;
    EnvSetGPU A(ca, opt), B(cb, opt), F(cf, opt);
    CHECK(!A.plan.HasHost(), "device set has host plugins");
    CHECK(B.fallbackStats.hostRewards == 2 && B.fallbackStats.hostTerminals == 2, "host plugin counts %d %d",
          B.fallbackStats.hostRewards, B.fallbackStats.hostTerminals);
    CHECK(F.fallbackStats.hostRewards == 1 && F.fallbackStats.hostTerminals == 0, "final set counts");
    const int P = A.state.num_players;
    int32_t* dAct = nullptr;
    RlgpuCheckHip(hipMalloc(&dAct, (size_t)P * sizeof(int32_t)), "actions");
    std::vector<int32_t> act(P);
    std::mt19937 rng(17);
    std::vector<float> ra(P), rb(P), rf(P), oa((size_t)P * RLGPU_OBS), ob((size_t)P * RLGPU_OBS);
    std::vector<uint8_t> ta(arenas), tb(arenas), tf(arenas);
    long terminals = 0, normal = 0, touches = 0, goals = 0;
    auto obs_equal = [&](const char* when, int step) {
        RlgpuCheckHip(hipMemcpy(oa.data(), A.state.obs, oa.size() * 4, hipMemcpyDeviceToHost), "obs");
        RlgpuCheckHip(hipMemcpy(ob.data(), B.state.obs, ob.size() * 4, hipMemcpyDeviceToHost), "obs");
        CHECK(std::memcmp(oa.data(), ob.data(), oa.size() * 4) == 0, "obs differ %s step %d", when, step);
    };
    for (int s = 0; s < steps && !g_fail; s++) {
        // mostly full throttle + boost straight ahead (DefaultAction row 18): kickoff cars face the ball, so
        // touches, goals and no-touch timeouts all happen
        for (auto& x : act) x = (int32_t)(rng() % 10 < 7 ? 18 : rng() % RLGPU_ACTIONS);
        RlgpuCheckHip(hipMemcpy(dAct, act.data(), act.size() * 4, hipMemcpyHostToDevice), "actions");
        for (EnvSetGPU* e : {&A, &B, &F}) {
            e->StepFirstHalf(false);
            e->StepSecondHalf(dAct, false);
        }
        RlgpuCheckHip(hipMemcpy(ra.data(), A.state.rewards, P * 4, hipMemcpyDeviceToHost), "rewards");
        RlgpuCheckHip(hipMemcpy(rb.data(), B.state.rewards, P * 4, hipMemcpyDeviceToHost), "rewards");
        RlgpuCheckHip(hipMemcpy(rf.data(), F.state.rewards, P * 4, hipMemcpyDeviceToHost), "rewards");
        RlgpuCheckHip(hipMemcpy(ta.data(), A.state.terminals, arenas, hipMemcpyDeviceToHost), "terminals");
        RlgpuCheckHip(hipMemcpy(tb.data(), B.state.terminals, arenas, hipMemcpyDeviceToHost), "terminals");
        RlgpuCheckHip(hipMemcpy(tf.data(), F.state.terminals, arenas, hipMemcpyDeviceToHost), "terminals");
        int bad_r = 0, bad_t = 0, bad_f = 0;
        for (int i = 0; i < P; i++) bad_r += std::memcmp(&ra[i], &rb[i], 4) != 0;
        for (int a = 0; a < arenas; a++) {
            bad_t += ta[a] != tb[a];
            terminals += ta[a] != 0;
            normal += ta[a] == NORMAL;
            for (int i = 0; i < 4; i++) bad_f += rf[a * 4 + i] != (tf[a] ? 1.f : 0.f);
        }
        for (auto& gs : B.gameStates) {
            for (auto& p : gs.players) touches += p.ballTouchedStep;
            goals += gs.goalScored;
        }
        CHECK(bad_r == 0, "step %d: %d rewards differ (first: %d)", s, bad_r, [&] {
            for (int i = 0; i < P; i++)
                if (ra[i] != rb[i]) return i;
            return -1;
        }());
        CHECK(bad_t == 0, "step %d: %d terminals differ", s, bad_t);
        CHECK(bad_f == 0, "step %d: %d isFinal rewards disagree with the terminals", s, bad_f);
        obs_equal("after the step", s);
        for (EnvSetGPU* e : {&A, &B, &F}) e->Reset();
        obs_equal("after the reset", s);
    }
    // GameStates for a StepCallbackFn: the device-only set's download equals the host set's plugin view
    const auto& ga = A.GetGameStates();
    const auto& gb = B.GetGameStates();
    int bad_g = 0;
    for (int a = 0; a < arenas; a++)
        for (int i = 0; i < 4; i++) {
            const Player &p = ga[a].players[i], &q = gb[a].players[i];
            bad_g += !(p.pos == q.pos && p.vel == q.vel && p.boost == q.boost && p.carId == q.carId && p.team == q.team);
        }
    CHECK(bad_g == 0, "%d players differ between GetGameStates of the two sets", bad_g);
    uint64_t resets = 0;
    for (auto& r : B.results) resets += static_cast<MyTouchBallReward*>(r.rewards[2].reward)->resets;
    CHECK(resets == (uint64_t)arenas + (uint64_t)terminals, "plugin Reset calls %llu, expected %ld",
          (unsigned long long)resets, arenas + terminals);
    CHECK(terminals > 0 && touches > 0, "no terminals (%ld) or touches (%ld) exercised", terminals, touches);
    (void)hipFree(dAct);
    std::printf("fallback: %d arenas x %d steps, %ld terminals (%ld normal), %ld touches, %ld goal steps; host steps %llu, "
                "reward calls %llu, terminal calls %llu, resets %llu: %s\n",
                arenas, steps, terminals, normal, touches, goals, (unsigned long long)B.fallbackStats.steps,
                (unsigned long long)B.fallbackStats.rewardCalls, (unsigned long long)B.fallbackStats.terminalCalls,
                (unsigned long long)B.fallbackStats.resetCalls, g_fail ? "FAILED" : "ok");
    return g_fail ? 1 : 0;
}

// ---- GPU: the trainer facade with host plugins + a StepCallbackFn vs the registry-only Learner ----
static int LearnerMode(int arenas, int iters) {
    using namespace GGL;
    LearnerConfig cfg = {};
    cfg.numGames = arenas;
    cfg.randomSeed = 7;
    cfg.ppo.tsPerItr = 24 * 4 * arenas;
    cfg.ppo.batchSize = cfg.ppo.tsPerItr;
    cfg.ppo.miniBatchSize = cfg.ppo.tsPerItr / 2;
    cfg.ppo.maxEpisodeDuration = 2.0;
    cfg.ppo.sharedHead.layerSizes = {64};
    cfg.ppo.policy.layerSizes = {64, 64};
    cfg.ppo.critic.layerSizes = {64, 64};
    for (PartialModelConfig* m : {&cfg.ppo.policy, &cfg.ppo.critic, &cfg.ppo.sharedHead}) {
        m->activationType = ModelActivationType::LEAKY_RELU;
        m->optimType = ModelOptimType::ADAMW;
    }
    cfg.checkpointFolder.clear();
    cfg.trainAgainstOldVersions = false;
    cfg.sendMetrics = false;
    LearnerGPUOptions o;
    o.quitKeyThread = false;
    o.displayReport = false;
    uint64_t calls = 0, players = 0;
    Learner A(DeviceEnv, cfg, nullptr, o);
    Learner B(HostEnv, cfg,
              [&](Learner*, const std::vector<GameState>& states, Report& report) {
                  calls++;
                  for (auto& s : states)
                      for (auto& p : s.players) {
                          players++;
                          report.AddAvg("Player/Speed", p.vel.Length());
                      }
              },
              o);
    CHECK(B.envSet->plan.HasHost(), "the user classes did not go to the host");
    for (int it = 0; it < iters && !g_fail; it++) {
        Report ra, rb;
        A.Iterate(ra);
        B.Iterate(rb);
        CHECK(A.totalTimesteps == B.totalTimesteps, "iteration %d: %llu vs %llu timesteps", it,
              (unsigned long long)A.totalTimesteps, (unsigned long long)B.totalTimesteps);
        for (auto& m : A.models) {
            const std::vector<float> a = A.ModelParams(m.index), b = B.ModelParams(m.index);
            int bad = 0;
            for (size_t i = 0; i < a.size(); i++) bad += std::memcmp(&a[i], &b[i], 4) != 0;
            CHECK(a.size() == b.size() && bad == 0, "iteration %d: %s: %d of %zu parameters differ", it, m.name, bad, a.size());
        }
        rb.Finish();
        CHECK(rb.Has("Player/Speed"), "the StepCallbackFn's report is missing");
    }
    CHECK(calls > 0 && players == calls * (uint64_t)arenas * 4, "callback calls %llu, players %llu",
          (unsigned long long)calls, (unsigned long long)players);
    std::printf("learner: %d arenas x %d iterations, %llu timesteps, %llu callback calls, host reward calls %llu: %s\n",
                arenas, iters, (unsigned long long)A.totalTimesteps, (unsigned long long)calls,
                (unsigned long long)B.envSet->fallbackStats.rewardCalls, g_fail ? "FAILED" : "ok");
    return g_fail ? 1 : 0;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::printf("usage: facade_test translate | fallback [arenas] [steps] | learner [arenas] [iterations]\n");
        return 2;
    }
    try {
        if (!std::strcmp(argv[1], "translate")) return Translate();
        if (!std::strcmp(argv[1], "learner"))
            return LearnerMode(argc > 2 ? std::atoi(argv[2]) : 64, argc > 3 ? std::atoi(argv[3]) : 2);
        if (!std::strcmp(argv[1], "fallback"))
            return Fallback(argc > 2 ? std::atoi(argv[2]) : 256, argc > 3 ? std::atoi(argv[3]) : 300);
    } catch (const std::exception& e) {
        std::printf("FAIL: exception %s\n", e.what());
        return 1;
    }
    return 2;
}
