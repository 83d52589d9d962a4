// RLGC.hpp -- the reference's env-plugin interface, restated for code that builds against this library without
// the reference tree: the types an EnvCreateFn returns (RG/EnvSet/EnvSet.h:14-24), the GameState / Player
// records the plugins read (RG/Gamestates/GameState.h, Player.h over RocketSim's CarState / BallState,
// RS/Sim/Car/Car.h:17-100, RS/Sim/Ball/Ball.h:17-42, RS/Math/MathTypes/MathTypes.h), the Reward /
// TerminalCondition plugin bases (RG/Rewards/Reward.h:7-96, RG/TerminalConditions/TerminalCondition.h) and the
// classes of the device registry with their public constructor fields (RG/Rewards/CommonRewards.h,
// KickoffProximityReward2v2Enhanced.h, ZeroSumReward.h, NoTouchCondition.h, GoalScoreCondition.h and
// src/ExampleMain.cpp:46-124).
//
// Same names, same members, same virtuals, so an EnvCreateFn written for the reference compiles here unchanged
// and EnvSetGPU.hpp compiles against either header set.  The registry classes carry no GetReward / IsTerminal
// body: the device evaluates them (EnvSetGPU translates them to rlgpu_reward_spec / rlgpu_terminal_spec).  A
// class of the user's own -- anything the translator's dynamic_casts do not recognise -- runs on the host,
// through its own virtuals, exactly as EnvSet::StepSecondHalf calls them (EnvSet.cpp:163-250).
//
// The arena an EnvCreateFn builds (RocketSim's Arena::Create / AddCar, RS/Sim/Arena/Arena.h:71,111) is restated as
// a record of what was asked for -- game mode, tick rate, cars (team, config), mutators -- which the facade
// checks against the one arena the kernels simulate (2v2 SOCCAR, Octanes added blue, orange, blue, orange at
// 120 Hz) and refuses with a named error otherwise.
//
// RLGPU_FACADE_USER_EXAMPLEMAIN_CLASSES: the including translation unit defines its own ScoreLimitCondition /
// LosingPenaltyReward, as src/ExampleMain.cpp:46-124 does: they are then the user's classes (host plugins through
// their own virtuals), not this header's registry declarations.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <functional>
#include <iostream>
#include <memory>
#include <stdexcept>
#include <string>
#include <typeinfo>
#include <vector>

// RocketSim's Framework.h helpers
#ifndef RS_MAX
#define RS_MAX(a, b) ((a) > (b) ? (a) : (b))
#define RS_MIN(a, b) ((a) < (b) ? (a) : (b))
#endif

namespace RLGC {

typedef std::vector<float> FList;  // RG/BasicTypes/Lists.h
typedef std::vector<int> IList;

// RocketSim's Vec (MathTypes.h:8-160): float components, Length = sqrtf(x*x + y*y + z*z), Normalized safe
struct Vec {
    float x = 0, y = 0, z = 0, _w = 0;
    Vec() = default;
    Vec(float x, float y, float z) : x(x), y(y), z(z) {}
    float LengthSq() const { return x * x + y * y + z * z; }
    float Length() const { return sqrtf(LengthSq()); }
    float LengthSq2D() const { return x * x + y * y; }
    float Length2D() const { return sqrtf(LengthSq2D()); }
    float Dot(const Vec& o) const { return x * o.x + y * o.y + z * o.z; }
    Vec Cross(const Vec& o) const { return {y * o.z - z * o.y, z * o.x - x * o.z, x * o.y - y * o.x}; }
    float DistSq(const Vec& o) const { return (*this - o).LengthSq(); }
    float Dist(const Vec& o) const { return sqrtf(DistSq(o)); }
    float DistSq2D(const Vec& o) const {
        float dx = x - o.x, dy = y - o.y;
        return dx * dx + dy * dy;
    }
    float Dist2D(const Vec& o) const { return sqrtf(DistSq2D(o)); }
    Vec Normalized() const {
        float l = Length();
        return l > 1.1920929e-07f * 1.1920929e-07f ? *this / l : Vec();
    }
    float& operator[](uint32_t i) { return (&x)[i]; }
    float operator[](uint32_t i) const { return (&x)[i]; }
    Vec operator+(const Vec& o) const { return {x + o.x, y + o.y, z + o.z}; }
    Vec operator-(const Vec& o) const { return {x - o.x, y - o.y, z - o.z}; }
    Vec operator*(const Vec& o) const { return {x * o.x, y * o.y, z * o.z}; }
    Vec operator/(const Vec& o) const { return {x / o.x, y / o.y, z / o.z}; }
    Vec operator*(float v) const { return {x * v, y * v, z * v}; }
    Vec operator/(float v) const { return {x / v, y / v, z / v}; }
    Vec& operator+=(const Vec& o) { return *this = *this + o; }
    Vec& operator-=(const Vec& o) { return *this = *this - o; }
    Vec& operator*=(float v) { return *this = *this * v; }
    Vec& operator/=(float v) { return *this = *this / v; }
    Vec operator-() const { return {-x, -y, -z}; }
    bool operator==(const Vec& o) const { return x == o.x && y == o.y && z == o.z; }
    bool operator!=(const Vec& o) const { return !(*this == o); }
};

// RocketSim's RotMat: the basis columns forward, right, up (MathTypes.h:162-260)
struct RotMat {
    Vec forward, right, up;
    static RotMat GetIdentity() { return {Vec(1, 0, 0), Vec(0, 1, 0), Vec(0, 0, 1)}; }
    Vec operator[](uint32_t i) const { return (&forward)[i]; }
    Vec& operator[](uint32_t i) { return (&forward)[i]; }
    Vec Dot(const Vec& v) const { return {v.Dot(forward), v.Dot(right), v.Dot(up)}; }
};

enum class Team : uint8_t { BLUE = 0, ORANGE = 1 };
#define RS_TEAM_FROM_Y(y) ((y) < 0 ? RLGC::Team::BLUE : RLGC::Team::ORANGE)

// ---- the arena an EnvCreateFn asks for (RS/Sim/GameMode.h, Arena.h, CarConfig.h) ----
enum class GameMode : uint8_t { SOCCAR, HOOPS, HEATSEEKER, SNOWDAY, DROPSHOT, THE_VOID };
struct CarConfig {  // the preset the hitbox and wheels come from (CarConfig.h:21-43)
    int preset;
    const char* name;
};
inline const CarConfig CAR_CONFIG_OCTANE{0, "Octane"}, CAR_CONFIG_DOMINUS{1, "Dominus"}, CAR_CONFIG_PLANK{2, "Plank"},
    CAR_CONFIG_BREAKOUT{3, "Breakout"}, CAR_CONFIG_HYBRID{4, "Hybrid"}, CAR_CONFIG_MERC{5, "Merc"};
struct MutatorConfig {};
struct ArenaConfig {};
struct Car {
    uint32_t id = 0;
    Team team = Team::BLUE;
    CarConfig config = CAR_CONFIG_OCTANE;
};
class Arena {
  public:
    GameMode gameMode = GameMode::SOCCAR;
    float tickRate = 120;
    bool mutatorsSet = false;
    std::vector<std::unique_ptr<Car>> cars;
    static Arena* Create(GameMode mode, const ArenaConfig& = {}, float tickRate = 120) {
        auto* a = new Arena();
        a->gameMode = mode;
        a->tickRate = tickRate;
        return a;
    }
    Car* AddCar(Team team, const CarConfig& config = CAR_CONFIG_OCTANE) {
        cars.emplace_back(new Car{(uint32_t)cars.size() + 1, team, config});  // car ids start at 1 (Arena.cpp)
        return cars.back().get();
    }
    void SetMutatorConfig(const MutatorConfig&) { mutatorsSet = true; }
    std::vector<Car*> GetCars() const {
        std::vector<Car*> v;
        for (auto& c : cars) v.push_back(c.get());
        return v;
    }
};

// The arena the kernels simulate: 2v2 SOCCAR at 120 Hz, Octanes added blue, orange, blue, orange (creation order
// is the player order: team of player p = p % 2).  Throws std::invalid_argument naming what differs.
inline void RequireDeviceArena(const Arena* a, int index) {
    if (!a) return;  // no arena: the device's own
    auto fail = [&](const std::string& what) {
        throw std::invalid_argument("EnvCreateFn(" + std::to_string(index) + "): " + what +
                                    " (the device simulates 2v2 SOCCAR at 120 Hz with Octanes added blue, orange, "
                                    "blue, orange)");
    };
    if (a->gameMode != GameMode::SOCCAR) fail("game mode " + std::to_string((int)a->gameMode) + " is not SOCCAR");
    if (a->tickRate != 120.f) fail("tick rate " + std::to_string(a->tickRate) + " is not 120");
    if (a->mutatorsSet) fail("mutators are set");
    if (a->cars.size() != 4) fail(std::to_string(a->cars.size()) + " cars instead of 4");
    for (size_t i = 0; i < a->cars.size(); i++) {
        if (a->cars[i]->team != (i % 2 ? Team::ORANGE : Team::BLUE))
            fail("car " + std::to_string(i) + " is on the wrong team for the blue, orange, blue, orange order");
        if (a->cars[i]->config.preset != CAR_CONFIG_OCTANE.preset)
            fail(std::string("car ") + std::to_string(i) + " is a " + a->cars[i]->config.name + ", not an Octane");
    }
}

struct CarControls {  // RS/Sim/CarControls.h:7-20
    float throttle = 0, steer = 0, pitch = 0, yaw = 0, roll = 0;
    bool jump = false, boost = false, handbrake = false;
};

struct BallHitInfo {  // RS/Sim/BallHitInfo/BallHitInfo.h:9-26
    bool isValid = false;
    Vec relativePosOnBall, ballPos, extraHitVel;
    uint64_t tickCountWhenHit = ~0ULL;
    uint64_t tickCountWhenExtraImpulseApplied = ~0ULL;
};

struct PhysState {  // RS/Sim/PhysState/PhysState.h
    Vec pos;
    RotMat rotMat = RotMat::GetIdentity();
    Vec vel, angVel;
};

struct BallState : PhysState {
    uint64_t updateCounter = 0;
};

struct CarState : PhysState {  // RS/Sim/Car/Car.h:17-100
    uint64_t updateCounter = 0;
    bool isOnGround = true;
    bool wheelsWithContact[4] = {};
    bool hasJumped = false, hasDoubleJumped = false, hasFlipped = false;
    Vec flipRelTorque;
    float jumpTime = 0, flipTime = 0;
    bool isFlipping = false, isJumping = false;
    float airTime = 0, airTimeSinceJump = 0;
    float boost = 100.f / 3.f;
    float timeSpentBoosting = 0;
    bool isSupersonic = false;
    float supersonicTime = 0, handbrakeVal = 0;
    bool isAutoFlipping = false;
    float autoFlipTimer = 0, autoFlipTorqueScale = 0;
    struct {
        bool hasContact = false;
        Vec contactNormal;
    } worldContact;
    struct {
        uint32_t otherCarID = 0;
        float cooldownTimer = 0;
    } carContact;
    bool isDemoed = false;
    float demoRespawnTimer = 0;
    BallHitInfo ballHitInfo;
    CarControls lastControls;
};

struct Action {  // RG/BasicTypes/Action.h
    float throttle = 0, steer = 0, pitch = 0, yaw = 0, roll = 0, jump = 0, boost = 0, handbrake = 0;
    constexpr static size_t ELEM_AMOUNT = 8;
    float& operator[](size_t i) { return (&throttle)[i]; }
    float operator[](size_t i) const { return (&throttle)[i]; }
};

struct PlayerEventState {  // RG/Gamestates/Player.h:6-12
    bool goal = false, save = false, assist = false, shot = false, shotPass = false;
    bool bump = false, bumped = false, demo = false, demoed = false;
};

struct Player : CarState {  // RG/Gamestates/Player.h:14-33
    Player* prev = nullptr;
    int index = -1;
    uint32_t carId = 0;
    Team team = Team::BLUE;
    PlayerEventState eventState = {};
    bool ballTouchedStep = false;
    bool ballTouchedTick = false;
    Action prevAction = {};
};

struct GameState {  // RG/Gamestates/GameState.h:19-74
    GameState* prev = nullptr;
    float deltaTime = 0;
    bool goalScored = false;
    int lastTouchCarID = -1;
    std::vector<Player> players;
    BallState ball;
    std::vector<bool> boostPads, boostPadsInv;
    std::vector<float> boostPadTimers, boostPadTimersInv;
    void* lastArena = nullptr;  // the device holds the arena: always null here
    uint64_t lastTickCount = 0;
    void* userInfo = nullptr;

    const std::vector<bool>& GetBoostPads(bool inverted) const { return inverted ? boostPadsInv : boostPads; }
    // the reference returns the opposite array here (GameState.h:60); kept, since plugins see it that way
    const std::vector<float>& GetBoostPadTimers(bool inverted) const {
        return inverted ? boostPadTimers : boostPadTimersInv;
    }
    bool IsEmpty() const { return players.empty(); }
    void MakeEmpty() { players.clear(); }
};

// ---- plugin bases (Reward.h:7-96, TerminalCondition.h) ----
class Reward {
  public:
    virtual void Reset(const GameState& initialState) {}
    virtual void PreStep(const GameState& state) {}
    virtual float GetReward(const Player& player, const GameState& state, bool isFinal) {
        throw std::runtime_error("GetReward() is unimplemented");
    }
    virtual std::vector<float> GetAllRewards(const GameState& state, bool isFinal) {
        std::vector<float> out(state.players.size());
        for (size_t i = 0; i < out.size(); i++) out[i] = GetReward(state.players[i], state, isFinal);
        return out;
    }
    virtual void GetAllRewardsInPlace(const GameState& state, bool isFinal, float* output) {
        for (size_t i = 0; i < state.players.size(); i++) output[i] = GetReward(state.players[i], state, isFinal);
    }
    virtual const std::vector<float>* GetInnerRewards() const { return nullptr; }
    virtual std::string GetName() {
        std::string n = typeid(*this).name();
        size_t i = n.rfind("::");
        return i == std::string::npos ? n : n.substr(i + 2);
    }
    virtual ~Reward() {}
};

struct WeightedReward {
    Reward* reward;
    float weight;
    WeightedReward(Reward* reward, float scale) : reward(reward), weight(scale) {}
    WeightedReward(Reward* reward, int scale) : reward(reward), weight((float)scale) {}
};

enum TerminalType { NOT_TERMINAL, NORMAL, TRUNCATED };

class TerminalCondition {
  public:
    virtual void Reset(const GameState& initialState) {}
    virtual bool IsTerminal(const GameState& currentState) = 0;
    virtual bool IsTruncation() = 0;
    virtual ~TerminalCondition() {}
};

// RewardWrapper.h / ZeroSumReward.h: the hot path calls GetAllRewardsInPlace, which ZeroSumReward does not
// override, so the wrapper forwards GetReward to its child
class RewardWrapper : public Reward {
  public:
    Reward* child;
    explicit RewardWrapper(Reward* child) : child(child) {}
    ~RewardWrapper() override { delete child; }
    void Reset(const GameState& s) override { child->Reset(s); }
    void PreStep(const GameState& s) override { child->PreStep(s); }
    float GetReward(const Player& p, const GameState& s, bool f) override { return child->GetReward(p, s, f); }
    std::string GetName() override { return child->GetName(); }
};

class ZeroSumReward : public RewardWrapper {
  public:
    float teamSpirit, opponentScale;
    ZeroSumReward(Reward* child, float teamSpirit, float opponentScale = 1, bool ownsFunc = true)
        : RewardWrapper(child), teamSpirit(teamSpirit), opponentScale(opponentScale) {}
};

// ---- the device registry's classes (fields as the reference declares them) ----
template <bool PlayerEventState::*VAR, bool NEGATIVE>
class PlayerDataEventReward : public Reward {};
typedef PlayerDataEventReward<&PlayerEventState::bump, false> BumpReward;
typedef PlayerDataEventReward<&PlayerEventState::bumped, true> BumpedPenalty;
typedef PlayerDataEventReward<&PlayerEventState::demo, false> DemoReward;
typedef PlayerDataEventReward<&PlayerEventState::demoed, true> DemoedPenalty;

namespace Math {
constexpr float KPHToVel(float kph) { return kph * (250.f / 9.f); }
constexpr float VelToKPH(float vel) { return vel / (250.f / 9.f); }
}  // namespace Math

class GoalReward : public Reward {
  public:
    float concedeScale;
    GoalReward(float concedeScale = -1) : concedeScale(concedeScale) {}
};
class VelocityReward : public Reward {
  public:
    bool isNegative;
    VelocityReward(bool isNegative = false) : isNegative(isNegative) {}
};
class VelocityBallToGoalReward : public Reward {
  public:
    bool ownGoal = false;
    VelocityBallToGoalReward(bool ownGoal = false) : ownGoal(ownGoal) {}
};
class VelocityPlayerToBallReward : public Reward {};
class FaceBallReward : public Reward {};
class TouchBallReward : public Reward {};
class SpeedReward : public Reward {};
class WavedashReward : public Reward {};
class PickupBoostReward : public Reward {};
class SaveBoostReward : public Reward {
  public:
    float exponent;
    SaveBoostReward(float exponent = 0.5f) : exponent(exponent) {}
};
class AirReward : public Reward {};
class TouchAccelReward : public Reward {};
class StrongTouchReward : public Reward {
  public:
    float minRewardedVel, maxRewardedVel;
    StrongTouchReward(float minSpeedKPH = 20, float maxSpeedKPH = 130) {
        minRewardedVel = Math::KPHToVel(minSpeedKPH);
        maxRewardedVel = Math::KPHToVel(maxSpeedKPH);
    }
};
class KickoffProximityReward2v2Enhanced : public Reward {
  public:
    float goerReward = 1.2f, cheaterReward = 0.6f, dynamicWeight = 0.3f, rotationPrepWeight = 0.2f;
};
#ifndef RLGPU_FACADE_USER_EXAMPLEMAIN_CLASSES
// src/ExampleMain.cpp:84-124 (its fields are private there; a translator in the reference tree needs them
// public or an accessor -- INTEGRATION.md section 3)
class LosingPenaltyReward : public Reward {
  public:
    explicit LosingPenaltyReward(float penaltyPerGoalBehind = 0.01f) : penaltyScale(penaltyPerGoalBehind) {}
    float penaltyScale;
    int blueScore = 0, orangeScore = 0;
};
#endif

class NoTouchCondition : public TerminalCondition {
  public:
    float timeSinceTouch = 0;
    float maxTime;
    NoTouchCondition(float maxTime) : maxTime(maxTime) {}
    bool IsTerminal(const GameState&) override { throw std::logic_error("NoTouchCondition runs on the device"); }
    bool IsTruncation() override { return true; }
};
class GoalScoreCondition : public TerminalCondition {
  public:
    bool IsTerminal(const GameState& s) override { return s.goalScored; }
    bool IsTruncation() override { return false; }
};
#ifndef RLGPU_FACADE_USER_EXAMPLEMAIN_CLASSES
// src/ExampleMain.cpp:46-82
class ScoreLimitCondition : public TerminalCondition {
  public:
    explicit ScoreLimitCondition(int limitGoals) : limit(limitGoals) {}
    bool IsTerminal(const GameState&) override { throw std::logic_error("ScoreLimitCondition runs on the device"); }
    bool IsTruncation() override { return false; }
    int limit;
    int blueScore = 0, orangeScore = 0;
};
#endif

// ---- builders the kernels implement (AdvancedObs.cpp, DefaultAction.cpp, KickoffState.cpp) ----
class ObsBuilder {
  public:
    virtual ~ObsBuilder() {}
};
class ActionParser {
  public:
    virtual ~ActionParser() {}
};
class StateSetter {
  public:
    virtual ~StateSetter() {}
};
class AdvancedObs : public ObsBuilder {};
class DefaultObs : public ObsBuilder {};        // RG/ObsBuilders/DefaultObs.h (declared; the kernels build AdvancedObs)
class DefaultAction : public ActionParser {};
class KickoffState : public StateSetter {};
class RandomState : public StateSetter {        // RG/StateSetters/RandomState.h (declared; not a device state setter)
  public:
    bool randBallSpeed = true, randCarSpeed = true, carsOnGround = true;
    RandomState(bool randBallSpeed = true, bool randCarSpeed = true, bool carsOnGround = true)
        : randBallSpeed(randBallSpeed), randCarSpeed(randCarSpeed), carsOnGround(carsOnGround) {}
};
class FuzzedKickoffState : public StateSetter {  // RG/StateSetters/FuzzedKickoffState.h
  public:
    constexpr static float FUZZ_POS_RANGE = 0.1f;
};

struct EnvCreateResult {  // RG/EnvSet/EnvSet.h:14-24
    Arena* arena = nullptr;  // checked by RequireDeviceArena; null = the device's 2v2 SOCCAR arena
    std::vector<WeightedReward> rewards;
    std::vector<TerminalCondition*> terminalConditions;
    ObsBuilder* obsBuilder = nullptr;
    ActionParser* actionParser = nullptr;
    StateSetter* stateSetter = nullptr;
    void* userInfo = nullptr;
};
typedef std::function<EnvCreateResult(int index)> EnvCreateFn;

struct EnvSetConfig {  // RG/EnvSet/EnvSet.h:27-34
    EnvCreateFn envCreateFn;
    int numArenas;
    int tickSkip;
    int actionDelay;
    bool saveRewards;
    bool shuffleRewardSampling = true;
};

}  // namespace RLGC

// RocketSim::Init (RS/RocketSim.cpp:12-100): the collision meshes of a folder of .cmf files.  The facade keeps the
// folder; the Learner loads its meshes into the env set when it exists (rlgpu_cmf_parse), else the built-in arena.
namespace RocketSim {
using RLGC::Arena;
using RLGC::CarConfig;
using RLGC::GameMode;
using RLGC::Team;
inline std::string& MeshFolder() {
    static std::string folder;
    return folder;
}
inline void Init(const std::filesystem::path& collisionMeshesFolder, bool silent = false) {
    MeshFolder() = collisionMeshesFolder.string();
    if (!silent && !std::filesystem::is_directory(collisionMeshesFolder))
        std::fprintf(stderr, "RocketSim::Init: no collision mesh folder at \"%s\": the built-in arena mesh is used\n",
                     MeshFolder().c_str());
}
}  // namespace RocketSim
