"""Reward / terminal-condition registry of the env set (include/rlgpu_env.h rlgpu_reward_spec /
rlgpu_terminal_spec) -- the Python face of the EnvCreateFn's plugin lists
(GigaLearnCPP/RLGymCPP/src/RLGymCPP/EnvSet/EnvSet.h:14-24; src/ExampleMain.cpp:128-226).

    from rlgpu.plugins import reward, zero_sum, terminal
    rewards = [reward("AirReward", 0.25), zero_sum(reward("GoalReward", 150), 1), ...]
    terminals = [terminal("NoTouchCondition", 8), terminal("ScoreLimitCondition", 3)]
    EnvSet(4096, rewards=rewards, terminals=terminals)

Names are the reference's class names; positional parameters are their constructor arguments, with
the reference's defaults.  A class the device registry does not hold (a user's own C++ plugin) has
no device code: it is refused here, and a raw unknown type id is refused by rlgpu_envset_create
(RLGPU_ERR_UNSUPPORTED with the id in rlgpu_last_error()).
"""
import numpy as np

REWARD_SPEC = np.dtype([("type", "<i4"), ("weight", "<f4"), ("params", "<f4", 3), ("zero_sum", "<i4"),
                        ("zero_sum_team_spirit", "<f4"), ("zero_sum_opponent_scale", "<f4")])
TERMINAL_SPEC = np.dtype([("type", "<i4"), ("param", "<f4")])
MAX_REWARDS, MAX_TERMINALS = 32, 8

# class name -> (RLGPU_RW_* id, constructor defaults)   (RG/Rewards/CommonRewards.h, ExampleMain.cpp:84-124)
REWARDS = {
    "AirReward": (0, ()),
    "WavedashReward": (1, ()),
    "KickoffProximityReward2v2Enhanced": (2, ()),
    "VelocityPlayerToBallReward": (3, ()),
    "StrongTouchReward": (4, (20.0, 130.0)),        # minSpeedKPH, maxSpeedKPH
    "TouchAccelReward": (5, ()),
    "VelocityBallToGoalReward": (6, (False,)),      # ownGoal
    "PickupBoostReward": (7, ()),
    "SaveBoostReward": (8, (0.5,)),                 # exponent
    "BumpReward": (9, ()),
    "DemoReward": (10, ()),
    "GoalReward": (11, (-1.0,)),                    # concedeScale
    "LosingPenaltyReward": (12, (0.01,)),           # penaltyPerGoalBehind
    "BumpedPenalty": (13, ()),
    "DemoedPenalty": (14, ()),
    "VelocityReward": (15, (False,)),               # isNegative
    "FaceBallReward": (16, ()),
    "TouchBallReward": (17, ()),
    "SpeedReward": (18, ()),
}
# class name -> (RLGPU_TC_* id, needs a parameter)   (RG/TerminalConditions/, ExampleMain.cpp:46-82)
TERMINALS = {"NoTouchCondition": (0, True), "ScoreLimitCondition": (1, True), "GoalScoreCondition": (2, False)}


class UnknownPlugin(KeyError):
    pass


# KickoffProximityReward2v2Enhanced's public tunables (KickoffProximityReward2v2Enhanced.h:9-12): the two its
# GetReward reads (:135, :175) are device parameters; cheaterReward / dynamicWeight are never read
KICKOFF_TUNABLES = {"goer_reward": 1.2, "rotation_prep_weight": 0.2}


def reward(name, weight, *params, **tunables):
    """WeightedReward{new <name>(*params), weight}.  KickoffProximityReward2v2Enhanced also takes the keyword
    tunables goer_reward / rotation_prep_weight (its member fields; defaults 1.2 / 0.2)."""
    if tunables:
        if name != "KickoffProximityReward2v2Enhanced" or set(tunables) - set(KICKOFF_TUNABLES):
            raise TypeError(f"{name} takes no keyword tunables {sorted(tunables)}")
        t = dict(KICKOFF_TUNABLES, **tunables)
        r = reward(name, weight)
        if (np.float32(t["goer_reward"]), np.float32(t["rotation_prep_weight"])) != (np.float32(1.2), np.float32(0.2)):
            r["params"][:] = (t["goer_reward"], t["rotation_prep_weight"], 1.0)
        return r
    if name not in REWARDS:
        raise UnknownPlugin(f"reward class {name!r} has no device implementation (registry: {sorted(REWARDS)})")
    rid, defaults = REWARDS[name]
    if len(params) > max(len(defaults), 0):
        raise TypeError(f"{name} takes {len(defaults)} constructor arguments")
    args = list(params) + list(defaults[len(params):])
    r = np.zeros((), REWARD_SPEC)
    r["type"], r["weight"] = rid, weight
    for i, v in enumerate(args):
        r["params"][i] = float(v)
    return r


def zero_sum(spec, team_spirit, opponent_scale=1.0):
    """ZeroSumReward(child, teamSpirit, opponentScale) around a reward(...) spec.  On the training
    hot path it is a pass-through, as in the reference (ZeroSumReward.cpp:3-48 overrides only
    GetAllRewards; EnvSet calls GetAllRewardsInPlace)."""
    r = spec.copy()
    r["zero_sum"], r["zero_sum_team_spirit"], r["zero_sum_opponent_scale"] = 1, team_spirit, opponent_scale
    return r


def terminal(name, param=None):
    if name not in TERMINALS:
        raise UnknownPlugin(f"terminal condition {name!r} has no device implementation (registry: {sorted(TERMINALS)})")
    tid, needs = TERMINALS[name]
    if needs and param is None:
        raise TypeError(f"{name} needs its constructor argument")
    t = np.zeros((), TERMINAL_SPEC)
    t["type"], t["param"] = tid, 0.0 if param is None else float(param)
    return t


def rewards_array(specs):
    a = np.array([np.asarray(s, REWARD_SPEC) for s in specs], REWARD_SPEC) if len(specs) else np.zeros(0, REWARD_SPEC)
    return np.ascontiguousarray(a)


def terminals_array(specs):
    a = np.array([np.asarray(s, TERMINAL_SPEC) for s in specs], TERMINAL_SPEC) if len(specs) else np.zeros(0, TERMINAL_SPEC)
    return np.ascontiguousarray(a)


def example_main():
    """ExampleMain's EnvCreateFunc lists (src/ExampleMain.cpp:132-187)."""
    rw = [reward("AirReward", 0.25), reward("WavedashReward", 0.12), reward("KickoffProximityReward2v2Enhanced", 5.0),
          reward("VelocityPlayerToBallReward", 4.0), reward("StrongTouchReward", 60, 20, 120),
          reward("TouchAccelReward", 6.0), zero_sum(reward("VelocityBallToGoalReward", 8.0), 1),
          reward("PickupBoostReward", 0.1), reward("SaveBoostReward", 0.010), zero_sum(reward("BumpReward", 20), 0.5),
          zero_sum(reward("DemoReward", 80), 0.5), zero_sum(reward("GoalReward", 150), 1),
          reward("LosingPenaltyReward", 1.0, 0.02)]
    tc = [terminal("NoTouchCondition", 8), terminal("ScoreLimitCondition", 3)]
    return rewards_array(rw), terminals_array(tc)
