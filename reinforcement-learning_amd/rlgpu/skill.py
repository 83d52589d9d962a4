"""Skill (ELO) tracking of the current policy against its old versions -- Python mirror of GigaLearnCPP's
SkillTrackerConfig (src/public/GigaLearnCPP/SkillTrackerConfig.h), SkillRating (PolicyVersionManager.h:12-52)
and PolicyVersionManager::RunSkillMatches / OnIteration (PolicyVersionManager.cpp:156-315).

The skill env set is its own rlgpu.EnvSet on the device: the Learner's arena setup with no rewards,
FuzzedKickoffState (include/rlgpu_env.h RLGPU_SS_FUZZED_KICKOFF) and GoalScoreCondition
(PolicyVersionManager.cpp:24-31).  A match step is the reference's: Reset (the arenas whose goal ended
them), StepFirstHalf, one mixed-policy inference over every player -- the current policy for the new team's
players, the old version (rlgpu_ppo_set_version) for the other team's (rlgpu_ppo_infer_actions_mixed; the
reference runs the two models on index-selected rows, PPOLearner::InferActionsFromModels) -- and
StepSecondHalf; every arena whose GameState has goalScored then updates the two ratings with ELO math in arena
order, in fp32 as the reference computes them.  The random picks (old version, new team) are the library's
counter-based host draws (rlgpu_host_uniform, stream 2: the C++ facade's PolicyVersionManager makes the same
picks) in place of RocketSim's Math::RandInt; the policy's multinomial draws use the PPO handle's Philox
stream on a step range of their own (2^40 + k: the step's high bits are folded into the Philox key, so these
uniforms never repeat the rollout's).
"""
import numpy as np

from . import env as _env
from . import plugins as _plugins

TICK_TIME = np.float32(1.0 / 120.0)  # RLGC::CommonValues::TICK_TIME


class SkillTrackerConfig:
    """SkillTrackerConfig.h (defaults as there)."""

    def __init__(self, **kw):
        self.enabled = False
        self.num_arenas = 16        # arenas of the skill env set
        self.sim_time = 45.0        # seconds simulated per run
        self.max_sim_time = 240.0   # seconds a continued run may last before the games are reset
        self.update_interval = 16   # iterations between runs
        self.rating_inc = 5.0       # ELO increment scale per goal
        self.initial_rating = 0.0   # rating of a mode seen for the first time
        self.deterministic = False  # argmax policies (off: the stochastic policy is what PPO optimises)
        for k, v in kw.items():
            if not hasattr(self, k):
                raise AttributeError(f"unknown SkillTrackerConfig field {k}")
            setattr(self, k, v)


class SkillRating:
    """Ratings per game mode name ("2v2"), fp32 (PolicyVersionManager.h:12-52)."""

    def __init__(self, data=None):
        self.data = {k: np.float32(v) for k, v in (data or {}).items()}

    @staticmethod
    def mode_name(teams):
        """GetModeName: "<players on the smaller team>v<players on the larger>"."""
        n = [0, 0]
        for t in teams:
            n[int(t)] += 1
        return f"{min(n)}v{max(n)}"

    def get(self, name, default):
        """GetRating: inserts the default for a new mode."""
        if name not in self.data:
            self.data[name] = np.float32(default)
        return self.data[name]

    def set(self, name, v):
        self.data[name] = np.float32(v)

    def copy(self):
        return SkillRating(self.data)

    def to_json(self):
        return {k: float(v) for k, v in self.data.items()}

    @classmethod
    def from_json(cls, j):
        return cls(j)


def elo_update(winner, loser, mode, rating_inc, initial_rating):
    """fnUpdateRatings (PolicyVersionManager.cpp:159-169) in fp32: expected = 1 / (10^((l - w) / 400) + 1);
    winner += inc * (1 - expected), loser += inc * (expected - 1).  winner and loser may be the same object
    (a version against itself)."""
    f = np.float32
    w = winner.get(mode, initial_rating)
    lo = loser.get(mode, initial_rating)
    exp_delta = f(f(lo - w) / f(400))
    expected = f(f(1) / f(np.power(f(10), exp_delta) + f(1)))
    winner.set(mode, f(w + f(f(rating_inc) * f(f(1) - expected))))
    lo = loser.get(mode, initial_rating)  # GetRating returns a reference: re-read after the winner's update
    loser.set(mode, f(lo + f(f(rating_inc) * f(expected - f(1)))))


class SkillTracker:
    """The skill half of PolicyVersionManager: the skill env set, the current ratings and the continuation
    state between runs."""

    RNG_STEP_BASE = 1 << 40  # Philox counter range of the matches' policy draws (the rollout uses small steps)

    def __init__(self, cfg, ppo, device, tick_skip=8, action_delay=7, seed=0, mesh=None, arith=0):
        self.cfg = cfg
        self.ppo = ppo
        self.device = device
        self.env = _env.EnvSet(cfg.num_arenas, seed=seed + 7919, tick_skip=tick_skip, action_delay=action_delay,
                               save_rewards=False, device=device, rewards=[],
                               terminals=[_plugins.terminal("GoalScoreCondition")], mesh=mesh, arith=arith,
                               state_setter=_env.FUZZED_KICKOFF_STATE)
        self.cur_ratings = SkillRating()
        self.cur_goals = 0
        self.do_continuation = False
        self.prev_old_version_index = 0
        self.prev_new_team = 0
        self.prev_sim_time = np.float32(0)
        self.iterations_since_ran = 0
        self.seed = seed
        self.runs = 0  # rlgpu_host_uniform counter: run r draws 2 r (version) and 2 r + 1 (team)
        self.steps_run = 0
        self.log = []  # (old version index, new team, goal events) per run, for reports and tests

    def close(self):
        self.env.close()

    def run(self, versions, report=None, on_step=None):
        """RunSkillMatches over `versions` (rlgpu.versions.PolicyVersion list, ratings updated in place).
        on_step(actions, old_rows) is called after each step's inference (tests)."""
        import torch
        cfg, E = self.cfg, self.env
        f = np.float32
        if self.do_continuation:
            assert self.prev_old_version_index < len(versions)
            old_index, new_team, total = self.prev_old_version_index, self.prev_new_team, f(self.prev_sim_time)
        else:
            from .learner import host_uniform
            n = len(versions)
            old_index = min(n - 1, int(host_uniform(self.seed, 2, 2 * self.runs) * n))
            new_team = min(1, int(host_uniform(self.seed, 2, 2 * self.runs + 1) * 2))
            total = f(0)
            E.reset()
        self.runs += 1
        self.do_continuation = False
        old = versions[old_index]
        self.ppo.set_version(old.params)
        # players of team new_team act with the current policy, the others with the old version
        team = torch.arange(E.num_players, device=self.device) % 2
        old_rows = (team != new_team).to(torch.uint8)
        prev_ratings = self.cur_ratings.copy()
        goals = []
        step_time = f(f(E.tick_skip) * TICK_TIME)
        t = f(0)
        while t < f(cfg.sim_time) and total < f(cfg.max_sim_time) and self.cur_goals < E.num_arenas:
            E.reset()
            E.step_first_half()
            actions, _ = self.ppo.infer_actions_mixed(E.obs, E.action_masks, old_rows,
                                                      step=self.RNG_STEP_BASE + self.steps_run,
                                                      deterministic=cfg.deterministic)
            self.steps_run += 1
            if on_step is not None:
                on_step(actions, old_rows)
            E.step_second_half(actions)
            gs = E.gamestates()
            for i in np.nonzero(gs["goal_scored"])[0]:
                teams = gs["players"]["team"][i]
                mode = SkillRating.mode_name(teams)
                ball_team = 0 if gs["ball"]["pos"][i][1] < 0 else 1  # RS_TEAM_FROM_Y
                if ball_team != new_team:
                    elo_update(self.cur_ratings, old.ratings, mode, cfg.rating_inc, cfg.initial_rating)
                else:
                    elo_update(old.ratings, self.cur_ratings, mode, cfg.rating_inc, cfg.initial_rating)
                goals.append((int(i), ball_team != new_team))
                self.cur_goals += 1
            t = f(t + step_time)
            total = f(total + step_time)
        if report is not None:
            for mode, r in self.cur_ratings.data.items():
                report["Rating/" + mode] = float(r)
        changes = {m: float(r) - float(prev_ratings.get(m, cfg.initial_rating)) for m, r in self.cur_ratings.data.items()}
        if self.cur_goals < E.num_arenas and total < f(cfg.max_sim_time):
            # not enough goals: the same pairing continues from the end position next run
            self.do_continuation = True
            self.prev_old_version_index = old_index
            self.prev_new_team = new_team
            self.prev_sim_time = total
        else:
            self.cur_goals = 0
        self.log.append({"old_version": old_index, "new_team": new_team, "goals": goals, "rating_changes": changes,
                         "sim_time": float(total), "continuation": self.do_continuation})
        return goals
