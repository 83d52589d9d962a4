"""Old policy versions for self-play -- Python mirror of GGL::PolicyVersionManager.

Reference map:
    PolicyVersionManager::AddVersion      PolicyVersionManager.cpp:38-62 (clone, sort by timesteps,
                                          drop the oldest beyond maxVersions)
    PolicyVersionManager::OnIteration     PolicyVersionManager.cpp:302-315 (a version every
                                          tsPerVersion timesteps, and after the first iteration)
    PolicyVersionManager::SaveVersions    PolicyVersionManager.cpp:64-104 (<checkpoint>/policy_versions/
                                          <timesteps>/POLICY.lt + STATS.json, stale dirs removed)
    PolicyVersionManager::LoadVersions    PolicyVersionManager.cpp:106-144 (refuses versions newer than
                                          the current model)
    LearnerConfig                         LearnerConfig.h:62-68 (tsPerVersion 25M, maxOldVersions 32,
                                          trainAgainstOldVersions, trainAgainstOldChance 0.15)

Versions are the policy's flat fp32 parameters -- followed by the shared head's when the model has
one, as the reference versions GetPolicyModels() (PPOLearner.cpp:665-674) and saves POLICY.lt +
SHARED_HEAD.lt per version -- kept in HBM (1.6 MB each at [512, 512]); the active
one is converted once per iteration into the PPO handle's second bf16 inference copy
(rlgpu_ppo_set_version) and used by the mixed-policy inference of the Learner.  With a skill tracker
(rlgpu.skill, LearnerConfig.skill_tracker) every version carries its ELO ratings (a copy of the current
ratings when it is added, PolicyVersionManager.cpp:47), STATS.json stores them under "skill_ratings", and
OnIteration runs the skill matches every update_interval iterations (PolicyVersionManager.cpp:302-315).
"""
import json
import os
import shutil

from . import checkpoint as _ckpt
from .skill import SkillRating


class PolicyVersion:
    def __init__(self, timesteps, params, ratings=None):
        self.timesteps = int(timesteps)
        self.params = params            # device tensor, flat fp32 policy (+ shared head) parameters
        self.ratings = ratings.copy() if isinstance(ratings, SkillRating) else SkillRating(ratings)


class PolicyVersionManager:
    def __init__(self, ppo, save_folder=None, max_versions=32, ts_per_version=25_000_000, skill=None):
        self.ppo = ppo
        self.skill = skill  # rlgpu.skill.SkillTracker or None
        self.save_folder = save_folder
        self.max_versions = max_versions
        self.ts_per_version = ts_per_version
        self.versions = []
        if save_folder:
            os.makedirs(save_folder, exist_ok=True)

    def add_version(self, timesteps, params=None):
        """AddVersion: a copy of the current policy (or of `params`)."""
        src = self.ppo.policy_version() if params is None else params
        v = PolicyVersion(timesteps, src.detach().clone(), self.skill.cur_ratings if self.skill is not None else None)
        self.versions.append(v)
        self.versions.sort(key=lambda x: x.timesteps)
        while len(self.versions) > self.max_versions:
            self.versions.pop(0)
        return v

    def on_iteration(self, total_timesteps, prev_timesteps, report=None):
        """OnIteration: a version every ts_per_version timesteps (and after the first iteration), then the skill
        matches every update_interval iterations once a version exists."""
        if total_timesteps // self.ts_per_version > prev_timesteps // self.ts_per_version or prev_timesteps == 0:
            self.add_version(total_timesteps)
        if self.skill is not None and self.skill.cfg.enabled:
            self.skill.iterations_since_ran += 1
            if self.skill.iterations_since_ran >= self.skill.cfg.update_interval and self.versions:
                self.skill.iterations_since_ran = 0
                self.skill.run(self.versions, report)

    def save_versions(self):
        if not self.save_folder:
            return
        keep = {v.timesteps for v in self.versions}
        saved = _ckpt.numbered_dirs(self.save_folder)
        for ts in saved - keep:
            shutil.rmtree(os.path.join(self.save_folder, str(ts)))
        for v in self.versions:
            if v.timesteps in saved:
                continue
            d = os.path.join(self.save_folder, str(v.timesteps))
            os.makedirs(d, exist_ok=True)
            import torch
            flat = v.params.detach().cpu()
            o = 0
            for mi in self._models():  # ModelSet::Save(folder, false): no optimizer files
                seq = self.ppo.torch_module(mi)
                with torch.no_grad():
                    for p in seq.parameters():
                        p.copy_(flat[o:o + p.numel()].view_as(p))
                        o += p.numel()
                _ckpt.write_model(seq, _ckpt.model_path(d, _ckpt.MODEL_NAMES[mi]))
            with open(os.path.join(d, "STATS.json"), "w") as f:
                json.dump({"skill_ratings": v.ratings.to_json()}, f, indent=4)

    def _models(self):
        return [m for m in self.ppo.models if m != 1]  # GetPolicyModels: policy (+ shared head)

    def load_versions(self, cur_timesteps):
        import torch
        self.versions = []
        if not self.save_folder:
            return
        for ts in sorted(_ckpt.numbered_dirs(self.save_folder)):
            if ts > cur_timesteps:
                raise ValueError(f"Tried to load saved policy version that is newer than our current model "
                                 f"({ts} > {cur_timesteps})")
            d = os.path.join(self.save_folder, str(ts))
            parts = []
            for mi in self._models():
                tensors = _ckpt.read_model_state(_ckpt.model_path(d, _ckpt.MODEL_NAMES[mi]))
                if [t.numel() for t in tensors] != self.ppo.model_sizes(mi):
                    raise ValueError(f"saved policy version in {d} has a different size than the current model")
                parts += [t.reshape(-1) for t in tensors]
            flat = torch.cat(parts).to(self.ppo.params.device)
            v = self.add_version(ts, flat)
            p = os.path.join(d, "STATS.json")
            if os.path.exists(p):
                with open(p) as f:
                    v.ratings = SkillRating.from_json(json.load(f).get("skill_ratings", {}))
