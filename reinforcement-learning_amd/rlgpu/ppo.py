"""PPO actor/critic over the C ABI of include/rlgpu_ppo.h -- the Python mirror of
GGL::PPOLearner (GigaLearnCPP/src/private/GigaLearnCPP/PPO/PPOLearner.h:41-59) and
GGL::Model (Util/Models.h:21-163).

Method map (reference -> here):
    Model(name, ModelConfig)                         -> part of PPO(...) (policy = 0, critic = 1,
                                                        shared_head = 2 when shared_layers is given)
    PPOLearner::InferActions(obs, masks, ...)        -> infer_actions(obs, masks, step)
    PPOLearner::InferCritic / InferCriticBatched     -> infer_critic(obs)
    PPOLearner::Learn per-minibatch body (:341-475)  -> minibatch(...)
    clip_grad_norm_ + ModelSet::StepOptims (:521-529)-> optimizer_step()
    Model::CopyParams / parameters()                 -> params (flat fp32 device tensor), model_slice()
"""
import ctypes
import math

from . import _lib
from ._lib import alias

MAX_LAYERS = 8
NUM_METRICS = 16
METRICS = ("entropy", "kl", "policy_loss", "critic_loss", "ratio", "clip_fraction", "count",
           "grad_norm_policy", "grad_norm_critic", "grad_norm_shared")
MODEL_NAMES = ("policy", "critic", "shared_head")  # GGL::Model::modelName (PPOLearner.cpp:66-72)


class _Cfg(ctypes.Structure):
    _fields_ = [("obs_size", ctypes.c_int32), ("num_actions", ctypes.c_int32),
                ("policy_layers", ctypes.c_int32 * MAX_LAYERS), ("n_policy_layers", ctypes.c_int32),
                ("critic_layers", ctypes.c_int32 * MAX_LAYERS), ("n_critic_layers", ctypes.c_int32),
                ("layer_norm", ctypes.c_int32), ("leaky_slope", ctypes.c_float),
                ("policy_lr", ctypes.c_float), ("critic_lr", ctypes.c_float),
                ("beta1", ctypes.c_float), ("beta2", ctypes.c_float), ("eps", ctypes.c_float),
                ("weight_decay", ctypes.c_float), ("clip_range", ctypes.c_float),
                ("entropy_scale", ctypes.c_float), ("max_grad_norm", ctypes.c_float),
                ("max_rows", ctypes.c_int32), ("seed", ctypes.c_uint64), ("train_gemm", ctypes.c_int32),
                ("infer_fp16", ctypes.c_int32), ("shared_layers", ctypes.c_int32 * MAX_LAYERS),
                ("n_shared_layers", ctypes.c_int32), ("sample_row_offset", ctypes.c_int64)]

GEMM_F32X6, GEMM_F32, GEMM_F16X3 = 0, 1, 2  # rlgpu_ppo_config.train_gemm (include/rlgpu_ppo.h)


_bound = False


def _bind():
    global _bound
    L = _lib.lib()
    if _bound:
        return L
    vp, i32, i64, u64, f32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float
    L.rlgpu_ppo_create.argtypes = [ctypes.POINTER(_Cfg), ctypes.POINTER(vp)]
    L.rlgpu_ppo_destroy.argtypes = [vp]
    L.rlgpu_ppo_buffers.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(i64)]
    L.rlgpu_ppo_model_range.argtypes = [vp, i32, ctypes.POINTER(i64), ctypes.POINTER(i64)]
    L.rlgpu_ppo_init_params.argtypes = [vp, u64, vp]
    L.rlgpu_ppo_refresh_half.argtypes = [vp, vp]
    L.rlgpu_ppo_forward.argtypes = [vp, i32, i32, vp, i32, vp, vp]
    L.rlgpu_ppo_infer_actions.argtypes = [vp, vp, vp, i32, i32, u64, vp, vp, vp]
    L.rlgpu_ppo_infer_critic.argtypes = [vp, vp, i64, vp, vp]
    L.rlgpu_mean_std.argtypes = [vp, i64, vp, vp]
    L.rlgpu_ppo_minibatch.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, i64, vp, vp, vp]
    L.rlgpu_ppo_optimizer_step.argtypes = [vp, vp, vp]
    L.rlgpu_ppo_zero_grad.argtypes = [vp, vp]
    L.rlgpu_ppo_optimizer_state.argtypes = [vp, ctypes.POINTER(i64), ctypes.POINTER(vp), ctypes.POINTER(vp)]
    L.rlgpu_ppo_set_optimizer_step.argtypes = [vp, i64]
    L.rlgpu_ppo_set_version.argtypes = [vp, vp, vp]
    L.rlgpu_ppo_infer_actions_mixed.argtypes = [vp, vp, vp, i32, i32, u64, vp, vp, vp, vp]
    L.rlgpu_permutation.argtypes = [i64, u64, u64, vp, vp]
    L.rlgpu_kernel_timing.argtypes = [i32]
    L.rlgpu_kernel_timing_read.argtypes = [vp, vp, vp, i32]
    _ = f32
    _bound = True
    return L


def param_count(obs_size, num_actions, layers, out=None, layer_norm=True):
    """Parameter count of a GGL::Model (Linear [+LayerNorm] per hidden layer + output Linear;
    out=0: no output layer, the shared head)."""
    n, prev = 0, obs_size
    for h in layers:
        n += prev * h + h + (2 * h if layer_norm else 0)
        prev = h
    o = num_actions if out is None else out
    return n + prev * o + o


class PPO:
    """Policy + critic (+ an optional shared head in front of both: PPOLearnerConfig::sharedHead),
    AdamW, fp32 training / bf16 inference, all in HBM."""

    def __init__(self, obs_size=167, num_actions=90, policy_layers=(512, 512), critic_layers=(512, 512),
                 layer_norm=True, policy_lr=2.5e-4, critic_lr=2.5e-4, clip_range=0.2, entropy_scale=0.035,
                 max_grad_norm=0.5, max_rows=50_000, seed=42, init=True, device="cuda:0",
                 betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, leaky_slope=0.01, train_gemm=GEMM_F16X3,
                 infer_fp16=False, shared_layers=()):
        import torch
        if not torch.cuda.is_available():
            raise _lib.RLGPUError("PPO needs an MI355X: the product path has no CPU fallback")
        L = _bind()
        self.device = torch.device(device)
        torch.cuda.set_device(self.device)
        c = _Cfg()
        c.obs_size, c.num_actions = obs_size, num_actions
        c.n_policy_layers, c.n_critic_layers = len(policy_layers), len(critic_layers)
        for i, v in enumerate(policy_layers):
            c.policy_layers[i] = v
        for i, v in enumerate(critic_layers):
            c.critic_layers[i] = v
        c.n_shared_layers = len(shared_layers)
        for i, v in enumerate(shared_layers):
            c.shared_layers[i] = v
        c.layer_norm, c.leaky_slope = int(layer_norm), leaky_slope
        self.leaky_slope = leaky_slope
        c.policy_lr, c.critic_lr = policy_lr, critic_lr
        c.beta1, c.beta2, c.eps, c.weight_decay = betas[0], betas[1], eps, weight_decay
        c.clip_range, c.entropy_scale, c.max_grad_norm = clip_range, entropy_scale, max_grad_norm
        c.max_rows, c.seed = max_rows, seed
        c.train_gemm = train_gemm
        c.infer_fp16 = int(infer_fp16)
        h = ctypes.c_void_p()
        _lib.check(L.rlgpu_ppo_create(ctypes.byref(c), ctypes.byref(h)), "rlgpu_ppo_create")
        self._h = h
        self.cfg = c
        # AdamW options per model (checkpoint.py's *_OPTIM.lt): the shared head steps at min(LR)
        self.optim_options = {"lr": (policy_lr, critic_lr, min(policy_lr, critic_lr)), "betas": tuple(betas), "eps": eps,
                              "weight_decay": weight_decay}
        self.obs_size, self.num_actions = obs_size, num_actions
        self.policy_layers, self.critic_layers, self.layer_norm = tuple(policy_layers), tuple(critic_layers), layer_norm
        self.shared_layers = tuple(shared_layers)
        self.max_rows = max_rows
        p, g, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int64()
        _lib.check(L.rlgpu_ppo_buffers(h, ctypes.byref(p), ctypes.byref(g), ctypes.byref(n)), "rlgpu_ppo_buffers")
        self.num_params = n.value
        self.params = alias(p.value, (n.value,), torch.float32, self.device)
        self.grads = alias(g.value, (n.value,), torch.float32, self.device)
        self.metrics = torch.zeros(NUM_METRICS, device=self.device)
        self.adv_stats = torch.zeros(2, device=self.device)
        if init:
            self.init_params(seed)

    @classmethod
    def wrap(cls, handle, device, policy_layers, critic_layers, max_rows, obs_size=167, num_actions=90,
             layer_norm=True, leaky_slope=0.01, metrics_source=None, owner=None, shared_layers=(), optim_options=None):
        """A PPO view of a handle owned elsewhere (the C++ Learner's PPOLearner): not destroyed
        by this object.  metrics_source(reset) -> (sums, count) replaces the own metric buffer."""
        import torch
        L = _bind()
        self = cls.__new__(cls)
        self._h, self._owned, self._owner = ctypes.c_void_p(handle), False, owner
        self.device = torch.device(device)
        self.obs_size, self.num_actions = obs_size, num_actions
        self.policy_layers, self.critic_layers, self.layer_norm = tuple(policy_layers), tuple(critic_layers), layer_norm
        self.shared_layers = tuple(shared_layers)
        self.leaky_slope, self.max_rows = leaky_slope, max_rows
        self.optim_options = optim_options
        p, g, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int64()
        _lib.check(L.rlgpu_ppo_buffers(self._h, ctypes.byref(p), ctypes.byref(g), ctypes.byref(n)), "rlgpu_ppo_buffers")
        self.num_params = n.value
        self.params = alias(p.value, (n.value,), torch.float32, self.device)
        self.grads = alias(g.value, (n.value,), torch.float32, self.device)
        self.metrics = torch.zeros(NUM_METRICS, device=self.device)
        self.adv_stats = torch.zeros(2, device=self.device)
        self._metrics_source = metrics_source
        return self

    _owned = True
    _metrics_source = None
    optim_options = None

    def close(self):
        if getattr(self, "_h", None):
            if self._owned:
                _lib.check(_lib.lib().rlgpu_ppo_destroy(self._h), "rlgpu_ppo_destroy")
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- parameters
    def model_range(self, model):
        off, cnt = ctypes.c_int64(), ctypes.c_int64()
        _lib.check(_lib.lib().rlgpu_ppo_model_range(self._h, model, ctypes.byref(off), ctypes.byref(cnt)), "model_range")
        return off.value, cnt.value

    def model_slice(self, model, grads=False):
        off, cnt = self.model_range(model)
        return (self.grads if grads else self.params)[off:off + cnt]

    @property
    def models(self):
        """Model indices present: policy, critic (and the shared head)."""
        return (0, 1, 2) if self.shared_layers else (0, 1)

    def flat(self, grads=False):
        """Concatenation of the models' parameters (or gradients) in torch parameters() order,
        without the alignment gap between models (policy, critic, shared head)."""
        import torch
        return torch.cat([self.model_slice(m, grads) for m in self.models])

    def policy_version(self):
        """The flat parameters an old policy version holds: the policy's, then the shared head's
        (PolicyVersionManager versions GetPolicyModels(), PPOLearner.cpp:665-674)."""
        import torch
        return torch.cat([self.model_slice(m) for m in self.models if m != 1])

    def model_in(self, model):
        return self.shared_layers[-1] if (self.shared_layers and model != 2) else self.obs_size

    def model_out(self, model):
        return (self.num_actions, 1, self.shared_layers[-1] if self.shared_layers else 0)[model]

    def init_params(self, seed):
        _lib.check(_lib.lib().rlgpu_ppo_init_params(self._h, seed, _lib.stream_ptr()), "init_params")

    def refresh_half(self):
        _lib.check(_lib.lib().rlgpu_ppo_refresh_half(self._h, _lib.stream_ptr()), "refresh_half")

    def torch_module(self, model):
        """An equivalent torch.nn.Sequential (torch parameters() order = the flat layout), on CPU,
        holding a copy of the current parameters: checkpoint export and test reference."""
        import torch
        layers = (self.policy_layers, self.critic_layers, self.shared_layers)[model]
        out = None if model == 2 else self.model_out(model)
        seq = make_sequential(self.model_in(model), out, layers, self.layer_norm, self.leaky_slope)
        flat = self.model_slice(model).detach().cpu()
        o = 0
        with torch.no_grad():
            for prm in seq.parameters():
                prm.copy_(flat[o:o + prm.numel()].view_as(prm))
                o += prm.numel()
        return seq

    def torch_chain(self, model):
        """shared head -> model as one torch.nn.Sequential (the module chain the reference's
        InferPolicyProbsFromModels / InferCritic run, PPOLearner.cpp:90-91,188-191)."""
        import torch
        mods = list(self.torch_module(2)) if (self.shared_layers and model != 2) else []
        return torch.nn.Sequential(*(mods + list(self.torch_module(model))))

    def load_torch_module(self, model, seq):
        import torch
        flat = torch.cat([p.detach().reshape(-1).float() for p in seq.parameters()])
        dst = self.model_slice(model)
        assert flat.numel() == dst.numel(), "architecture mismatch"
        dst.copy_(flat.to(self.device))
        self.refresh_half()

    # ---------------------------------------------------------------- inference
    def forward(self, model, x, half=False, out=None):
        import torch
        n = x.shape[0]
        width = self.model_out(model)
        out = torch.empty((n, width), device=self.device) if out is None else out
        _lib.check(_lib.lib().rlgpu_ppo_forward(self._h, model, int(half), _lib.ptr(x.contiguous()), n, _lib.ptr(out),
                                                _lib.stream_ptr()), "rlgpu_ppo_forward")
        return out

    def infer_actions(self, obs, masks, step=0, deterministic=False, actions=None, logp=None):
        import torch
        n = obs.shape[0]
        actions = torch.empty(n, dtype=torch.int32, device=self.device) if actions is None else actions
        logp = torch.empty(n, device=self.device) if logp is None else logp
        _lib.check(_lib.lib().rlgpu_ppo_infer_actions(self._h, _lib.ptr(obs), _lib.ptr(masks), n, int(deterministic),
                                                      step, _lib.ptr(actions), _lib.ptr(logp), _lib.stream_ptr()),
                   "rlgpu_ppo_infer_actions")
        return actions, logp

    def set_version(self, policy_params):
        """bf16 inference copy of an old policy version (flat fp32 parameters on the device: the
        policy's, then the shared head's -- policy_version())."""
        cnt = sum(self.model_range(m)[1] for m in self.models if m != 1)
        if policy_params.numel() != cnt:
            raise _lib.RLGPUError("policy version has the wrong parameter count")
        _lib.check(_lib.lib().rlgpu_ppo_set_version(self._h, _lib.ptr(policy_params.contiguous()), _lib.stream_ptr()),
                   "rlgpu_ppo_set_version")

    def infer_actions_mixed(self, obs, masks, old_rows, step=0, deterministic=False, actions=None, logp=None):
        """Rows with old_rows != 0 act with the version of set_version (their logp is not written)."""
        import torch
        n = obs.shape[0]
        actions = torch.empty(n, dtype=torch.int32, device=self.device) if actions is None else actions
        logp = torch.empty(n, device=self.device) if logp is None else logp
        _lib.check(_lib.lib().rlgpu_ppo_infer_actions_mixed(self._h, _lib.ptr(obs), _lib.ptr(masks), n, int(deterministic),
                                                            step, _lib.ptr(old_rows), _lib.ptr(actions), _lib.ptr(logp),
                                                            _lib.stream_ptr()), "rlgpu_ppo_infer_actions_mixed")
        return actions, logp

    def infer_critic(self, obs, out=None):
        import torch
        n = obs.shape[0]
        out = torch.empty(n, device=self.device) if out is None else out
        _lib.check(_lib.lib().rlgpu_ppo_infer_critic(self._h, _lib.ptr(obs), n, _lib.ptr(out), _lib.stream_ptr()),
                   "rlgpu_ppo_infer_critic")
        return out

    # ---------------------------------------------------------------- learning
    def adv_normalizer(self, adv):
        _lib.check(_lib.lib().rlgpu_mean_std(_lib.ptr(adv), adv.numel(), _lib.ptr(self.adv_stats), _lib.stream_ptr()),
                   "rlgpu_mean_std")
        return self.adv_stats

    def minibatch(self, obs, masks, actions, old_logp, adv, target, index, start, n, batch_size):
        _lib.check(_lib.lib().rlgpu_ppo_minibatch(
            self._h, _lib.ptr(obs), _lib.ptr(masks), _lib.ptr(actions), _lib.ptr(old_logp), _lib.ptr(adv),
            _lib.ptr(target), _lib.ptr(index), start, n, batch_size, _lib.ptr(self.adv_stats), _lib.ptr(self.metrics),
            _lib.stream_ptr()), "rlgpu_ppo_minibatch")
        self._count += 1

    _count = 0

    def optimizer_step(self):
        _lib.check(_lib.lib().rlgpu_ppo_optimizer_step(self._h, _lib.ptr(self.metrics), _lib.stream_ptr()),
                   "rlgpu_ppo_optimizer_step")

    def zero_grad(self):
        _lib.check(_lib.lib().rlgpu_ppo_zero_grad(self._h, _lib.stream_ptr()), "zero_grad")

    def read_metrics(self, reset=True):
        """Report entries of PPOLearner::Learn (:537-566): means over the accumulated minibatches."""
        if self._metrics_source is not None:
            m, cnt = self._metrics_source(reset)
            cnt = max(cnt, 1)
            return {"Policy Entropy": m[0] / cnt, "Mean KL Divergence": m[1] / cnt, "Policy Loss": m[2] / cnt,
                    "Critic Loss": m[3] / cnt, "Ratio": m[4] / cnt, "SB3 Clip Fraction": m[5] / cnt,
                    "Policy Grad Norm": m[7], "Critic Grad Norm": m[8], "Shared Head Grad Norm": m[9]}
        m = self.metrics.cpu().tolist()
        cnt = max(self._count, 1)
        rep = {"Policy Entropy": m[0] / cnt, "Mean KL Divergence": m[1] / cnt, "Policy Loss": m[2] / cnt,
               "Critic Loss": m[3] / cnt, "Ratio": m[4] / cnt, "SB3 Clip Fraction": m[5] / cnt,
               "Policy Grad Norm": m[7], "Critic Grad Norm": m[8], "Shared Head Grad Norm": m[9]}
        if reset:
            self.metrics.zero_()
            self._count = 0
        return rep

    def optimizer_state(self):
        import torch
        step, m, v = ctypes.c_int64(), ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check(_lib.lib().rlgpu_ppo_optimizer_state(self._h, ctypes.byref(step), ctypes.byref(m), ctypes.byref(v)),
                   "optimizer_state")
        return (step.value, alias(m.value, (self.num_params,), torch.float32, self.device),
                alias(v.value, (self.num_params,), torch.float32, self.device))

    def set_optimizer_step(self, step):
        _lib.check(_lib.lib().rlgpu_ppo_set_optimizer_step(self._h, int(step)), "set_optimizer_step")

    def model_sizes(self, model):
        """Per-parameter element counts in torch order (GetSeqSizes, Models.cpp:79-87)."""
        return [p.numel() for p in self.torch_module(model).parameters()]


def make_sequential(obs_size, out, layers, layer_norm=True, leaky_slope=0.01):
    """GGL::Model's module list (Models.cpp:7-33): per hidden layer Linear [, LayerNorm],
    LeakyReLU; then the output Linear (none when out is None: the shared head, addOutputLayer
    false).  CPU, torch default init."""
    import torch
    mods, prev = [], obs_size
    for hdim in layers:
        mods.append(torch.nn.Linear(prev, hdim))
        if layer_norm:
            mods.append(torch.nn.LayerNorm(hdim))
        mods.append(torch.nn.LeakyReLU(leaky_slope))
        prev = hdim
    if out is not None:
        mods.append(torch.nn.Linear(prev, out))
    return torch.nn.Sequential(*mods)


KERNEL_TIMING_SLOTS = ("forward / input-gradient GEMMs", "weight-gradient GEMMs", "LayerNorm forward",
                       "LayerNorm backward")


def kernel_timing(enable):
    """Start (clearing earlier records) or stop the learn-phase kernel timing (rlgpu_kernel_timing)."""
    _bind()
    _lib.check(_lib.lib().rlgpu_kernel_timing(1 if enable else 0), "rlgpu_kernel_timing")


def kernel_timing_read():
    """{slot name: (ms summed, work summed -- flops or bytes --, launches)} since kernel_timing(True)."""
    import numpy as np
    _bind()
    n = len(KERNEL_TIMING_SLOTS)
    ms, work, cnt = np.zeros(n), np.zeros(n), np.zeros(n, np.int64)
    _lib.check(_lib.lib().rlgpu_kernel_timing_read(ms.ctypes.data, work.ctypes.data, cnt.ctypes.data, n),
               "rlgpu_kernel_timing_read")
    return {k: (float(ms[i]), float(work[i]), int(cnt[i])) for i, k in enumerate(KERNEL_TIMING_SLOTS)}


def permutation(n, seed, counter, out=None, device="cuda:0"):
    """ExperienceBuffer shuffle (ExperienceBuffer.cpp:130): random permutation of [0, n) on device."""
    import torch
    out = torch.empty(n, dtype=torch.int32, device=device) if out is None else out
    _bind()
    _lib.check(_lib.lib().rlgpu_permutation(n, seed, counter, _lib.ptr(out), _lib.stream_ptr()), "rlgpu_permutation")
    return out


def log_num_actions(a):
    return math.log(a)
