"""PPO outer loop for the batched Joystick env, in PyTorch on MI355X.

The reference trains with brax PPO through ``common/runner.py:86-118``:
``ppo.train(environment, wrap_env_fn=wrapper.wrap_for_brax_training, randomization_fn=...)``
with ``locomotion_params.brax_ppo_config("BerkeleyHumanoidJoystickFlatTerrain")``
(mujoco_playground, not vendored in the reference; values restated in ``PPOConfig``).
This module restates brax's algorithm (brax/training/agents/ppo: networks.py, losses.py,
train.py; running_statistics.py) on torch tensors that never leave the GPU:

* policy: MLP -> (loc, raw scale); NormalTanh distribution, scale = softplus(raw) + 1e-3,
  action = tanh(sample); log-prob with the tanh Jacobian; entropy with a sampled Jacobian term
* value: MLP on ``privileged_state`` (``value_obs_key``), policy on ``state``
* observation normaliser: running mean / variance over every env-step of every rank
  (one RCCL all-reduce of (count, sum, sum of squares) per update)
* unroll ``unroll_length`` env-steps for all envs, GAE (lambda, discount, truncation-aware
  bootstrap), ``num_updates_per_batch`` epochs of ``num_minibatches`` shuffled minibatches,
  clipped surrogate + 0.25 * value MSE + entropy bonus, Adam, global-norm clipping, gradients
  all-reduced over RCCL between ranks (data parallel, one process per GPU)
"""

from __future__ import annotations

import ctypes as C
import math
import os
import time
from dataclasses import asdict, dataclass, field
from typing import Callable, Dict, Optional, Sequence

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class PPOConfig:
    """brax_ppo_config("BerkeleyHumanoidJoystickFlatTerrain") as the reference runner uses it
    (common/runner.py:86-89; num_timesteps from open_duck_mini_v2/runner.py:44). The values come from
    mujoco_playground's locomotion_params, an upstream dependency the reference does not vendor and
    whose version is unpinned (pyproject.toml: playground>=0.0.3): restated, not pinned."""
    num_timesteps: int = 150_000_000     # open_duck_mini_v2/runner.py:44
    num_evals: int = 15
    reward_scaling: float = 1.0
    episode_length: int = 1000
    normalize_observations: bool = True
    action_repeat: int = 1
    unroll_length: int = 20
    num_minibatches: int = 32
    num_updates_per_batch: int = 4
    discounting: float = 0.97
    gae_lambda: float = 0.95
    learning_rate: float = 3e-4
    entropy_cost: float = 0.005
    num_envs: int = 8192
    batch_size: int = 256
    max_grad_norm: float = 1.0
    clipping_epsilon: float = 0.2
    normalize_advantage: bool = True
    policy_hidden_layer_sizes: Sequence[int] = (512, 256, 128)
    value_hidden_layer_sizes: Sequence[int] = (512, 256, 128)
    policy_obs_key: str = "state"
    value_obs_key: str = "privileged_state"
    seed: int = 0


# ---------------------------------------------------------------------------------------
# networks (brax ppo/networks.py: MLP with swish, NormalTanhDistribution)
# ---------------------------------------------------------------------------------------
class _SplitKLinearFn(torch.autograd.Function):
    """y = x W^T + b whose weight gradient dW = dY^T X is formed as SPLITK partial products over
    row blocks of the batch and their sum: the learner's minibatches are K = 5120 rows deep and only
    a few 32 x 32 output tiles wide, which one GEMM runs on a fraction of the chip (31 us -> 14-20 us
    per layer on MI355X, `tools/bench_dw.py`)."""

    SPLITK = 4

    @staticmethod
    def forward(ctx, x, w, b):
        x2 = x.reshape(-1, x.shape[-1])
        ctx.save_for_backward(x2, w)
        ctx.xshape = x.shape
        return torch.addmm(b, x2, w.t()).view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x2, w = ctx.saved_tensors
        g2 = gy.reshape(-1, gy.shape[-1])
        n, S = g2.shape[0], _SplitKLinearFn.SPLITK
        gx = g2.mm(w).view(ctx.xshape) if ctx.needs_input_grad[0] else None
        if g2.shape[1] >= 8 and n % S == 0 and n >= 64 * S:
            gw = torch.bmm(g2.view(S, n // S, -1).transpose(1, 2), x2.view(S, n // S, -1)).sum(0)
        else:
            gw = g2.t().mm(x2)
        return gx, gw, g2.sum(0)


class SplitKLinear(nn.Linear):
    """nn.Linear (same parameters, state dict and export) with the split-K weight gradient."""

    def forward(self, x):
        return _SplitKLinearFn.apply(x, self.weight, self.bias)


def mlp(sizes: Sequence[int], out: int) -> nn.Sequential:
    layers, prev = [], sizes[0]
    for h in sizes[1:]:
        layers += [SplitKLinear(prev, h), nn.SiLU()]
        prev = h
    layers.append(SplitKLinear(prev, out))
    for m in layers:  # brax: lecun_uniform kernels, zero bias
        if isinstance(m, nn.Linear):
            bound = math.sqrt(3.0 / m.in_features)
            nn.init.uniform_(m.weight, -bound, bound)
            nn.init.zeros_(m.bias)
    return nn.Sequential(*layers)


MIN_STD = 1e-3
POLICY_SAMPLE_MAX_ACTIONS = 16  # duck_policy_sample (csrc/duck_mlp.hip): one lane per action dim of a 16-lane row


def _log_det_jac_tanh(x: torch.Tensor) -> torch.Tensor:
    """log |d tanh(x) / dx| = 2 (log 2 - x - softplus(-2x)) (brax distribution.TanhBijector)."""
    return 2.0 * (math.log(2.0) - x - F.softplus(-2.0 * x))


class NormalTanh:
    """brax distribution.NormalTanhDistribution (event size = action size)."""

    def __init__(self, logits: torch.Tensor):
        loc, raw = logits.chunk(2, dim=-1)
        self.loc, self.scale = loc, F.softplus(raw) + MIN_STD

    def sample_raw(self, gen: Optional[torch.Generator] = None) -> torch.Tensor:
        eps = torch.randn(self.loc.shape, device=self.loc.device, generator=gen)
        return self.loc + self.scale * eps

    def log_prob(self, raw: torch.Tensor) -> torch.Tensor:
        z = (raw - self.loc) / self.scale
        lp = -0.5 * z * z - torch.log(self.scale) - 0.5 * math.log(2 * math.pi)
        return (lp - _log_det_jac_tanh(raw)).sum(-1)

    def entropy(self, gen: Optional[torch.Generator] = None) -> torch.Tensor:
        ent = 0.5 + 0.5 * math.log(2 * math.pi) + torch.log(self.scale)
        return (ent + _log_det_jac_tanh(self.sample_raw(gen))).sum(-1)

    def mode(self) -> torch.Tensor:
        return torch.tanh(self.loc)


class RunningStatistics(nn.Module):
    """brax running_statistics: mean / std over all observations seen (all ranks).

    State (count, mean, summed_var, std) is fp64 like brax's; ``std`` starts at 1 so an
    un-updated normaliser is the identity shifted by a zero mean (running_statistics.init_state).
    """

    def __init__(self, size: int, std_eps: float = 0.0, std_min: float = 1e-6, std_max: float = 1e6):
        super().__init__()
        self.register_buffer("count", torch.zeros((), dtype=torch.float64))
        self.register_buffer("mean", torch.zeros(size, dtype=torch.float64))
        self.register_buffer("summed_var", torch.zeros(size, dtype=torch.float64))
        self.register_buffer("std", torch.ones(size, dtype=torch.float64))
        # fp32 copies for normalize(): the same conversions, made once per update instead of per call
        # (two conversion kernels less in every policy / value evaluation; not checkpointed)
        self.register_buffer("mean32", torch.zeros(size), persistent=False)
        self.register_buffer("std32", torch.ones(size), persistent=False)
        self.register_buffer("istd32", torch.ones(size), persistent=False)  # 1 / std32 (the fused MLP's loads)
        self.std_eps, self.std_min, self.std_max = std_eps, std_min, std_max

    @torch.no_grad()
    def _refresh(self) -> None:
        self.mean32.copy_(self.mean)
        self.std32.copy_(self.std)
        self.istd32.copy_(1.0 / self.std)

    def _load_from_state_dict(self, *args, **kwargs):
        super()._load_from_state_dict(*args, **kwargs)
        self._refresh()

    @torch.no_grad()
    def update(self, x: torch.Tensor) -> None:
        """Fold a batch [..., size] in (parallel-variance merge; one all-reduce across ranks)."""
        x = x.reshape(-1, x.shape[-1])
        k = x.shape[-1]
        stats = torch.cat([torch.full((1,), float(x.shape[0]), dtype=torch.float64, device=x.device),
                           self._moments(x)])
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(stats)
        n, s, ss = stats[0], stats[1:1 + k], stats[1 + k:]
        bmean = s / n
        bvar = torch.clamp(ss - n * bmean * bmean, min=0.0)  # batch sum of squared deviations
        tot = self.count + n
        delta = bmean - self.mean
        self.mean += delta * (n / tot)
        self.summed_var += bvar + delta * delta * (self.count * n / tot)
        self.count.copy_(tot)
        var = self.summed_var / self.count
        self.std.copy_(torch.clamp(torch.sqrt(var + self.std_eps), self.std_min, self.std_max))
        self._refresh()

    def _moments(self, x: torch.Tensor) -> torch.Tensor:
        """[column sums | column sums of squares] of a batch [N, size] in fp64: the ``duck_column_stats``
        HIP kernel for fp32 GPU batches (torch's fp64 column reductions took 1.8 ms each on a 163,840-row
        rollout batch, 8 % of an update's learning time), torch's reductions for host tensors (tests,
        CPU-only toy runs). Both sum in fp64 (no fp64 copy of the batch)."""
        if not (x.is_cuda and x.dtype == torch.float32):
            return torch.cat([x.sum(0, dtype=torch.float64),
                              torch.linalg.vector_norm(x, 2, dim=0, dtype=torch.float64) ** 2])
        from .native import check, lib
        L = lib()
        x = x.contiguous()
        n, k = x.shape
        need = max(1, L.duck_column_stats_scratch(n, k))
        scratch = getattr(self, "_cs_scratch", None)
        if scratch is None or scratch.numel() < need or scratch.device != x.device:
            scratch = self._cs_scratch = torch.empty(need, dtype=torch.float64, device=x.device)
        out = torch.empty(2 * k, dtype=torch.float64, device=x.device)
        check(L.duck_column_stats(n, k, x.data_ptr(), out.data_ptr(), scratch.data_ptr(),
                                  torch.cuda.current_stream(x.device).cuda_stream))
        return out

    def normalize(self, x: torch.Tensor) -> torch.Tensor:
        if x.dtype == torch.float32:
            return (x - self.mean32) / self.std32
        return (x - self.mean.to(x.dtype)) / self.std.to(x.dtype)


class ActorCritic(nn.Module):
    def __init__(self, obs_size: int, priv_size: int, action_size: int, cfg: PPOConfig):
        super().__init__()
        self.policy = mlp([obs_size] + list(cfg.policy_hidden_layer_sizes), 2 * action_size)
        self.value = mlp([priv_size] + list(cfg.value_hidden_layer_sizes), 1)
        self.obs_norm = RunningStatistics(obs_size)
        self.priv_norm = RunningStatistics(priv_size)
        self.normalize = cfg.normalize_observations

    def policy_logits(self, obs: torch.Tensor) -> torch.Tensor:
        return self.policy(self.obs_norm.normalize(obs) if self.normalize else obs)

    def value_of(self, priv: torch.Tensor) -> torch.Tensor:
        return self.value(self.priv_norm.normalize(priv) if self.normalize else priv).squeeze(-1)


# ---------------------------------------------------------------------------------------
# losses (brax ppo/losses.py)
# ---------------------------------------------------------------------------------------
@torch.no_grad()
def compute_gae_torch(truncation: torch.Tensor, termination: torch.Tensor, rewards: torch.Tensor, values: torch.Tensor,
                bootstrap_value: torch.Tensor, lambda_: float, discount: float):
    """Time-major [T, B] GAE with truncation masking (brax losses.compute_gae)."""
    trunc_mask = 1.0 - truncation
    values_t_plus_1 = torch.cat([values[1:], bootstrap_value[None]], dim=0)
    deltas = (rewards + discount * (1.0 - termination) * values_t_plus_1 - values) * trunc_mask
    acc = torch.zeros_like(bootstrap_value)
    out = torch.empty_like(values)
    for t in range(values.shape[0] - 1, -1, -1):
        acc = deltas[t] + discount * (1.0 - termination[t]) * trunc_mask[t] * lambda_ * acc
        out[t] = acc
    vs = out + values
    vs_t_plus_1 = torch.cat([vs[1:], bootstrap_value[None]], dim=0)
    advantages = (rewards + discount * (1.0 - termination) * vs_t_plus_1 - values) * trunc_mask
    return vs, advantages


@torch.no_grad()
def compute_gae(truncation: torch.Tensor, termination: torch.Tensor, rewards: torch.Tensor, values: torch.Tensor,
                bootstrap_value: torch.Tensor, lambda_: float, discount: float):
    """GAE: the ``duck_gae`` HIP kernel for fp32 GPU tensors (one launch instead of ~120 small
    ones per minibatch), the torch recursion for host tensors (CPU-only toy runs, tests)."""
    if not values.is_cuda:
        return compute_gae_torch(truncation, termination, rewards, values, bootstrap_value, lambda_, discount)
    from .native import check, lib
    T, B = values.shape
    args = [t.contiguous() for t in (truncation, termination, rewards, values, bootstrap_value)]
    if any(a.dtype != torch.float32 for a in args):
        raise TypeError("compute_gae on the GPU takes float32 tensors")
    vs, adv = torch.empty_like(args[3]), torch.empty_like(args[3])
    check(lib().duck_gae(T, B, *(a.data_ptr() for a in args), float(lambda_), float(discount), vs.data_ptr(),
                         adv.data_ptr(), torch.cuda.current_stream(values.device).cuda_stream))
    return vs, adv


class _FusedLoss(torch.autograd.Function):
    """The PPO loss after GAE as one ``duck_ppo_loss`` HIP launch (csrc/duck_ppo.hip): the forward
    returns [loss, policy_loss, v_loss, entropy] and the kernel's gradients w.r.t. the logits and
    the baseline, which the backward scales by d loss (the three metrics are detached)."""

    @staticmethod
    def forward(ctx, logits, baseline, raw_action, old_logprob, adv, vs, eps, clip_eps, entropy_cost, normalize):
        from .native import check, lib
        args = [t.detach().contiguous() for t in (logits, raw_action, old_logprob, adv, vs, baseline, eps)]
        if any(a.dtype != torch.float32 for a in args):
            raise TypeError("the fused PPO loss takes float32 tensors")
        lg, ra, olp, ad, v, bl, ep = args
        A = ra.shape[-1]
        N = ra.numel() // A
        # the kernel indexes every operand by (N, A) unchecked: a mismatch must be an error here,
        # not an out-of-bounds device read (the torch expression would raise on it too)
        if A < 1 or lg.shape[-1] != 2 * A or lg.numel() != 2 * N * A or ep.numel() != N * A:
            raise ValueError(f"fused PPO loss: logits {tuple(lg.shape)} / eps {tuple(ep.shape)} do not match "
                             f"raw_action {tuple(ra.shape)} (N={N}, A={A})")
        for name, t in (("old_logprob", olp), ("adv", ad), ("vs", v), ("baseline", bl)):
            if t.numel() != N:
                raise ValueError(f"fused PPO loss: {name} holds {t.numel()} values, expected N={N}")
        out = torch.empty(lib().duck_ppo_loss_out_size(N), dtype=torch.float32, device=lg.device)  # + scratch
        g_lg, g_bl = torch.empty_like(lg), torch.empty_like(bl)
        check(lib().duck_ppo_loss(N, A, lg.data_ptr(), ra.data_ptr(), olp.data_ptr(), ad.data_ptr(), v.data_ptr(),
                                  bl.data_ptr(), ep.data_ptr(), float(clip_eps), float(entropy_cost), int(normalize),
                                  out.data_ptr(), g_lg.data_ptr(), g_bl.data_ptr(),
                                  torch.cuda.current_stream(lg.device).cuda_stream))
        ctx.save_for_backward(g_lg, g_bl)
        return out[:4]

    @staticmethod
    def backward(ctx, g_out):
        g_lg, g_bl = ctx.saved_tensors
        return g_lg * g_out[0], g_bl * g_out[0], None, None, None, None, None, None, None, None


def ppo_loss(net: ActorCritic, batch: Dict[str, torch.Tensor], cfg: PPOConfig, gen: Optional[torch.Generator],
             fused: Optional[bool] = None):
    """batch tensors are time-major [T, B, ...]; returns (loss, metrics). On the GPU the part after
    the networks and GAE runs as the fused ``duck_ppo_loss`` kernel (one launch instead of ~150 small
    autograd kernels per minibatch; ``fused=False`` or DUCK_PPO_FUSED=0 keeps the torch expression
    below, which is also its test reference)."""
    logits = net.policy_logits(batch["obs"])
    # the baseline [T, B] and the bootstrap value [B] in one pass of the value network
    priv, nxt = batch["priv"], batch["next_priv"][-1]
    v_all = net.value_of(torch.cat([priv.reshape(-1, priv.shape[-1]), nxt], 0))
    baseline, bootstrap = v_all[: priv.shape[0] * priv.shape[1]].view(priv.shape[:2]), v_all[priv.shape[0] * priv.shape[1]:]
    rewards = batch["reward"] * cfg.reward_scaling
    truncation = batch["truncation"]
    termination = batch["done"] * (1.0 - truncation)
    if fused is None:
        fused = logits.is_cuda and os.environ.get("DUCK_PPO_FUSED", "1") != "0"
    if fused:
        vs, adv = compute_gae(truncation, termination, rewards, baseline.detach(), bootstrap.detach(), cfg.gae_lambda,
                              cfg.discounting)
        loc = logits[..., : logits.shape[-1] // 2]
        eps = torch.randn(loc.shape, device=loc.device, generator=gen)  # the entropy sample, as NormalTanh draws it
        out = _FusedLoss.apply(logits, baseline, batch["raw_action"], batch["log_prob"], adv, vs, eps,
                               cfg.clipping_epsilon, cfg.entropy_cost, bool(cfg.normalize_advantage))
        return out[0], {"policy_loss": out[1].detach(), "v_loss": out[2].detach(), "entropy": out[3].detach()}
    dist_ = NormalTanh(logits)
    target_lp = dist_.log_prob(batch["raw_action"])
    vs, adv = compute_gae(truncation, termination, rewards, baseline.detach(), bootstrap.detach(), cfg.gae_lambda,
                          cfg.discounting)
    if cfg.normalize_advantage:
        adv = (adv - adv.mean()) / (adv.std(unbiased=False) + 1e-8)
    rho = torch.exp(target_lp - batch["log_prob"])
    s1 = rho * adv
    s2 = torch.clamp(rho, 1.0 - cfg.clipping_epsilon, 1.0 + cfg.clipping_epsilon) * adv
    policy_loss = -torch.minimum(s1, s2).mean()
    v_loss = ((vs - baseline) ** 2).mean() * 0.5 * 0.5
    entropy = dist_.entropy(gen).mean()
    loss = policy_loss + v_loss - cfg.entropy_cost * entropy
    return loss, {"policy_loss": policy_loss.detach(), "v_loss": v_loss.detach(), "entropy": entropy.detach()}


class FusedGrad:
    """One minibatch's loss and parameter gradients without autograd: both networks' MLPs forward and
    backward through the duck_mlp_* HIP kernels (csrc/duck_mlp.hip: fp32 MFMA GEMMs with the observation
    normaliser, bias, swish and its derivative fused into their loads and stores; weight gradients as
    split-K partial products summed in fixed order), GAE and the loss through duck_gae /
    duck_ppo_loss. It computes what ``ppo_loss(..., fused=True)`` + ``loss.backward()`` compute (the
    test compares the two), in ~40 launches instead of ~100, most of them MFMA GEMMs.

    The parameters' ``.grad`` are views of one flat buffer that the final reduction overwrites (never
    set to None), so the all-reduce over ranks is a single collective on that buffer."""

    SPLITS = 16      # partial products per weight gradient at most (duck_mlp_wgrad's row blocks)
    # workgroups a weight gradient aims for (its 64 x 32 tiles times its row blocks)
    WGRAD_TARGET = int(os.environ.get("DUCK_WGRAD_TARGET", "768"))

    def __init__(self, net: ActorCritic, rows: int, boot_rows: int, device):
        from .native import lib
        self.lib = lib()
        self.net = net
        self.params = list(net.parameters())
        self.P = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(self.P, device=device)
        # the parameters become views of one flat buffer too (same values, same module / state dict), so
        # clip + Adam is one pass over flat arrays (duck_clip_adam)
        self.pflat = torch.cat([p.detach().reshape(-1) for p in self.params]).contiguous()
        self.off, o = {}, 0
        for p in self.params:
            self.off[id(p)] = o
            p.data = self.pflat[o:o + p.numel()].view_as(p)
            p.grad = self.flat[o:o + p.numel()].view_as(p)
            o += p.numel()
        self.exp_avg = torch.zeros(self.P, device=device)
        self.exp_avg_sq = torch.zeros(self.P, device=device)
        self.adam_step = torch.zeros(1, dtype=torch.int32, device=device)
        self.adam_scratch = torch.zeros(self.lib.duck_clip_adam_scratch_size(self.P), device=device)
        # zeroed once: a layer that uses fewer row blocks than SPLITS leaves its other partials at 0
        self.part = torch.zeros(self.SPLITS * self.P, device=device)
        # one rank (set by _Learner): the weight-gradient partials are summed by the update's first launch
        # (duck_clip_adam_reduce) instead of a duck_mlp_wgrad_reduce launch of their own
        self.defer_reduce = False
        self.pol = [m for m in net.policy if isinstance(m, nn.Linear)]
        self.val = [m for m in net.value if isinstance(m, nn.Linear)]
        self.N, self.Nv = rows, rows + boot_rows

        def bufs(layers, n):
            return {"Z": [torch.empty(n, m.out_features, device=device) for m in layers[:-1]],
                    "H": [torch.empty(n, m.out_features, device=device) for m in layers[:-1]],
                    "dZ": [torch.empty(n, m.out_features, device=device) for m in layers[:-1]],
                    "out": torch.empty(n, layers[-1].out_features, device=device)}
        self.bp, self.bv = bufs(self.pol, self.N), bufs(self.val, self.Nv)
        A = self.pol[-1].out_features // 2
        self.g_lg = torch.empty(self.N, 2 * A, device=device)
        self.d_val = torch.zeros(self.Nv, 1, device=device)   # rows N.. (the bootstrap) stay 0: detached
        self.loss_out = torch.empty(self.lib.duck_ppo_loss_out_size(self.N), device=device)

    def _forward(self, layers, b, x, norm, n, stream):
        from .native import check
        mean, istd = (norm.mean32.data_ptr(), norm.istd32.data_ptr()) if norm is not None else (None, None)
        inp = x
        for i, m in enumerate(layers):
            last = i == len(layers) - 1
            y = b["out"] if last else b["Z"][i]
            check(self.lib.duck_mlp_gemm(0 if last else 1, n, m.in_features, m.out_features, inp.data_ptr(),
                                         m.weight.data_ptr(), m.bias.data_ptr(), None, y.data_ptr(),
                                         None if last else b["H"][i].data_ptr(), mean if i == 0 else None,
                                         istd if i == 0 else None, stream))
            if not last:
                inp = b["H"][i]
        return b["out"]

    # grouped launches (duck_mlp_group): the policy's and the value network's layers at one depth share a
    # launch, forward and backward (4 + 4 launches per minibatch instead of 8 + 14)
    def _prob_fwd(self, layers, b, x, norm, n, i):
        from .native import DuckMlpProblem
        m = layers[i]
        last = i == len(layers) - 1
        inp = x if i == 0 else b["H"][i - 1]
        mean, istd = (norm.mean32.data_ptr(), norm.istd32.data_ptr()) if (i == 0 and norm is not None) else (None, None)
        return DuckMlpProblem(0 if last else 1, n, m.in_features, m.out_features, inp.data_ptr(), m.weight.data_ptr(),
                              m.bias.data_ptr(), None, (b["out"] if last else b["Z"][i]).data_ptr(),
                              None if last else b["H"][i].data_ptr(), mean, istd, 0, 0, 0, 0, None)

    def _probs_bwd(self, layers, b, x, norm, dout, n, i):
        from .native import DuckMlpProblem
        m = layers[i]
        d = dout if i == len(layers) - 1 else b["dZ"][i]
        h = x if i == 0 else b["H"][i - 1]
        mean, istd = (norm.mean32.data_ptr(), norm.istd32.data_ptr()) if (i == 0 and norm is not None) else (None, None)
        tiles = -(-m.out_features // 64) * -(-(m.in_features + 1) // 32)
        splits = max(1, min(self.SPLITS, -(-self.WGRAD_TARGET // tiles), n // 64))
        out = [DuckMlpProblem(3, n, m.in_features, m.out_features, d.data_ptr(), h.data_ptr(), None, None, None, None,
                              mean, istd, splits, self.P, self.off[id(m.weight)], self.off[id(m.bias)],
                              self.part.data_ptr())]
        if i > 0:
            out.append(DuckMlpProblem(2, n, m.out_features, m.in_features, d.data_ptr(), m.weight.data_ptr(), None,
                                      b["Z"][i - 1].data_ptr(), b["dZ"][i - 1].data_ptr(), None, None, None,
                                      0, 0, 0, 0, None))
        return out

    def _group(self, probs, stream):
        from .native import DuckMlpProblem, check
        arr = (DuckMlpProblem * len(probs))(*probs)
        bn = self._tile_width(probs)
        bm = self._row_tile(probs) if bn == 32 else 64
        if bm == 32 and hasattr(self.lib, "duck_mlp_group_tiles"):
            check(self.lib.duck_mlp_group_tiles(len(probs), arr, 32, 32, stream))
        elif bn != 32 and hasattr(self.lib, "duck_mlp_group_bn"):
            check(self.lib.duck_mlp_group_bn(len(probs), arr, bn, stream))
        else:
            check(self.lib.duck_mlp_group(len(probs), arr, stream))

    @staticmethod
    def _row_tile(probs) -> int:
        """Output tile height of a grouped launch (duck_mlp_group_tiles; bit-identical either way): 32 when
        the launch has fewer than 2,048 of the 64 x 32 tiles and no GEMM reduces over more than 256 -- there
        the doubled workgroup count fills the chip (per launch, same box: the third and fourth layers'
        forward 15.9 -> 15.3 and 7.5 -> 6.4 us, the deepest backward launch 15.4 -> 11.9, the next 26.2 ->
        25.4); the wide layers keep 64 rows (their forward 40.0 -> 41.1 us at 32). DUCK_MLP_BM_AUTO = 0: 64."""
        if os.environ.get("DUCK_MLP_BM_AUTO", "1") == "0":
            return 64
        tiles, red = 0, 0
        for p in probs:
            if p.kind == 3:
                tiles += -(-p.M // 64) * -(-(p.R + 1) // 32) * p.splits
            else:
                tiles += -(-p.N // 64) * -(-p.M // 32)
                red = max(red, p.R)
        return 32 if tiles < 2048 and red <= 256 else 64

    @staticmethod
    def _tile_width(probs) -> int:
        """Output tile width of a grouped launch (duck_mlp_group_bn; bit-identical either way). 32: with 64
        every launch ran slower on the final learner (288 -> 324 us per minibatch,
        profiles/r06_ppo_tiles_ab.txt). DUCK_MLP_BN = 64 to try it."""
        return 64 if os.environ.get("DUCK_MLP_BN", "32") == "64" else 32

    def _backward(self, layers, b, x, norm, dout, n, stream):
        from .native import check
        d = dout
        for i in range(len(layers) - 1, -1, -1):
            m = layers[i]
            h = x if i == 0 else b["H"][i - 1]
            mean, istd = (norm.mean32.data_ptr(), norm.istd32.data_ptr()) if (i == 0 and norm is not None) else (None, None)
            # row blocks: enough workgroups to fill the chip (64 x 32 tiles over [W | b])
            tiles = -(-m.out_features // 64) * -(-(m.in_features + 1) // 32)
            splits = max(1, min(self.SPLITS, -(-self.WGRAD_TARGET // tiles), n // 64))
            check(self.lib.duck_mlp_wgrad(n, m.out_features, m.in_features, d.data_ptr(), h.data_ptr(), mean, istd,
                                          splits, self.part.data_ptr(), self.P, self.off[id(m.weight)],
                                          self.off[id(m.bias)], stream))
            if i > 0:
                dz = b["dZ"][i - 1]
                check(self.lib.duck_mlp_gemm(2, n, m.out_features, m.in_features, d.data_ptr(), m.weight.data_ptr(),
                                             None, b["Z"][i - 1].data_ptr(), dz.data_ptr(), None, None, None, stream))
                d = dz

    def gather(self, data: Dict[str, torch.Tensor], idx: torch.Tensor) -> Dict[str, torch.Tensor]:
        """The minibatch's trajectories (columns idx of the [T, B, ...] buffers) into persistent buffers:
        the value network's input [priv rows | the bootstrap rows] assembled in place (no cat), and of
        next_priv only the last step (the bootstrap observation; the rest is never read)."""
        from .native import DuckGatherField, check
        T, mb = data["reward"].shape[0], idx.numel()
        if not hasattr(self, "_mb"):
            self._mb = {k: torch.empty((T, mb) + v.shape[2:], device=v.device, dtype=v.dtype)
                        for k, v in data.items() if k not in ("priv", "next_priv")}
            self._xv = torch.empty(self.Nv, data["priv"].shape[-1], device=idx.device)
        if not hasattr(self.lib, "duck_gather_columns"):  # (A/B baselines built before the gather kernel)
            for k, buf in self._mb.items():
                torch.index_select(data[k], 1, idx, out=buf)
            torch.index_select(data["priv"], 1, idx, out=self._xv[:self.N].view(T, mb, -1))
            torch.index_select(data["next_priv"][-1], 0, idx, out=self._xv[self.N:])
            return {**self._mb, "xv": self._xv}
        # every field in one duck_gather_columns launch (the rollout buffers and these are persistent,
        # so the field table is built once; a captured learner graph replays the same pointers); with the
        # observation normalisers applied on the way (duck_gather_columns_norm), so the first layers'
        # GEMMs read plain rows
        on, pn = (self.net.obs_norm, self.net.priv_norm) if self.net.normalize else (None, None)
        pre = on is not None and hasattr(self.lib, "duck_gather_columns_norm")
        key = (tuple(v.data_ptr() for v in data.values()), idx.data_ptr(), pre)
        if getattr(self, "_gkey", None) != key:
            fl = []
            for k, buf in self._mb.items():
                v = data[k]
                fl.append((v, buf, v.shape[0], v.shape[1], v[0, 0].numel()))
            pv, npv = data["priv"], data["next_priv"]
            fl.append((pv, self._xv[:self.N], T, pv.shape[1], pv.shape[-1]))
            fl.append((npv[-1], self._xv[self.N:], 1, npv.shape[1], npv.shape[-1]))
            for v, _, _, _, _ in fl:
                if v.dtype != torch.float32 or not v.is_contiguous():
                    raise ValueError("duck_gather_columns needs contiguous float32 rollout buffers")
            self._gfields = (DuckGatherField * len(fl))(*[DuckGatherField(v.data_ptr(), d.data_ptr(), t, b, w)
                                                          for v, d, t, b, w in fl])
            if pre:
                names = list(self._mb) + ["priv", "next_priv"]
                ptr = []
                for k in names:
                    nm = on if k == "obs" else (pn if k in ("priv", "next_priv") else None)
                    ptr += [nm.mean32.data_ptr(), nm.istd32.data_ptr()] if nm is not None else [None, None]
                self._gnorm = (C.c_void_p * len(ptr))(*ptr)
            self._gkey = key
        if idx.dtype != torch.int64:
            raise ValueError("minibatch indices must be int64")
        st = torch.cuda.current_stream(idx.device).cuda_stream
        if pre:
            check(self.lib.duck_gather_columns_norm(len(self._gfields), self._gfields, self._gnorm, idx.data_ptr(), mb,
                                                    st))
            return {**self._mb, "xv": self._xv, "normalized": True}
        check(self.lib.duck_gather_columns(len(self._gfields), self._gfields, idx.data_ptr(), mb, st))
        return {**self._mb, "xv": self._xv}

    def __call__(self, mb: Dict[str, torch.Tensor], cfg: PPOConfig, gen: Optional[torch.Generator],
                 metrics: bool = True):
        """mb: the minibatch [T, B, ...] (gather's output, or any dict with obs, priv, next_priv, ...)"""
        from .native import check
        net = self.net
        T, B = mb["reward"].shape
        N = T * B
        if N != self.N or self.Nv != N + B:
            raise ValueError(f"FusedGrad was sized for {self.N} rows, got {T} x {B}")
        st = torch.cuda.current_stream(self.flat.device).cuda_stream
        # (gather's rows may already be normalised: then the first layers take no op(X))
        on, pn = (net.obs_norm, net.priv_norm) if net.normalize and not mb.get("normalized", False) else (None, None)
        obs = mb["obs"].reshape(N, -1)
        xv = mb["xv"] if "xv" in mb else torch.cat([mb["priv"].reshape(N, -1), mb["next_priv"][-1]], 0)
        grouped = hasattr(self.lib, "duck_mlp_group") and len(self.pol) == len(self.val)
        if grouped:
            for i in range(len(self.pol)):
                self._group([self._prob_fwd(self.pol, self.bp, obs, on, N, i),
                             self._prob_fwd(self.val, self.bv, xv, pn, self.Nv, i)], st)
            logits, v_all = self.bp["out"], self.bv["out"].view(-1)
        else:
            logits = self._forward(self.pol, self.bp, obs, on, N, st)
            v_all = self._forward(self.val, self.bv, xv, pn, self.Nv, st).view(-1)
        baseline, bootstrap = v_all[:N].view(T, B), v_all[N:]
        A = logits.shape[-1] // 2
        ra, olp = mb["raw_action"].contiguous(), mb["log_prob"].contiguous()
        if hasattr(self.lib, "duck_gae_stats") and B <= 1024:
            # GAE from the raw done / truncation / reward fields and the advantage statistics in one launch,
            # the loss with those statistics (round 6: 2 launches instead of 7 per minibatch)
            if getattr(self, "_vs", None) is None or self._vs.shape != (T, B):
                self._vs = torch.empty(T, B, device=logits.device)
                self._adv = torch.empty(T, B, device=logits.device)
                self._stats = torch.empty(2, device=logits.device)
            tr, dn, rw = (mb[k].contiguous() for k in ("truncation", "done", "reward"))
            check(self.lib.duck_gae_stats(T, B, tr.data_ptr(), dn.data_ptr(), rw.data_ptr(), float(cfg.reward_scaling),
                                          baseline.data_ptr(), bootstrap.data_ptr(), float(cfg.gae_lambda),
                                          float(cfg.discounting), self._vs.data_ptr(), self._adv.data_ptr(),
                                          int(bool(cfg.normalize_advantage)), self._stats.data_ptr(), st))
            eps = torch.randn((T, B, A), device=logits.device, generator=gen)  # the entropy sample (NormalTanh)
            # (metrics=False: the gradients without the loss sums, which only the reported minibatch needs)
            loss_fn = self.lib.duck_ppo_loss_stats if metrics or A > 16 or not hasattr(self.lib, "duck_ppo_loss_grad") \
                else self.lib.duck_ppo_loss_grad
            check(loss_fn(N, A, logits.data_ptr(), ra.data_ptr(), olp.data_ptr(),
                                               self._adv.data_ptr(), self._vs.data_ptr(), baseline.data_ptr(),
                                               eps.data_ptr(), float(cfg.clipping_epsilon), float(cfg.entropy_cost),
                                               self._stats.data_ptr(), self.loss_out.data_ptr(), self.g_lg.data_ptr(),
                                               self.d_val.data_ptr(), st))
        else:
            truncation = mb["truncation"]
            termination = mb["done"] * (1.0 - truncation)
            vs, adv = compute_gae(truncation, termination, mb["reward"] * cfg.reward_scaling, baseline, bootstrap,
                                  cfg.gae_lambda, cfg.discounting)
            eps = torch.randn((T, B, A), device=logits.device, generator=gen)  # the entropy sample, as NormalTanh draws it
            check(self.lib.duck_ppo_loss(N, A, logits.data_ptr(), ra.data_ptr(), olp.data_ptr(), adv.data_ptr(),
                                         vs.data_ptr(), baseline.data_ptr(), eps.data_ptr(), float(cfg.clipping_epsilon),
                                         float(cfg.entropy_cost), int(bool(cfg.normalize_advantage)),
                                         self.loss_out.data_ptr(), self.g_lg.data_ptr(), self.d_val.data_ptr(), st))
        if grouped:
            for i in range(len(self.pol) - 1, -1, -1):
                self._group(self._probs_bwd(self.pol, self.bp, obs, on, self.g_lg, N, i) +
                            self._probs_bwd(self.val, self.bv, xv, pn, self.d_val, self.Nv, i), st)
        else:
            self._backward(self.pol, self.bp, obs, on, self.g_lg, N, st)
            self._backward(self.val, self.bv, xv, pn, self.d_val, self.Nv, st)
        if not self.defer_reduce:
            check(self.lib.duck_mlp_wgrad_reduce(self.P, self.SPLITS, self.part.data_ptr(), self.flat.data_ptr(), st))
        o = self.loss_out
        return {"loss": o[0], "policy_loss": o[1], "v_loss": o[2], "entropy": o[3]}


def _fused_update(fg: "FusedGrad", cfg: PPOConfig) -> None:
    """clip_grad_norm_(max_grad_norm) + Adam(learning_rate) on FusedGrad's flat buffers (duck_clip_adam)"""
    from .native import check
    st = torch.cuda.current_stream(fg.flat.device).cuda_stream
    if fg.defer_reduce:  # the weight-gradient partials summed into fg.flat by the first launch
        check(fg.lib.duck_clip_adam_reduce(fg.P, fg.SPLITS, fg.part.data_ptr(), fg.pflat.data_ptr(), fg.flat.data_ptr(),
                                           fg.exp_avg.data_ptr(), fg.exp_avg_sq.data_ptr(), fg.adam_scratch.data_ptr(),
                                           fg.adam_step.data_ptr(), float(cfg.learning_rate), 0.9, 0.999, 1e-8,
                                           float(cfg.max_grad_norm or 0.0), st))
        return
    check(fg.lib.duck_clip_adam(fg.P, fg.pflat.data_ptr(), fg.flat.data_ptr(), fg.exp_avg.data_ptr(),
                                fg.exp_avg_sq.data_ptr(), fg.adam_scratch.data_ptr(), fg.adam_step.data_ptr(),
                                float(cfg.learning_rate), 0.9, 0.999, 1e-8, float(cfg.max_grad_norm or 0.0), st))


def fused_grad_available(device) -> bool:
    """the fused learner runs on the GPU when libduck.so exports the duck_mlp_* kernels
    (DUCK_PPO_FUSED_MLP=0 keeps the autograd learner)"""
    if torch.device(device).type != "cuda" or os.environ.get("DUCK_PPO_FUSED_MLP", "1") == "0":
        return False
    from .native import lib
    return hasattr(lib(), "duck_mlp_gemm")


def allreduce_grads(params: Sequence[torch.nn.Parameter]) -> None:
    """Data-parallel gradient mean over ranks: one flattened RCCL all-reduce (xGMI ring)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    grads = [p.grad for p in params if p.grad is not None]
    base = grads[0]._base if grads and grads[0]._base is not None else None
    if base is not None and all(g._base is base for g in grads) and base.numel() == sum(g.numel() for g in grads):
        dist.all_reduce(base)       # FusedGrad: every gradient is a view of one flat buffer
        base /= dist.get_world_size()
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat)
    flat /= dist.get_world_size()
    o = 0
    for g in grads:
        g.copy_(flat[o:o + g.numel()].view_as(g))
        o += g.numel()


def broadcast_params(module: nn.Module) -> None:
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, 0)


# ---------------------------------------------------------------------------------------
# training loop (brax ppo/train.py structure)
# ---------------------------------------------------------------------------------------
class _Learner:
    """One SGD minibatch step: gather -> loss -> backward -> (grad all-reduce) -> clip -> Adam.

    On the GPU the step is captured once into HIP graphs and replayed for every minibatch
    (≈300 small kernels per step would otherwise be launch-bound): graph 1 = gather + loss +
    backward into static grads, then the RCCL all-reduce runs eagerly (world > 1), graph 2 =
    global-norm clip + Adam. The first ``WARMUP`` steps run eagerly on a side stream (they are
    real updates, as torch's capture recipe requires), so the update sequence is unchanged.
    """

    WARMUP = 3

    def __init__(self, net: ActorCritic, opt, cfg: PPOConfig, data: Dict[str, torch.Tensor], mb: int,
                 device: torch.device, use_graph: bool, fused_mlp: Optional[bool] = None):
        self.net, self.opt, self.cfg, self.data = net, opt, cfg, data
        self.params = list(net.parameters())
        if fused_mlp is None:
            fused_mlp = fused_grad_available(device)
        T = cfg.unroll_length
        self.fused = FusedGrad(net, T * mb, mb, device) if fused_mlp else None
        world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        if self.fused is not None and world == 1 and hasattr(self.fused.lib, "duck_clip_adam_reduce"):
            self.fused.defer_reduce = True   # no all-reduce between the backward and the update
        self.idx = torch.zeros(mb, dtype=torch.long, device=device)
        self.use_graph = use_graph
        self.calls = 0
        self.g1 = self.g2 = None
        self.out = None

    def _fwd_bwd(self, idx: Optional[torch.Tensor] = None, metrics: bool = True):
        idx = self.idx if idx is None else idx
        if self.fused is not None:   # writes every .grad (views of one flat buffer)
            return self.fused(self.fused.gather(self.data, idx), self.cfg, None, metrics)
        mbatch = {k: v[:, idx] for k, v in self.data.items()}
        loss, m = ppo_loss(self.net, mbatch, self.cfg, None)
        # gradients set to None before the backward that is captured: it then writes them instead of
        # zero-filling and accumulating (one fill + one add kernel per parameter tensor saved)
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        return {"loss": loss.detach(), **m}

    def _apply(self):
        if self.fused is not None:
            _fused_update(self.fused, self.cfg)   # clip + Adam in two launches on the flat buffers
            return
        torch.nn.utils.clip_grad_norm_(self.params, self.cfg.max_grad_norm)
        self.opt.step()

    def step(self, idx: torch.Tensor) -> Dict[str, torch.Tensor]:
        self.idx.copy_(idx)
        self.calls += 1
        if not self.use_graph:
            out = self._fwd_bwd()
            allreduce_grads(self.params)
            self._apply()
            return out
        if self.calls <= self.WARMUP:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                out = self._fwd_bwd()
                allreduce_grads(self.params)
                self._apply()
            torch.cuda.current_stream().wait_stream(s)
            return out
        if self.g1 is None:
            self.g1, self.g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g1):
                self.out = self._fwd_bwd()
            with torch.cuda.graph(self.g2, pool=self.g1.pool()):
                self._apply()
        self.g1.replay()
        allreduce_grads(self.params)
        self.g2.replay()
        return self.out

    def _epoch_graph_ok(self) -> bool:
        world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        return self.use_graph and self.fused is not None and world == 1 and \
            os.environ.get("DUCK_PPO_EPOCH_GRAPH", "1") != "0"

    def epoch(self, perm: torch.Tensor, mb: int) -> Dict[str, torch.Tensor]:
        """One pass over the shuffled batch: minibatch k takes perm[k mb : (k + 1) mb]. With one rank and
        the fused learner the whole epoch -- every minibatch's gather, loss, backward, clip and Adam -- is
        ONE captured graph reading its indices from a static permutation buffer, replayed per epoch (round
        6: the per-minibatch replays cost a host round trip, an index copy, the generator-state fills of
        each replay and the gap between the two graphs, ~30 us of a ~390 us minibatch,
        profiles/r06_ppo_trace_summary_before.txt). Several ranks keep the per-minibatch graphs: the
        gradient all-reduce runs between them."""
        n = perm.numel() // mb
        if not self._epoch_graph_ok():
            out = None
            for k in range(n):
                out = self.step(perm[k * mb:(k + 1) * mb])
            return out
        if getattr(self, "eg", None) is None and self.calls < self.WARMUP:
            # the first epoch runs eagerly on a side stream (real updates: torch's capture recipe)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for k in range(n):
                    self.idx.copy_(perm[k * mb:(k + 1) * mb])
                    out = self._fwd_bwd()
                    self._apply()
            torch.cuda.current_stream().wait_stream(s)
            self.calls += n
            return out
        if getattr(self, "eg", None) is None:
            self.perm_buf = torch.empty_like(perm)
            self.eg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.eg):
                for k in range(n):
                    # (the loss sums of the epoch's last minibatch only: the others' are never read)
                    self.eout = self._fwd_bwd(self.perm_buf[k * mb:(k + 1) * mb], metrics=k == n - 1)
                    self._apply()
        self.perm_buf.copy_(perm)
        self.eg.replay()
        self.calls += n
        return self.eout


class _Rollout:
    """The unroll of ``train``: ``unroll_length`` env-steps of all envs with the policy sampling, every
    transition written in place into the time-major buffers. On the GPU the policy runs through the
    duck_mlp_gemm kernels (normaliser fused) and duck_policy_sample (NormalTanh sample, log-prob and
    tanh in one launch, counter-based threefry draws whose counter lives on the device), so the whole
    unroll -- policy, env.step, buffer writes -- is captured once as a HIP graph and replayed per
    update (~600 small launches per unroll otherwise). The first unroll runs eagerly (allocations)."""

    def __init__(self, env, net: ActorCritic, cfg: PPOConfig, data: Dict[str, torch.Tensor], unrolls: int,
                 device, use_graph: bool, seed: int):
        from .native import lib
        self.env, self.net, self.cfg, self.data = env, net, cfg, data
        self.unrolls, self.n = unrolls, env.num_envs
        self.lib = lib()
        self.pol = [m for m in net.policy if isinstance(m, nn.Linear)]
        n, dev = self.n, device
        self.Z = [torch.empty(n, m.out_features, device=dev) for m in self.pol[:-1]]
        self.H = [torch.empty(n, m.out_features, device=dev) for m in self.pol[:-1]]
        self.logits = torch.empty(n, self.pol[-1].out_features, device=dev)
        self.action = torch.empty(n, self.pol[-1].out_features // 2, device=dev)
        self.ctr = torch.zeros(1, dtype=torch.int32, device=dev)
        self.seed = (int(seed) * 0x9E3779B97F4A7C15 + 0x5EED) & 0xFFFFFFFFFFFFFFFF
        self.use_graph, self.calls, self.graph = use_graph, 0, None

    def _policy(self, obs: torch.Tensor, st) -> torch.Tensor:
        from .native import check
        norm = self.net.obs_norm if self.net.normalize else None
        inp = obs
        for i, m in enumerate(self.pol):
            last = i == len(self.pol) - 1
            check(self.lib.duck_mlp_gemm(0 if last else 1, self.n, m.in_features, m.out_features, inp.data_ptr(),
                                         m.weight.data_ptr(), m.bias.data_ptr(), None,
                                         (self.logits if last else self.Z[i]).data_ptr(),
                                         None if last else self.H[i].data_ptr(),
                                         norm.mean32.data_ptr() if (i == 0 and norm is not None) else None,
                                         norm.istd32.data_ptr() if (i == 0 and norm is not None) else None, st))
            if not last:
                inp = self.H[i]
        return self.logits

    def _store(self, pairs, st) -> None:
        """Rows [n, ...] into rows of the time-major buffers: every (source, destination) pair in one
        duck_gather_columns launch with the identity index (one launch per env-step instead of six
        copies); a pair that is not two contiguous float32 tensors is copied by torch."""
        from .native import DuckGatherField, check
        n = self.n
        if getattr(self, "_ident", None) is None:
            self._ident = torch.arange(n, dtype=torch.int64, device=self.logits.device)
        ok = [(a, b) for a, b in pairs if a.dtype == b.dtype == torch.float32 and a.is_contiguous()
              and b.is_contiguous() and a.numel() == b.numel() and a.numel() % n == 0]
        for a, b in pairs:
            if not any(a is x and b is y for x, y in ok):
                b.copy_(a)
        if not ok:
            return
        if not hasattr(self.lib, "duck_gather_columns"):
            for a, b in ok:
                b.copy_(a)
            return
        fl = (DuckGatherField * len(ok))(*[DuckGatherField(a.data_ptr(), b.data_ptr(), 1, n, a.numel() // n)
                                           for a, b in ok])
        check(self.lib.duck_gather_columns(len(ok), fl, self._ident.data_ptr(), n, st))

    def _unroll(self, state):
        from .native import check
        cfg, data, n = self.cfg, self.data, self.n
        st = torch.cuda.current_stream(self.logits.device).cuda_stream
        A = self.action.shape[1]
        pk, vk, T = cfg.policy_obs_key, cfg.value_obs_key, cfg.unroll_length
        for u in range(self.unrolls):
            cols = slice(u * n, (u + 1) * n)
            self._store([(state.obs[pk], data["obs"][0, cols]), (state.obs[vk], data["priv"][0, cols])], st)
            for t in range(T):
                logits = self._policy(state.obs[pk], st)
                check(self.lib.duck_policy_sample(n, A, logits.data_ptr(), self.seed, self.ctr.data_ptr(),
                                                  data["raw_action"][t, cols].data_ptr(),
                                                  data["log_prob"][t, cols].data_ptr(), self.action.data_ptr(), st))
                self.env.step(state, self.action, inplace=True)  # obs already copied out
                # the transition's outcome, and the observations the next env-step starts from (the
                # state's obs after this step: they are row t + 1 of obs / priv, and next_priv's last row
                # -- the only one the learner reads, the bootstrap observation)
                out = [(state.reward, data["reward"][t, cols]), (state.done, data["done"][t, cols]),
                       (state.info["truncation"], data["truncation"][t, cols])]
                if t + 1 < T:
                    out += [(state.obs[pk], data["obs"][t + 1, cols]), (state.obs[vk], data["priv"][t + 1, cols])]
                else:
                    out.append((state.obs[vk], data["next_priv"][t, cols]))
                self._store(out, st)

    @torch.no_grad()
    def run(self, state) -> None:
        self.calls += 1
        if not self.use_graph or self.calls == 1:
            self._unroll(state)
            return
        if self.graph is None:
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self._unroll(state)
        self.graph.replay()


@torch.no_grad()
def _torch_unroll(env, net: ActorCritic, cfg: PPOConfig, data: Dict[str, torch.Tensor], state, unrolls: int,
                  gen: torch.Generator) -> None:
    """The unroll with the torch policy and torch's normal sampler (CPU runs, DUCK_PPO_FUSED_MLP=0)."""
    n = env.num_envs
    for u in range(unrolls):
        cols = slice(u * n, (u + 1) * n)
        for t in range(cfg.unroll_length):
            obs, priv = state.obs[cfg.policy_obs_key], state.obs[cfg.value_obs_key]
            data["obs"][t, cols] = obs
            data["priv"][t, cols] = priv
            d = NormalTanh(net.policy_logits(obs))
            raw = d.sample_raw(gen)
            data["raw_action"][t, cols] = raw
            data["log_prob"][t, cols] = d.log_prob(raw)
            env.step(state, torch.tanh(raw), inplace=True)  # obs already copied out
            data["reward"][t, cols] = state.reward
            data["done"][t, cols] = state.done
            data["truncation"][t, cols] = state.info["truncation"]
            data["next_priv"][t, cols] = state.obs[cfg.value_obs_key]


def check_device_error(env, what: str) -> None:
    """Raise DuckError when a launch on ``env``'s handle set its sticky device error word
    (duck_device_error: e.g. a latency-kernel cross-wave wait that timed out and left NaN qpos in its
    workgroup's envs). Call after a synchronise: the word is written by the kernel itself."""
    err = env.device_error() if hasattr(env, "device_error") else 0
    if err:
        from .native import DuckError
        raise DuckError(f"device error word 0x{err:x} set during the {what} (duck_device_error): the "
                        "transitions of this batch are not valid")


@dataclass
class TrainResult:
    net: ActorCritic
    metrics: list = field(default_factory=list)
    env_steps: int = 0
    seconds: float = 0.0
    timing: dict = field(default_factory=lambda: {"rollout_s": 0.0, "learn_s": 0.0})


def train(env, cfg: PPOConfig, progress_fn: Optional[Callable[[int, dict], None]] = None,
          eval_env=None, max_updates: Optional[int] = None, device=None,
          policy_params_fn: Optional[Callable[[int, "ActorCritic"], None]] = None,
          restore_checkpoint_path: Optional[str] = None, use_graph: Optional[bool] = None) -> TrainResult:
    """Train on a batched env with the Joystick surface (reset(rng) / step(state, action)).

    ``env`` is already wrapped for training (episode length + auto-reset, DR if wanted) and
    holds this rank's ``num_envs / world`` envs. One update consumes ``batch_size *
    num_minibatches`` trajectories of ``unroll_length`` steps over all ranks; with the default
    config that is one unroll of all 8192 envs per update, as brax PPO does (train.py).
    """
    device = torch.device(device or env.device)
    if use_graph is None:
        use_graph = device.type == "cuda" and os.environ.get("DUCK_PPO_GRAPH", "1") != "0"
    rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    torch.manual_seed(cfg.seed + rank)
    gen = torch.Generator(device=device)
    gen.manual_seed(cfg.seed * 7919 + rank)
    obs_size = env.observation_size[cfg.policy_obs_key][0]
    priv_size = env.observation_size[cfg.value_obs_key][0]
    A = env.action_size
    net = ActorCritic(obs_size, priv_size, A, cfg).to(device)
    if restore_checkpoint_path is not None:  # brax: restores policy + normaliser (and value) params
        ck = torch.load(restore_checkpoint_path, map_location=device, weights_only=True)
        net.load_state_dict(ck["state_dict"])
    broadcast_params(net)
    # on the GPU the fused (single multi-tensor kernel) Adam, graph-capturable
    cuda = device.type == "cuda"
    opt = torch.optim.Adam(net.parameters(), lr=cfg.learning_rate, capturable=cuda, fused=cuda or None)
    n = env.num_envs  # envs on this rank (brax: num_envs // devices)
    traj_per_update = cfg.batch_size * cfg.num_minibatches // world  # this rank's share
    if traj_per_update % n != 0 or traj_per_update % cfg.num_minibatches != 0:
        raise ValueError("batch_size * num_minibatches / world must be a multiple of the envs per rank "
                         "and of num_minibatches (brax ppo.train asserts)")
    unrolls_per_update = traj_per_update // n
    steps_per_update = unrolls_per_update * cfg.unroll_length * n * world
    n_updates = max(1, cfg.num_timesteps // steps_per_update)
    if max_updates is not None:
        n_updates = min(n_updates, max_updates)
    T, B = cfg.unroll_length, traj_per_update
    mb = B // cfg.num_minibatches
    # rollout buffers, time-major [T, B, ...], written in place by the unroll (static for the graphs)
    shapes = {"obs": (obs_size,), "priv": (priv_size,), "raw_action": (A,), "log_prob": (), "reward": (),
              "done": (), "truncation": (), "next_priv": (priv_size,)}
    data = {k: torch.zeros((T, B) + sh, dtype=torch.float32, device=device) for k, sh in shapes.items()}
    learner = _Learner(net, opt, cfg, data, mb, device, use_graph)
    # the GPU unroll through the duck_mlp / duck_policy_sample kernels, graph-captured (DUCK_PPO_FUSED_MLP=0:
    # the torch policy and torch's normal sampler; also for models with more than 16 actuators, which
    # duck_policy_sample's one-lane-per-action-dim layout does not take)
    roller = _Rollout(env, net, cfg, data, unrolls_per_update, device, use_graph, cfg.seed * 7919 + rank) \
        if fused_grad_available(device) and A <= POLICY_SAMPLE_MAX_ACTIONS else None
    state = env.reset(rng=cfg.seed)  # streams are keyed by global env id: ranks draw disjoint envs
    result = TrainResult(net=net)
    # brax: num_evals evaluations spread evenly over training, the first before any update
    eval_every = max(1, n_updates // max(1, cfg.num_evals - 1)) if cfg.num_evals > 1 else None
    if eval_env is not None and cfg.num_evals > 0 and rank == 0:
        m0 = evaluate(net, eval_env, cfg, rng=cfg.seed + 10_007)
        if progress_fn is not None:
            progress_fn(0, m0)
    t0 = time.time()

    def _sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    for upd in range(n_updates):
        _sync()
        t_roll = time.time()
        # ---- rollouts: unroll_length env-steps of all envs, policy in inference mode ----
        if roller is not None:
            roller.run(state)
        else:
            _torch_unroll(env, net, cfg, data, state, unrolls_per_update, gen)
        _sync()
        # a replayed graph never re-enters duck_step, whose entry check would raise: read the
        # handle's sticky device error word here, before the batch reaches the learner
        check_device_error(env, "rollout")
        t_learn = time.time()
        result.timing["rollout_s"] += t_learn - t_roll
        if cfg.normalize_observations:  # brax updates the normaliser with the fresh batch first
            net.obs_norm.update(data["obs"])
            net.priv_norm.update(data["priv"])
        # ---- learning: epochs x shuffled minibatches of whole trajectories ----
        for _ in range(cfg.num_updates_per_batch):
            perm = torch.randperm(B, device=device, generator=gen)
            last = learner.epoch(perm, mb)
        _sync()
        result.timing["learn_s"] += time.time() - t_learn
        result.env_steps += steps_per_update
        rew = data["reward"].mean()
        if world > 1:
            dist.all_reduce(rew)
            rew /= world
        metrics = {"train/reward_per_step": float(rew),
                   **{f"train/{k}": float(v) for k, v in last.items()},
                   "env_steps": result.env_steps, "sps": result.env_steps / (time.time() - t0)}
        if eval_env is not None and rank == 0 and eval_every is not None and (
                (upd + 1) % eval_every == 0 or upd + 1 == n_updates):
            metrics.update(evaluate(net, eval_env, cfg, rng=cfg.seed + 10_007 + upd))
            if policy_params_fn is not None:
                policy_params_fn(result.env_steps, net)
        result.metrics.append(metrics)
        if progress_fn is not None and rank == 0:
            progress_fn(result.env_steps, metrics)
    result.seconds = time.time() - t0
    return result


@torch.no_grad()
def evaluate(net: ActorCritic, eval_env, cfg: PPOConfig, rng: int) -> Dict[str, float]:
    """brax Evaluator: one episode per eval env with the deterministic policy (tanh(loc)).

    ``eval_env`` is wrapped like the training env (auto-reset); as brax's EvalWrapper does,
    each env's return stops accumulating at its first ``done``.
    """
    state = eval_env.reset(rng=rng)
    n = eval_env.num_envs
    ret = torch.zeros(n, device=eval_env.device)
    length = torch.zeros(n, device=eval_env.device)
    active = torch.ones(n, device=eval_env.device)
    for _ in range(cfg.episode_length // cfg.action_repeat):
        act = NormalTanh(net.policy_logits(state.obs[cfg.policy_obs_key])).mode()
        eval_env.step(state, act, inplace=True)
        ret += state.reward * active
        length += active
        active = active * (1.0 - state.done)
    if eval_env.device.type == "cuda":
        torch.cuda.synchronize(eval_env.device)
    check_device_error(eval_env, "evaluation")   # the last launch is not followed by another duck_step
    return {"eval/episode_reward": float(ret.mean()), "eval/episode_reward_std": float(ret.std(unbiased=False)),
            "eval/avg_episode_length": float(length.mean())}


def save_checkpoint(net: ActorCritic, cfg: PPOConfig, path: str) -> None:
    """torch state_dict + config + sizes (the reference saves orbax params)."""
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    sizes = {"obs": net.policy[0].in_features, "priv": net.value[0].in_features,
             "action": net.policy[-1].out_features // 2}
    torch.save({"state_dict": net.state_dict(), "config": asdict(cfg), "sizes": sizes}, path)


def load_checkpoint(path: str, device="cpu") -> ActorCritic:
    ck = torch.load(path, map_location=device, weights_only=True)
    cfg = PPOConfig(**ck["config"])
    z = ck["sizes"]
    net = ActorCritic(z["obs"], z["priv"], z["action"], cfg).to(device)
    net.load_state_dict(ck["state_dict"])
    return net
