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
    """brax_ppo_config("BerkeleyHumanoidJoystickFlatTerrain") as the reference runner uses it."""
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
def mlp(sizes: Sequence[int], out: int) -> nn.Sequential:
    layers, prev = [], sizes[0]
    for h in sizes[1:]:
        layers += [nn.Linear(prev, h), nn.SiLU()]
        prev = h
    layers.append(nn.Linear(prev, out))
    for m in layers:  # brax: lecun_uniform kernels, zero bias
        if isinstance(m, nn.Linear):
            bound = math.sqrt(3.0 / m.in_features)
            nn.init.uniform_(m.weight, -bound, bound)
            nn.init.zeros_(m.bias)
    return nn.Sequential(*layers)


MIN_STD = 1e-3


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
        self.std_eps, self.std_min, self.std_max = std_eps, std_min, std_max

    @torch.no_grad()
    def update(self, x: torch.Tensor) -> None:
        """Fold a batch [..., size] in (parallel-variance merge; one all-reduce across ranks)."""
        x = x.reshape(-1, x.shape[-1]).to(torch.float64)
        k = x.shape[-1]
        stats = torch.cat([torch.full((1,), float(x.shape[0]), dtype=torch.float64, device=x.device),
                           x.sum(0), (x * x).sum(0)])
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

    def normalize(self, x: torch.Tensor) -> torch.Tensor:
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
def compute_gae(truncation: torch.Tensor, termination: torch.Tensor, rewards: torch.Tensor, values: torch.Tensor,
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


def ppo_loss(net: ActorCritic, batch: Dict[str, torch.Tensor], cfg: PPOConfig, gen: Optional[torch.Generator]):
    """batch tensors are time-major [T, B, ...]; returns (loss, metrics)."""
    logits = net.policy_logits(batch["obs"])
    baseline = net.value_of(batch["priv"])
    bootstrap = net.value_of(batch["next_priv"][-1])
    rewards = batch["reward"] * cfg.reward_scaling
    truncation = batch["truncation"]
    termination = batch["done"] * (1.0 - truncation)
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


def allreduce_grads(params: Sequence[torch.nn.Parameter]) -> None:
    """Data-parallel gradient mean over ranks: one flattened RCCL all-reduce (xGMI ring)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    grads = [p.grad for p in params if p.grad is not None]
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
          restore_checkpoint_path: Optional[str] = None) -> TrainResult:
    """Train on a batched env with the Joystick surface (reset(rng) / step(state, action)).

    ``env`` is already wrapped for training (episode length + auto-reset, DR if wanted) and
    holds ``cfg.num_envs`` envs (per rank). One update consumes ``batch_size * num_minibatches``
    trajectories of ``unroll_length`` steps; with the default config that is one unroll of all
    8192 envs per update, as brax PPO does.
    """
    device = torch.device(device or env.device)
    rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    torch.manual_seed(cfg.seed + rank)
    gen = torch.Generator(device=device)
    gen.manual_seed(cfg.seed * 7919 + rank)
    obs_size = env.observation_size[cfg.policy_obs_key][0]
    priv_size = env.observation_size[cfg.value_obs_key][0]
    net = ActorCritic(obs_size, priv_size, env.action_size, cfg).to(device)
    if restore_checkpoint_path is not None:  # brax: restores policy + normaliser (and value) params
        ck = torch.load(restore_checkpoint_path, map_location=device, weights_only=True)
        net.load_state_dict(ck["state_dict"])
    broadcast_params(net)
    opt = torch.optim.Adam(net.parameters(), lr=cfg.learning_rate)
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
    state = env.reset(rng=cfg.seed)  # streams are keyed by global env id: ranks draw disjoint envs
    result = TrainResult(net=net)
    # brax: num_evals evaluations spread evenly over training, the first before any update
    eval_every = max(1, n_updates // max(1, cfg.num_evals - 1)) if cfg.num_evals > 1 else None
    if eval_env is not None and cfg.num_evals > 0 and rank == 0:
        m0 = evaluate(net, eval_env, cfg, rng=cfg.seed + 10_007)
        if progress_fn is not None:
            progress_fn(0, m0)
    t0 = time.time()
    T = cfg.unroll_length

    def _sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    for upd in range(n_updates):
        _sync()
        t_roll = time.time()
        # ---- rollouts: unroll_length env-steps of all envs, policy in inference mode ----
        chunks = []
        for _ in range(unrolls_per_update):
            buf = {k: [] for k in ("obs", "priv", "raw_action", "log_prob", "reward", "done", "truncation", "next_priv")}
            with torch.no_grad():
                for t in range(T):
                    obs = state.obs[cfg.policy_obs_key].clone()
                    priv = state.obs[cfg.value_obs_key].clone()
                    d = NormalTanh(net.policy_logits(obs))
                    raw = d.sample_raw(gen)
                    buf["obs"].append(obs)
                    buf["priv"].append(priv)
                    buf["raw_action"].append(raw)
                    buf["log_prob"].append(d.log_prob(raw))
                    env.step(state, torch.tanh(raw))
                    buf["reward"].append(state.reward.clone())
                    buf["done"].append(state.done.clone())
                    buf["truncation"].append(state.info["truncation"].clone())
                    buf["next_priv"].append(state.obs[cfg.value_obs_key].clone())
            chunks.append({k: torch.stack(v) for k, v in buf.items()})  # [T, n, ...]
        data = {k: torch.cat([c[k] for c in chunks], dim=1) for k in chunks[0]}  # [T, B, ...]
        _sync()
        t_learn = time.time()
        result.timing["rollout_s"] += t_learn - t_roll
        if cfg.normalize_observations:  # brax updates the normaliser with the fresh batch first
            net.obs_norm.update(data["obs"])
            net.priv_norm.update(data["priv"])
        # ---- learning: epochs x shuffled minibatches of whole trajectories ----
        B = data["obs"].shape[1]
        mb = B // cfg.num_minibatches
        last = {}
        for _ in range(cfg.num_updates_per_batch):
            perm = torch.randperm(B, device=device, generator=gen)
            for i in range(0, B - mb + 1, mb):
                idx = perm[i:i + mb]
                mbatch = {k: v[:, idx] for k, v in data.items()}
                loss, m = ppo_loss(net, mbatch, cfg, gen)
                opt.zero_grad(set_to_none=True)
                loss.backward()
                allreduce_grads(list(net.parameters()))
                torch.nn.utils.clip_grad_norm_(net.parameters(), cfg.max_grad_norm)
                opt.step()
                last = m
        _sync()
        result.timing["learn_s"] += time.time() - t_learn
        result.env_steps += steps_per_update
        rew = data["reward"].mean()
        if world > 1:
            dist.all_reduce(rew)
            rew /= world
        metrics = {"train/reward_per_step": float(rew), "train/loss": float(loss.detach()),
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
        eval_env.step(state, act)
        ret += state.reward * active
        length += active
        active = active * (1.0 - state.done)
    return {"eval/episode_reward": float(ret.mean()), "eval/episode_reward_std": float(ret.std(unbiased=False)),
            "eval/avg_episode_length": float(length.mean())}


def save_checkpoint(net: ActorCritic, cfg: PPOConfig, path: str) -> None:
    """torch state_dict + config (the reference saves orbax params)."""
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    torch.save({"state_dict": net.state_dict(), "config": asdict(cfg)}, path)


def load_checkpoint(path: str, obs_size: int, priv_size: int, action_size: int, device="cpu") -> ActorCritic:
    ck = torch.load(path, map_location=device, weights_only=True)
    cfg = PPOConfig(**ck["config"])
    net = ActorCritic(obs_size, priv_size, action_size, cfg).to(device)
    net.load_state_dict(ck["state_dict"])
    return net
