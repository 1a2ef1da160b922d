"""PPO outer loop: brax semantics restated in torch, checked on CPU.

The learner is independent of the env kernel, so these tests drive it with a small torch env
that has the Joystick surface (``reset(rng)`` / in-place ``step(state, action)``, dict obs,
``done`` / ``info["truncation"]``) — no GPU needed. ``test_gpu_ppo`` in test_gpu_env.py drives
the real HIP env.
"""

import math
import os
import socket
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from open_duck_playground_amd import ppo


# ---------------------------------------------------------------------------------------
class ToyEnv:
    """Track a target: obs = target in [-0.8, 0.8]^A, reward = 1 - mean |action - target|.

    Episodes end after ``episode_length`` steps (truncation) or, for env ids in the upper
    half, when |action - target| > 0.9 everywhere (termination); both auto-reset.
    """

    action_size = 3

    def __init__(self, num_envs=64, episode_length=16, seed=0):
        self.num_envs, self.episode_length, self.device = num_envs, episode_length, torch.device("cpu")
        self.seed, self.g = seed, torch.Generator().manual_seed(seed)
        self.observation_size = {"state": (self.action_size,), "privileged_state": (self.action_size + 1,)}

    def _target(self, n):
        return (torch.rand(n, self.action_size, generator=self.g) * 1.6 - 0.8)

    def reset(self, rng=0):
        self.g.manual_seed(rng * 1000 + self.seed)  # like the env's global-id keyed streams
        t = self._target(self.num_envs)
        steps = torch.zeros(self.num_envs)
        return SimpleNamespace(obs={"state": t, "privileged_state": torch.cat([t, steps[:, None]], 1)},
                               reward=torch.zeros(self.num_envs), done=torch.zeros(self.num_envs),
                               info={"truncation": torch.zeros(self.num_envs), "steps": steps})

    def step(self, state, action, inplace=True):  # in place, like Joystick.step(..., inplace=True)
        t = state.obs["state"]
        err = (action - t).abs()
        state.reward.copy_(1.0 - err.mean(1))
        steps = state.info["steps"] + 1
        term = (err.min(1).values > 0.9) & (torch.arange(self.num_envs) >= self.num_envs // 2)
        trunc = (steps >= self.episode_length) & ~term
        done = term | trunc
        state.done.copy_(done.float())
        state.info["truncation"].copy_(trunc.float())
        steps = torch.where(done, torch.zeros_like(steps), steps)
        new_t = torch.where(done[:, None], self._target(self.num_envs), t)
        state.info["steps"] = steps
        state.obs["state"] = new_t
        state.obs["privileged_state"] = torch.cat([new_t, steps[:, None] / self.episode_length], 1)
        return state


def small_cfg(**kw):
    base = dict(num_timesteps=10 ** 9, num_evals=0, episode_length=16, unroll_length=8, num_minibatches=4,
                num_updates_per_batch=2, num_envs=64, batch_size=16, learning_rate=1e-3,
                policy_hidden_layer_sizes=(32, 32), value_hidden_layer_sizes=(32, 32))
    base.update(kw)
    return ppo.PPOConfig(**base)


# ---------------------------------------------------------------------------------------
def gae_numpy(truncation, termination, rewards, values, bootstrap, lam, discount):
    """Straight-line restatement of brax losses.compute_gae (one env column at a time)."""
    T, B = rewards.shape
    vs = np.zeros_like(values)
    adv = np.zeros_like(values)
    for b in range(B):
        acc = 0.0
        vnext = np.append(values[1:, b], bootstrap[b])
        delta = (rewards[:, b] + discount * (1 - termination[:, b]) * vnext - values[:, b]) * (1 - truncation[:, b])
        for t in reversed(range(T)):
            acc = delta[t] + discount * (1 - termination[t, b]) * (1 - truncation[t, b]) * lam * acc
            vs[t, b] = acc + values[t, b]
        vsn = np.append(vs[1:, b], bootstrap[b])
        adv[:, b] = (rewards[:, b] + discount * (1 - termination[:, b]) * vsn - values[:, b]) * (1 - truncation[:, b])
    return vs, adv


def test_gae_matches_restatement():
    rng = np.random.default_rng(0)
    T, B = 20, 7
    r, v, boot = rng.normal(size=(T, B)), rng.normal(size=(T, B)), rng.normal(size=B)
    done = (rng.random((T, B)) < 0.15).astype(np.float64)
    trunc = done * (rng.random((T, B)) < 0.5)
    term = done * (1 - trunc)
    vs, adv = ppo.compute_gae(*(torch.tensor(a) for a in (trunc, term, r, v, boot)), 0.95, 0.97)
    vs_n, adv_n = gae_numpy(trunc, term, r, v, boot, 0.95, 0.97)
    np.testing.assert_allclose(vs.numpy(), vs_n, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(adv.numpy(), adv_n, rtol=1e-12, atol=1e-12)


def test_gae_no_done_is_discounted_lambda_return():
    # with no episode ends and lambda = 1, vs is the discounted return bootstrapped at T
    T = 6
    r = torch.arange(1.0, T + 1, dtype=torch.float64)[:, None]
    v = torch.zeros(T, 1, dtype=torch.float64)
    z = torch.zeros(T, 1, dtype=torch.float64)
    vs, _ = ppo.compute_gae(z, z, r, v, torch.tensor([2.0], dtype=torch.float64), 1.0, 0.9)
    exp = sum(0.9 ** k * (k + 1) for k in range(T)) + 0.9 ** T * 2.0
    assert abs(float(vs[0, 0]) - exp) < 1e-12


def test_normal_tanh_log_prob_and_entropy():
    torch.manual_seed(0)
    logits = torch.randn(5, 8, dtype=torch.float64)
    d = ppo.NormalTanh(logits)
    raw = d.sample_raw()
    loc, raw_scale = logits.chunk(2, -1)
    scale = torch.nn.functional.softplus(raw_scale) + 1e-3
    td = torch.distributions.TransformedDistribution(torch.distributions.Normal(loc, scale),
                                                     [torch.distributions.TanhTransform()])
    exp = td.log_prob(torch.tanh(raw)).sum(-1)
    np.testing.assert_allclose(d.log_prob(raw).numpy(), exp.numpy(), rtol=1e-6, atol=1e-6)
    # entropy = Normal entropy + E[log|J|]: its mean over many draws matches a Monte Carlo estimate
    g = torch.Generator().manual_seed(1)
    ents = torch.stack([d.entropy(g) for _ in range(4000)]).mean(0)
    mc = -torch.stack([td.log_prob(torch.tanh(td.base_dist.sample())).sum(-1) for _ in range(4000)]).mean(0)
    np.testing.assert_allclose(ents.numpy(), mc.numpy(), rtol=0.05, atol=0.05)
    np.testing.assert_allclose(d.mode().numpy(), torch.tanh(loc).numpy())


def test_running_statistics_matches_numpy():
    rng = np.random.default_rng(3)
    rs = ppo.RunningStatistics(4)
    x0 = torch.randn(3, 4)
    assert torch.allclose(rs.normalize(x0), x0)  # identity before any update
    batches = [rng.normal(loc=[0, 5, -3, 100], scale=[1, 0.1, 4, 20], size=(n, 4)) for n in (10, 37, 1, 200)]
    for b in batches:
        rs.update(torch.tensor(b, dtype=torch.float32))
    allx = np.concatenate(batches).astype(np.float32).astype(np.float64)
    np.testing.assert_allclose(rs.mean.numpy(), allx.mean(0), rtol=1e-10, atol=1e-10)
    np.testing.assert_allclose(rs.std.numpy(), allx.std(0), rtol=1e-9)
    assert int(rs.count) == len(allx)


def test_mlp_init_and_shapes():
    net = ppo.ActorCritic(101, 172, 14, ppo.PPOConfig())
    sizes = [m.out_features for m in net.policy if isinstance(m, torch.nn.Linear)]
    assert sizes == [512, 256, 128, 28]
    assert isinstance(net.policy[1], torch.nn.SiLU)
    assert net.value_of(torch.zeros(3, 172)).shape == (3,)
    w = net.policy[0].weight
    assert float(w.detach().abs().max()) <= math.sqrt(3.0 / 101) + 1e-6


def test_ppo_learns_toy_env():
    torch.manual_seed(0)
    env = ToyEnv()
    cfg = small_cfg(num_timesteps=64 * 8 * 60)
    res = ppo.train(env, cfg)
    first = np.mean([m["train/reward_per_step"] for m in res.metrics[:3]])
    last = np.mean([m["train/reward_per_step"] for m in res.metrics[-3:]])
    assert res.env_steps == 64 * 8 * 60 and len(res.metrics) == 60
    assert last > first + 0.15, (first, last)
    ev = ppo.evaluate(res.net, ToyEnv(num_envs=32, seed=5), cfg, rng=9)
    assert ev["eval/episode_reward"] > 0.75 * cfg.episode_length


class FaultyToyEnv(ToyEnv):
    """ToyEnv whose handle reports a sticky device error word after ``fail_after`` steps, the way
    libduck's duck_device_error does after a latency-kernel wait timed out. Its step never raises
    itself, as a replayed HIP graph never re-enters duck_step's entry check."""

    def __init__(self, fail_after, **kw):
        super().__init__(**kw)
        self.fail_after, self.steps = fail_after, 0

    def step(self, state, action, inplace=True):
        self.steps += 1
        return super().step(state, action, inplace)

    def device_error(self, clear=False):
        return 1 if self.steps > self.fail_after else 0


def test_train_raises_on_device_error_word():
    """training must not run on after a launch set the device error word (NaN qpos in a
    workgroup's envs): train() reads it after every rollout and raises DuckError."""
    from open_duck_playground_amd.native import DuckError
    env = FaultyToyEnv(fail_after=8 * 3 + 2)   # clean for 3 unrolls of 8 steps, faults in the 4th
    res = []
    with pytest.raises(DuckError, match="device error word 0x1 set during the rollout"):
        ppo.train(env, small_cfg(), max_updates=6, progress_fn=lambda s, m: res.append(s))
    assert res == [512, 1024, 1536]     # the three clean updates completed, the faulty batch did not
    with pytest.raises(DuckError, match="during the evaluation"):
        ppo.evaluate(ppo.ActorCritic(3, 4, 3, small_cfg()), FaultyToyEnv(fail_after=3, num_envs=8), small_cfg(), rng=0)


def test_batch_size_contract():
    env = ToyEnv(num_envs=48)
    with pytest.raises(ValueError):
        ppo.train(env, small_cfg(num_envs=48), max_updates=1)


def test_checkpoint_roundtrip(tmp_path):
    env = ToyEnv()
    cfg = small_cfg()
    res = ppo.train(env, cfg, max_updates=2)
    p = str(tmp_path / "ck.pt")
    ppo.save_checkpoint(res.net, cfg, p)
    net2 = ppo.load_checkpoint(p)
    x = torch.randn(5, 3)
    assert torch.equal(net2.policy_logits(x), res.net.policy_logits(x))
    # restore resumes from the same parameters (normaliser buffers included)
    res2 = ppo.train(env, cfg, max_updates=0, restore_checkpoint_path=p)
    assert torch.equal(res2.net.policy_logits(x), res.net.policy_logits(x))
    assert torch.equal(res2.net.obs_norm.std, res.net.obs_norm.std)


# ---------------------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    env = ToyEnv(num_envs=32, seed=rank)  # this rank's half of 64 envs
    cfg = small_cfg(num_envs=64)
    res = ppo.train(env, cfg, max_updates=3, device=torch.device("cpu"))
    flat = torch.cat([p.detach().reshape(-1) for p in res.net.parameters()])
    out[rank] = (flat.numpy().copy(), res.net.obs_norm.mean.numpy().copy(), int(res.net.obs_norm.count),
                 res.env_steps)
    torch.distributed.destroy_process_group()


def test_two_rank_data_parallel_stays_in_sync():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    (p0, m0, c0, s0), (p1, m1, c1, s1) = out[0], out[1]
    assert np.array_equal(p0, p1)  # identical init (broadcast) + all-reduced grads -> identical params
    assert np.array_equal(m0, m1) and c0 == c1 == 3 * 8 * 64  # normaliser saw both ranks' batches
    assert s0 == s1 == 3 * 8 * 64


@pytest.mark.parametrize("n,out", [(5120, 256), (4096, 28), (100, 64), (5120, 1)])
def test_split_k_linear_matches_linear(n, out):
    """SplitKLinear: the same outputs and gradients as nn.Linear (split-K weight gradient for deep
    batches, the plain product otherwise)."""
    torch.manual_seed(0)
    a = ppo.SplitKLinear(37, out)
    b = torch.nn.Linear(37, out)
    b.load_state_dict(a.state_dict())
    x1 = torch.randn(n, 37, requires_grad=True)
    x2 = x1.detach().clone().requires_grad_(True)
    gy = torch.randn(n, out)
    ya, yb = a(x1), b(x2)
    assert torch.allclose(ya, yb, atol=1e-6)
    ya.backward(gy)
    yb.backward(gy)
    assert torch.allclose(x1.grad, x2.grad, atol=1e-5)
    assert torch.allclose(a.weight.grad, b.weight.grad, rtol=1e-5, atol=1e-4)
    assert torch.allclose(a.bias.grad, b.bias.grad, rtol=1e-5, atol=1e-4)


def test_grouped_launch_row_tiles(monkeypatch):
    """FusedGrad._row_tile on the learner's grouped launches (5,120-row minibatch, 512-256-128 MLPs, 101 / 172
    inputs, 14 actions): 64-row tiles where many tiles or a long reduction fill the chip, 32-row tiles for the
    third / fourth layers and the deepest backward launches (profiles/r06_ppo_tiles_ab.txt)."""
    from open_duck_playground_amd.native import DuckMlpProblem

    def gemm(kind, n, r, m):
        return DuckMlpProblem(kind, n, r, m, None, None, None, None, None, None, None, None, 0, 0, 0, 0, None)

    def wgrad(n, r, m, splits):
        return DuckMlpProblem(3, n, r, m, None, None, None, None, None, None, None, None, splits, 0, 0, 0, None)

    N, Nv = 5120, 5376
    rt = ppo.FusedGrad._row_tile
    assert rt([gemm(1, N, 101, 512), gemm(1, Nv, 172, 512)]) == 64            # first layers' forward
    assert rt([gemm(1, N, 512, 256), gemm(1, Nv, 512, 256)]) == 64            # second layers: long reduction
    assert rt([gemm(1, N, 256, 128), gemm(1, Nv, 256, 128)]) == 32            # third layers
    assert rt([gemm(0, N, 128, 28), gemm(0, Nv, 128, 1)]) == 32               # heads
    assert rt([wgrad(N, 256, 512, 12), gemm(2, N, 256, 512),                   # dgrad of the first layers
               wgrad(Nv, 256, 512, 12), gemm(2, Nv, 256, 512)]) == 64
    assert rt([wgrad(N, 128, 256, 16), gemm(2, N, 128, 256),
               wgrad(Nv, 128, 256, 16), gemm(2, Nv, 128, 256)]) == 32
    monkeypatch.setenv("DUCK_MLP_BM_AUTO", "0")
    assert rt([gemm(1, N, 256, 128)]) == 64
