"""PPO outer loop on the HIP env: rollouts through libduck, learner in torch."""

import json
import os

import numpy as np
import pytest
import torch

from open_duck_playground_amd import ppo, runner
from open_duck_playground_amd.joystick import Joystick, domain_randomize, wrap_for_brax_training

pytestmark = pytest.mark.gpu


def test_ppo_updates_on_hip_env(gpu):
    n = 512
    env = wrap_for_brax_training(Joystick("flat_terrain", num_envs=n, device=gpu), episode_length=1000,
                                 randomization_fn=domain_randomize, rng=3)
    cfg = ppo.PPOConfig(num_envs=n, batch_size=16, num_minibatches=32, num_evals=0)
    res = ppo.train(env, cfg, max_updates=3)
    assert len(res.metrics) == 3 and res.env_steps == 3 * 20 * n
    for m in res.metrics:
        assert all(np.isfinite(v) for v in m.values())
    assert int(res.net.obs_norm.count) == 3 * 20 * n
    # the normaliser follows the obs: home-pose joint offsets (state[13:27]) stay near 0
    assert float(res.net.obs_norm.mean[13:27].abs().max()) < 0.5
    ev = ppo.evaluate(res.net, wrap_for_brax_training(Joystick("flat_terrain", num_envs=32, device=gpu),
                                                      episode_length=50), ppo.PPOConfig(episode_length=50), rng=1)
    assert np.isfinite(ev["eval/episode_reward"]) and 1 <= ev["eval/avg_episode_length"] <= 50


def test_runner_cli_one_update(gpu, tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    monkeypatch.setattr(runner.BaseRunner, "make_ppo_params",
                        lambda self: ppo.PPOConfig(num_timesteps=self.num_timesteps, num_envs=256, batch_size=8,
                                                   num_minibatches=32, episode_length=40, num_evals=2))
    runner.main(["--output_dir", "ck", "--num_timesteps", str(2 * 20 * 256), "--num_eval_envs", "16"])
    lines = [json.loads(x) for x in open(tmp_path / "ck" / "metrics.jsonl")]
    assert lines[0]["step"] == 0 and "eval/episode_reward" in lines[0]
    assert lines[-1]["step"] == 2 * 20 * 256
    cks = sorted(p for p in os.listdir(tmp_path / "ck") if p.endswith(".pt"))
    assert cks, os.listdir(tmp_path / "ck")
    assert os.path.exists(tmp_path / "ck" / cks[-1].replace(".pt", ".onnx"))
    net = ppo.load_checkpoint(str(tmp_path / "ck" / cks[-1]), device=gpu)
    assert net.policy_logits(torch.zeros(2, 101, device=gpu)).shape == (2, 28)
    # resume from it
    runner.main(["--output_dir", "ck2", "--num_timesteps", str(20 * 256), "--num_eval_envs", "16",
                 "--restore_checkpoint_path", str(tmp_path / "ck" / cks[-1])])


def test_graph_learner_matches_eager(gpu):
    """The HIP-graph learner replays the same update sequence as the eager one.

    entropy_cost = 0 takes the learner's only random draw (the entropy sample) out of the
    gradients, so both paths see identical numbers and differ only if the graph is wrong.
    """
    out = []
    for use_graph in (False, True):
        env = wrap_for_brax_training(Joystick("flat_terrain", num_envs=256, device=gpu), episode_length=1000)
        cfg = ppo.PPOConfig(num_envs=256, batch_size=8, num_minibatches=32, num_evals=0, entropy_cost=0.0)
        res = ppo.train(env, cfg, max_updates=2, use_graph=use_graph)
        out.append(torch.cat([p.detach().reshape(-1) for p in res.net.parameters()]))
    err = (out[0] - out[1]).abs().max().item()
    assert err < 1e-5, err


@pytest.mark.parametrize("T,B", [(20, 5120), (7, 1000), (1, 3), (0, 4), (5, 0)])
def test_gae_kernel_matches_restatement(gpu, T, B):
    from tests.test_ppo import gae_numpy
    rng = np.random.default_rng(T * 1000 + B)
    r, v, boot = rng.normal(size=(T, B)), rng.normal(size=(T, B)), rng.normal(size=B)
    done = (rng.random((T, B)) < 0.1).astype(np.float64)
    trunc = done * (rng.random((T, B)) < 0.5)
    term = done * (1 - trunc)
    f32 = [x.astype(np.float32).astype(np.float64) for x in (trunc, term, r, v, boot)]
    ins = [torch.tensor(x, dtype=torch.float32, device=gpu) for x in f32]
    vs, adv = ppo.compute_gae(*ins, 0.95, 0.97)
    vs_n, adv_n = gae_numpy(*f32, 0.95, 0.97)
    np.testing.assert_allclose(vs.cpu().numpy(), vs_n, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(adv.cpu().numpy(), adv_n, rtol=1e-5, atol=1e-5)


def test_runner_standing_env(gpu, tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    monkeypatch.setattr(runner.BaseRunner, "make_ppo_params",
                        lambda self: ppo.PPOConfig(num_timesteps=self.num_timesteps, num_envs=256, batch_size=8,
                                                   num_minibatches=32, episode_length=40, num_evals=0))
    runner.main(["--output_dir", "ck", "--env", "standing", "--num_timesteps", str(20 * 256)])
    line = json.loads(open(tmp_path / "ck" / "metrics.jsonl").readline())
    assert line["step"] == 20 * 256 and np.isfinite(line["train/loss"])
