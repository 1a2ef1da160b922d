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
    net = ppo.load_checkpoint(str(tmp_path / "ck" / cks[-1]), 101, 172, 14, device=gpu)
    assert net.policy_logits(torch.zeros(2, 101, device=gpu)).shape == (2, 28)
    # resume from it
    runner.main(["--output_dir", "ck2", "--num_timesteps", str(20 * 256), "--num_eval_envs", "16",
                 "--restore_checkpoint_path", str(tmp_path / "ck" / cks[-1])])
