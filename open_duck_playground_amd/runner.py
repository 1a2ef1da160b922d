"""Training runner for Open Duck Mini v2 on MI355X (open_duck_mini_v2/runner.py + common/runner.py).

Same command line as the reference's ``python -m playground.open_duck_mini_v2.runner``:
``--output_dir``, ``--num_timesteps``, ``--env``, ``--task``, ``--restore_checkpoint_path``.
Differences: the learner is ``ppo.train`` (PyTorch on the GPU, RCCL gradient all-reduce when
launched one process per GPU under ``torch.distributed.run``); checkpoints are torch state
dicts (``<output_dir>/<date>_<step>.pt``) instead of orbax trees, each written next to its
ONNX policy (``onnx_export``, same contract as common/export_onnx.py); metrics go to a JSON-lines
file (``<output_dir>/metrics.jsonl``) instead of tensorboardX, which is not installed here.
"""

from __future__ import annotations

import argparse
import json
import os
from dataclasses import asdict, replace
from datetime import datetime
from pathlib import Path

import torch
import torch.distributed as dist

from .onnx_export import export_onnx
from .joystick import Joystick, domain_randomize, wrap_for_brax_training
from .ppo import ActorCritic, PPOConfig, save_checkpoint, train
from .sharding import shard_from_env
from .standing import Standing


class BaseRunner:
    """common/runner.py:24-118."""

    def __init__(self, args: argparse.Namespace) -> None:
        self.args = args
        self.output_dir = Path.cwd() / Path(args.output_dir)
        self.num_timesteps = args.num_timesteps
        self.restore_checkpoint_path = None
        self.env = None
        self.eval_env = None
        self.randomizer = None
        self.rank = 0

    def progress_callback(self, num_steps: int, metrics: dict) -> None:
        os.makedirs(self.output_dir, exist_ok=True)
        # which step kernel ran (include/duck.h DUCK_STEP_*; the kernels agree bit for bit, recorded for
        # the run's provenance)
        kernels = {"train": getattr(self.env, "step_kernel", None)}
        if self.eval_env is not None:
            kernels["eval"] = getattr(self.eval_env, "step_kernel", None)
        with open(self.output_dir / "metrics.jsonl", "a") as f:
            f.write(json.dumps({"step": num_steps, **metrics, "step_kernel": kernels}) + "\n")
        if "eval/episode_reward" in metrics:
            print("-----------")
            print(f'STEP: {num_steps} reward: {metrics["eval/episode_reward"]} '
                  f'reward_std: {metrics["eval/episode_reward_std"]}')
            print("-----------")

    def policy_params_fn(self, current_step: int, net: ActorCritic) -> None:
        d = datetime.now().strftime("%Y_%m_%d_%H%M%S")
        path = f"{self.output_dir}/{d}_{current_step}.pt"
        print(f"Saving checkpoint (step: {current_step}): {path}")
        save_checkpoint(net, self.ppo_params, path)
        export_onnx(net, self.action_size, self.obs_size, output_path=f"{self.output_dir}/{d}_{current_step}.onnx")

    def make_ppo_params(self) -> PPOConfig:
        return replace(PPOConfig(), num_timesteps=self.num_timesteps)

    def train(self, max_updates=None):
        self.ppo_params = self.make_ppo_params()
        if self.rank == 0:
            print(f"PPO params: {asdict(self.ppo_params)}")
        return train(self.env, self.ppo_params, progress_fn=self.progress_callback, eval_env=self.eval_env,
                     policy_params_fn=self.policy_params_fn, restore_checkpoint_path=self.restore_checkpoint_path,
                     max_updates=max_updates)


class OpenDuckMiniV2Runner(BaseRunner):
    """open_duck_mini_v2/runner.py:11-31: env + eval env + domain randomisation, sharded per rank."""

    def __init__(self, args: argparse.Namespace) -> None:
        super().__init__(args)
        available_envs = {"joystick": Joystick, "standing": Standing}  # open_duck_mini_v2/runner.py:14-17
        if args.env not in available_envs:
            raise ValueError(f"Unknown env {args.env}")
        env_cls = available_envs[args.env]
        cfg = self.make_ppo_params()
        if dist.is_available() and dist.is_initialized():
            self.rank = dist.get_rank()
        world = int(os.environ.get("WORLD_SIZE", "1"))
        if cfg.num_envs % world:
            raise ValueError(f"num_envs {cfg.num_envs} must divide over {world} ranks")
        shard = shard_from_env(cfg.num_envs // world)  # brax splits num_envs over devices
        dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)) % max(1, torch.cuda.device_count()))
        self.env = env_cls(task=args.task, num_envs=shard.per_rank, device=dev, env_offset=shard.env_offset)
        self.env = wrap_for_brax_training(self.env, episode_length=cfg.episode_length,
                                          randomization_fn=domain_randomize, rng=cfg.seed)
        self.eval_env = None
        if self.rank == 0:
            self.eval_env = env_cls(task=args.task, num_envs=args.num_eval_envs, device=dev, env_offset=1 << 24)
            self.eval_env = wrap_for_brax_training(self.eval_env, episode_length=cfg.episode_length,
                                                   randomization_fn=domain_randomize, rng=cfg.seed + 1)
        self.action_size = self.env.action_size
        self.obs_size = int(self.env.observation_size["state"][0])
        self.restore_checkpoint_path = args.restore_checkpoint_path
        if self.rank == 0:
            print(f"Observation size: {self.obs_size}")


def main(argv=None) -> None:
    parser = argparse.ArgumentParser(description="Open Duck Mini Runner Script (MI355X)")
    parser.add_argument("--output_dir", type=str, default="checkpoints", help="Where to save the checkpoints")
    parser.add_argument("--num_timesteps", type=int, default=150000000)
    parser.add_argument("--env", type=str, default="joystick", help="env")
    parser.add_argument("--task", type=str, default="flat_terrain", help="Task to run")
    parser.add_argument("--restore_checkpoint_path", type=str, default=None,
                        help="Resume training from this checkpoint")
    parser.add_argument("--num_eval_envs", type=int, default=128, help="brax ppo.train default")
    parser.add_argument("--max_updates", type=int, default=None, help="stop after this many PPO updates")
    args = parser.parse_args(argv)
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1 and not dist.is_initialized():
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)))
        dist.init_process_group(os.environ.get("DUCK_DIST_BACKEND", "nccl"))
    runner = OpenDuckMiniV2Runner(args)
    runner.train(max_updates=args.max_updates)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
