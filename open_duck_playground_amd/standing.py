"""Standing task for Open Duck Mini v2 (playground/open_duck_mini_v2/standing.py), on MI355X.

Same model, physics, action delay, pushes, noise and info bookkeeping as ``Joystick``; the
kernel's task switch (``duck_env_config.task``) selects what differs in the reference:

* ``default_config`` (standing.py:44-100): smaller gyro/accelerometer noise, reward scales
  orientation / torques / action_rate / stand_still / alive / head_pos, head yaw +-2.7
* reset (:200-321): base velocity U(+-0.5), ``motor_targets`` starts at zero
* step (:323-460): no imitation phase, no motor speed limit, command resampled after 500
  steps with a zero walking part (:608-661)
* obs (:462-575): state[85] = gyro, accel, command, q - q0, 0.05 qd, 3 last actions, contact;
  privileged[153] = state + the same privileged block as Joystick without imitation fields
* rewards (:577-606): orientation = |upvector_xy|^2, stand_still over the legs only
  (``ignore_head=True``), head_pos gated on a walking command (always 0 here, as in the reference)
"""

from __future__ import annotations

from typing import Any, Dict, Optional, Union

import torch

from .cabi import STANDING_METRIC_NAMES, TASK_STANDING
from .config import ConfigDict, standing_default_config
from .joystick import Joystick

USE_IMITATION_REWARD = False  # standing.py:42


def default_config() -> ConfigDict:
    return standing_default_config()


class Standing(Joystick):
    """Standing policy (standing.py:103), batched on one MI355X."""

    TASK = TASK_STANDING
    METRICS = STANDING_METRIC_NAMES

    def __init__(self, task: str = "flat_terrain", config: ConfigDict = None,
                 config_overrides: Optional[Dict[str, Union[str, int, list]]] = None, num_envs: int = 1,
                 device: Union[str, torch.device] = "cuda:0", env_offset: int = 0) -> None:
        super().__init__(task=task, config=config or default_config(), config_overrides=config_overrides,
                         num_envs=num_envs, device=device, use_imitation=False, env_offset=env_offset)
