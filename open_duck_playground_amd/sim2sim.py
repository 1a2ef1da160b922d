"""Single-robot 50 Hz control loop with an ONNX policy in the loop (mirror of
playground/open_duck_mini_v2/mujoco_infer.py:16-241 and mujoco_infer_base.py:7-285).

The reference steps CPU MuJoCo (``mujoco.mj_step``) at 500 Hz in a viewer loop and runs the ONNX
policy every ``decimation`` = 10 steps. Here the physics of one control period (10 substeps) is one
``duck_physics_step`` launch of the HIP kernels for a single env, the policy runs on the host
(``onnx_infer.OnnxInfer``), and the viewer / keyboard / wall-clock pacing are replaced by an explicit
``run(n_periods, command)`` (``realtime=True`` sleeps like the reference's loop).

Observation (mujoco_infer.py:67-103), 101 values: gyro, accelerometer with +1.3 added to x (this
script applies it; the training env's obs does not, joystick.py:502), command[7], actuator joint
angles - default, 0.05 * joint velocities, the last three actions, motor targets, foot contacts
(any penetrating contact between a foot and the floor, mujoco_infer_base.py:259-282), imitation
phase (cos, sin) advanced by ``phase_frequency_factor`` per period (:184-205).
"""

from __future__ import annotations

import time
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import constants
from .joystick import Joystick
from .onnx_infer import OnnxInfer

USE_MOTOR_SPEED_LIMITS = True  # mujoco_infer.py:14


class MjInfer:
    """MjInfer(model_path, reference_data, onnx_model_path, standing) on one MI355X env."""

    def __init__(self, model_path: str = "flat_terrain", reference_data: Optional[str] = None,
                 onnx_model_path: Optional[str] = None, standing: bool = False, device="cuda:0", policy=None):
        self.env = Joystick(model_path, num_envs=1, device=device, use_imitation=False)
        m = self.model = self.env.mj_model
        self.device = torch.device(device)
        self.sim_dt = 0.002   # mujoco_infer_base.py:15-18
        self.decimation = 10
        self.standing = standing
        self.head_control_mode = self.standing
        self.dof_vel_scale = 0.05
        self.action_scale = 0.25
        self.max_motor_velocity = 5.24
        self.phase_frequency_factor = 1.0
        self.num_dofs = m.nu
        self.policy = policy if policy is not None else OnnxInfer(onnx_model_path, awd=True)
        if not standing:
            table = np.load(reference_data or constants.POLY_COEFFICIENTS, allow_pickle=False)
            self.nb_steps_in_period = int(table["nb_steps_in_period"])
        self.actuator_qpos_addr = np.array([m.jnt_qposadr[j] for j in m.actuator_trnid])
        self.actuator_qvel_addr = np.array([m.jnt_dofadr[j] for j in m.actuator_trnid])
        names = m.names["sensor"]
        self.gyro_addr = int(m.sensor_adr[names.index("gyro")])
        self.accelerometer_addr = int(m.sensor_adr[names.index("accelerometer")])
        floor = m.id("geom", "floor")
        self._foot_slots = []
        for foot in constants.FEET_GEOMS:  # the pairs (floor, foot): 4 contact slots each
            g = m.id("geom", foot)
            p = [k for k in range(m.npair) if {int(m.pair_geom1[k]), int(m.pair_geom2[k])} == {floor, g}][0]
            self._foot_slots.append(slice(4 * p, 4 * p + 4))
        key = m.names["key"].index("home")
        self.default_actuator = m.key_ctrl[key].copy()
        self.motor_targets = self.default_actuator.copy()
        self.prev_motor_targets = self.default_actuator.copy()
        self.last_action = np.zeros(self.num_dofs)
        self.last_last_action = np.zeros(self.num_dofs)
        self.last_last_last_action = np.zeros(self.num_dofs)
        self.commands = [0.0] * 7
        self.imitation_i = 0.0
        self.imitation_phase = np.array([0.0, 0.0])
        self.saved_obs: List[np.ndarray] = []
        # MJInferBase.__init__: MjData at qpos0 with zero ctrl, one mj_step, then the home keyframe's
        # qpos and ctrl (the velocity of that first step is kept)
        t = lambda a: torch.tensor(np.asarray(a, dtype=np.float32)[:, None], device=self.device)  # noqa: E731
        self.qpos, self.qvel = t(m.qpos0), t(np.zeros(m.nv))
        self.warm, self.ctrl = t(np.zeros(m.nv)), t(np.zeros(m.nu))
        self.aux = torch.zeros(self.env.aux_size(), 1, dtype=torch.float32, device=self.device)
        self.env.physics_step(self.qpos, self.qvel, self.warm, self.ctrl, 1, self.aux)
        self.qpos.copy_(t(m.key_qpos[key]))
        self.ctrl.copy_(t(self.default_actuator))
        self._aux_np = None

    # --- one control period of physics (mj_step x decimation) ---------------------------------
    def _physics(self):
        self.env.physics_step(self.qpos, self.qvel, self.warm, self.ctrl, self.decimation, self.aux)
        torch.cuda.synchronize(self.device)
        self._aux_np = self.aux[:, 0].cpu().numpy().astype(np.float64)

    def _aux(self, name: str) -> np.ndarray:
        m = self.model
        sizes = [("qacc", m.nv), ("qacc_smooth", m.nv), ("qvel", m.nv), ("qfrc_smooth", m.nv),
                 ("actuator_force", m.nu), ("sensordata", m.nsensordata), ("con_dist", 4 * m.npair)]
        o = 0
        for k, n in sizes:
            if k == name:
                return self._aux_np[o:o + n]
            o += n
        raise KeyError(name)

    def get_gyro(self) -> np.ndarray:
        return self._aux("sensordata")[self.gyro_addr:self.gyro_addr + 3].copy()

    def get_accelerometer(self) -> np.ndarray:
        return self._aux("sensordata")[self.accelerometer_addr:self.accelerometer_addr + 3].copy()

    def get_feet_contacts(self):
        d = self._aux("con_dist")
        return tuple(bool((d[s] < 0).any()) for s in self._foot_slots)

    def get_obs(self, command: Sequence[float]) -> np.ndarray:
        """mujoco_infer.py:67-103 (state of the last mj_step of the period, sensors as mj_step left them)."""
        gyro = self.get_gyro()
        accelerometer = self.get_accelerometer()
        accelerometer[0] += 1.3
        qpos = self.qpos[:, 0].cpu().numpy().astype(np.float64)
        qvel = self.qvel[:, 0].cpu().numpy().astype(np.float64)
        joint_angles = qpos[self.actuator_qpos_addr]
        joint_vel = qvel[self.actuator_qvel_addr]
        contacts = np.array(self.get_feet_contacts(), dtype=np.float64)
        return np.concatenate([gyro, accelerometer, np.asarray(command, dtype=np.float64),
                               joint_angles - self.default_actuator, joint_vel * self.dof_vel_scale,
                               self.last_action, self.last_last_action, self.last_last_last_action,
                               self.motor_targets, contacts, self.imitation_phase])

    def control_step(self):
        """One policy period of mujoco_infer.py:175-241: decimation substeps, then obs -> action -> ctrl."""
        self._physics()
        if not self.standing:
            self.imitation_i += 1.0 * self.phase_frequency_factor
            self.imitation_i = self.imitation_i % self.nb_steps_in_period
            ph = self.imitation_i / self.nb_steps_in_period * 2 * np.pi
            self.imitation_phase = np.array([np.cos(ph), np.sin(ph)])
        obs = self.get_obs(self.commands)
        self.saved_obs.append(obs)
        action = np.asarray(self.policy.infer(obs), dtype=np.float64)
        self.last_last_last_action = self.last_last_action.copy()
        self.last_last_action = self.last_action.copy()
        self.last_action = action.copy()
        self.motor_targets = self.default_actuator + action * self.action_scale
        if USE_MOTOR_SPEED_LIMITS:
            lim = self.max_motor_velocity * (self.sim_dt * self.decimation)
            self.motor_targets = np.clip(self.motor_targets, self.prev_motor_targets - lim,
                                         self.prev_motor_targets + lim)
            self.prev_motor_targets = self.motor_targets.copy()
        self.ctrl.copy_(torch.tensor(self.motor_targets.astype(np.float32)[:, None], device=self.device))
        return obs, action

    def run(self, n_periods: int, command: Optional[Sequence[float]] = None, realtime: bool = False):
        if command is not None:
            self.commands = list(command)
        period = self.sim_dt * self.decimation
        for _ in range(n_periods):
            t0 = time.time()
            self.control_step()
            if realtime:
                time.sleep(max(0.0, period - (time.time() - t0)))
        return self.saved_obs
