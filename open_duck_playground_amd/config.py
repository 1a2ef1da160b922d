"""Env configuration: ``default_config()`` and the host-side bookkeeping of the reference.

* ``ConfigDict`` is a minimal stand-in for ``ml_collections.config_dict`` (not installed):
  attribute access, nesting, ``update`` with dotted keys for ``config_overrides``.
* ``default_config`` has the keys and defaults of ``joystick.py:49-102``.
* ``env_config_struct`` fills the C struct the kernels read, deriving the same index maps
  as ``OpenDuckMiniV2Env.__init__`` (``base.py:63-132``) and ``Joystick._post_init``
  (``joystick.py:121-200``).
"""

from __future__ import annotations

import copy
from typing import Any, Dict, Optional

import numpy as np

from . import constants
from .cabi import DuckEnvConfig
from .mjcf import JNT_FREE, Model

# module flags of joystick.py:45-46
USE_IMITATION_REWARD = True
USE_MOTOR_SPEED_LIMITS = True


class ConfigDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def __deepcopy__(self, memo):
        return ConfigDict({k: copy.deepcopy(v, memo) for k, v in self.items()})

    def update_from_flattened(self, overrides: Dict[str, Any]):
        for key, v in overrides.items():
            node = self
            parts = key.split(".")
            for p in parts[:-1]:
                node = node[p]
            if parts[-1] not in node:
                raise KeyError(f"unknown config key {key}")
            node[parts[-1]] = v
        return self


def create(**kw) -> ConfigDict:
    return ConfigDict(kw)


def default_config() -> ConfigDict:
    """Same keys/defaults as joystick.default_config (joystick.py:49-102)."""
    return create(
        ctrl_dt=0.02,
        sim_dt=0.002,
        episode_length=1000,
        action_repeat=1,
        action_scale=0.25,
        dof_vel_scale=0.05,
        history_len=0,
        soft_joint_pos_limit_factor=0.95,
        max_motor_velocity=5.24,
        noise_config=create(
            level=1.0,
            action_min_delay=0,
            action_max_delay=3,
            imu_min_delay=0,
            imu_max_delay=3,
            scales=create(hip_pos=0.03, knee_pos=0.05, ankle_pos=0.08, joint_vel=2.5, gravity=0.1, linvel=0.1,
                          gyro=0.1, accelerometer=0.05),
        ),
        reward_config=create(
            scales=create(tracking_lin_vel=2.5, tracking_ang_vel=6.0, torques=-1.0e-3, action_rate=-0.5,
                          stand_still=-0.2, alive=20.0, imitation=1.0),
            tracking_sigma=0.01,
        ),
        push_config=create(enable=True, interval_range=[5.0, 10.0], magnitude_range=[0.1, 1.0]),
        lin_vel_x=[-0.15, 0.15],
        lin_vel_y=[-0.2, 0.2],
        ang_vel_yaw=[-1.0, 1.0],
        neck_pitch_range=[-0.34, 1.1],
        head_pitch_range=[-0.78, 0.78],
        head_yaw_range=[-1.5, 1.5],
        head_roll_range=[-0.5, 0.5],
        head_range_factor=1.0,
    )


def standing_default_config() -> ConfigDict:
    """Same keys/defaults as standing.default_config (standing.py:44-100)."""
    return create(
        ctrl_dt=0.02,
        sim_dt=0.002,
        episode_length=1000,
        action_repeat=1,
        action_scale=0.25,
        dof_vel_scale=0.05,
        history_len=0,
        soft_joint_pos_limit_factor=0.95,
        noise_config=create(
            level=1.0,
            action_min_delay=0,
            action_max_delay=3,
            imu_min_delay=0,
            imu_max_delay=3,
            scales=create(hip_pos=0.03, knee_pos=0.05, ankle_pos=0.08, joint_vel=2.5, gravity=0.1, linvel=0.1,
                          gyro=0.05, accelerometer=0.005),
        ),
        reward_config=create(
            scales=create(orientation=-0.5, torques=-1.0e-3, action_rate=-0.375, stand_still=-0.3, alive=20.0,
                          head_pos=-2.0),
            tracking_sigma=0.01,
        ),
        push_config=create(enable=True, interval_range=[5.0, 10.0], magnitude_range=[0.1, 1.0]),
        neck_pitch_range=[-0.34, 1.1],
        head_pitch_range=[-0.78, 0.78],
        head_yaw_range=[-2.7, 2.7],
        head_roll_range=[-0.5, 0.5],
        head_range_factor=1.0,
    )


def qpos_noise_scale(config: ConfigDict, nu: int) -> np.ndarray:
    """Bug-compatible joint-noise scales (joystick.py:184-200): indices come from the
    10-joint JOINTS_ORDER_NO_HEAD list but index the nu-long actuator vector."""
    s = np.zeros(nu)
    names = constants.JOINTS_ORDER_NO_HEAD
    hip = [i for i, j in enumerate(names) if "_hip" in j]
    knee = [i for i, j in enumerate(names) if "_knee" in j]
    ankle = [i for i, j in enumerate(names) if "_ankle" in j]
    s[hip] = config.noise_config.scales.hip_pos
    s[knee] = config.noise_config.scales.knee_pos
    s[ankle] = config.noise_config.scales.ankle_pos
    return s


class AddressMaps:
    """Index maps of OpenDuckMiniV2Env.__init__ (base.py:63-132)."""

    def __init__(self, m: Model):
        jn = m.names["jnt"]
        self.actuator_names = list(m.names["actuator"])
        self.joint_names = list(jn)
        free = [k for k in range(m.njnt) if m.jnt_type[k] == JNT_FREE]
        self.floating_base_name = jn[free[0]]
        self.backlash_joint_names = [j for j in jn if j not in self.actuator_names and j != self.floating_base_name]
        self.actuator_joint_ids = [jn.index(n) for n in self.actuator_names]
        self.actuator_joint_qpos_addr = [int(m.jnt_qposadr[j]) for j in self.actuator_joint_ids]
        self.actuator_qvel_addr = [int(m.jnt_dofadr[j]) for j in self.actuator_joint_ids]
        self.backlash_joint_ids = [jn.index(n) for n in self.backlash_joint_names]
        self.backlash_joint_qpos_addr = [int(m.jnt_qposadr[j]) for j in self.backlash_joint_ids]
        self.floating_base_qpos_addr = int(m.jnt_qposadr[free[0]])
        self.floating_base_qvel_addr = int(m.jnt_dofadr[free[0]])
        self.backlash_idx_to_add = [i for i, a in enumerate(self.actuator_names)
                                    if a + "_backlash" not in self.backlash_joint_names]
        # per-actuator backlash qpos address (-1 where joystick.py:538-541 inserts a 0)
        self.backlash_qposadr = []
        for a in self.actuator_names:
            nm = a + "_backlash"
            self.backlash_qposadr.append(int(m.jnt_qposadr[jn.index(nm)]) if nm in jn else -1)


def env_config_struct(m: Model, config: ConfigDict, use_imitation: bool, auto_reset: bool = False,
                      domain_randomize: bool = False, task: int = 0) -> DuckEnvConfig:
    """task 0 = Joystick (joystick.py), 1 = Standing (standing.py: no imitation, no motor speed
    limits, zero walking command, orientation + head_pos terms)."""
    c = DuckEnvConfig()
    standing = task == 1
    c.task = int(task)
    maps = AddressMaps(m)
    nu = m.nu
    c.ctrl_dt = config.ctrl_dt
    c.sim_dt = config.sim_dt
    c.n_substeps = int(round(config.ctrl_dt / config.sim_dt))
    c.episode_length = int(config.episode_length)
    c.auto_reset = int(auto_reset)
    c.action_scale = config.action_scale
    c.dof_vel_scale = config.dof_vel_scale
    c.max_motor_velocity = config.get("max_motor_velocity", 0.0)
    c.use_imitation = int(use_imitation and not standing)
    c.use_motor_speed_limits = int(USE_MOTOR_SPEED_LIMITS and not standing)
    nc = config.noise_config
    c.noise_level = nc.level
    c.action_min_delay, c.action_max_delay = int(nc.action_min_delay), int(nc.action_max_delay)
    c.imu_min_delay, c.imu_max_delay = int(nc.imu_min_delay), int(nc.imu_max_delay)
    c.noise_gyro = nc.scales.gyro
    c.noise_accelerometer = nc.scales.accelerometer
    c.noise_gravity = nc.scales.gravity
    c.noise_joint_vel = nc.scales.joint_vel
    c.qpos_noise_scale[:nu] = [float(x) for x in qpos_noise_scale(config, nu)]
    sc = config.reward_config.scales
    for k in ("tracking_lin_vel", "tracking_ang_vel", "torques", "action_rate", "alive", "imitation",
              "stand_still", "orientation", "head_pos"):
        setattr(c, "scale_" + k, float(sc.get(k, 0.0)))
    c.tracking_sigma = config.reward_config.tracking_sigma
    c.push_enable = int(bool(config.push_config.enable))
    c.push_interval_range[:] = list(config.push_config.interval_range)
    c.push_magnitude_range[:] = list(config.push_config.magnitude_range)
    for k in ("lin_vel_x", "lin_vel_y", "ang_vel_yaw", "neck_pitch_range", "head_pitch_range", "head_yaw_range",
              "head_roll_range"):
        # Standing samples no walking command (standing.py:614-655): U(0, 0) draws 0.0 exactly
        getattr(c, k)[:] = list(config.get(k, [0.0, 0.0]))
    c.head_range_factor = config.head_range_factor
    key = m.names["key"].index("home")
    c.default_actuator[:nu] = [float(x) for x in m.key_ctrl[key]]
    c.init_qpos[:m.nq] = [float(x) for x in m.key_qpos[key]]
    c.actuator_qposadr[:nu] = maps.actuator_joint_qpos_addr
    c.actuator_qveladr[:nu] = maps.actuator_qvel_addr
    c.backlash_qposadr[:nu] = maps.backlash_qposadr
    c.imu_site = m.id("site", "imu")
    c.left_foot_site = m.id("site", constants.FEET_SITES[0])
    c.right_foot_site = m.id("site", constants.FEET_SITES[1])
    c.floor_geom = m.id("geom", "floor")
    c.left_foot_geom = m.id("geom", constants.FEET_GEOMS[0])
    c.right_foot_geom = m.id("geom", constants.FEET_GEOMS[1])
    adr = lambda name: int(m.sensor_adr[m.id("sensor", name)])
    c.sens_gyro = adr(constants.GYRO_SENSOR)
    c.sens_accelerometer = adr(constants.ACCELEROMETER_SENSOR)
    c.sens_upvector = adr(constants.GRAVITY_SENSOR)
    c.sens_local_linvel = adr(constants.LOCAL_LINVEL_SENSOR)
    c.sens_global_angvel = adr(constants.GLOBAL_ANGVEL_SENSOR)
    c.sens_left_foot_linvel = adr("left_foot_global_linvel")
    c.sens_right_foot_linvel = adr("right_foot_global_linvel")
    c.domain_randomize = int(domain_randomize)
    return c


def apply_overrides(config: Optional[ConfigDict], overrides: Optional[Dict[str, Any]]) -> ConfigDict:
    cfg = copy.deepcopy(config if config is not None else default_config())
    if overrides:
        cfg.update_from_flattened(overrides)
    return cfg
