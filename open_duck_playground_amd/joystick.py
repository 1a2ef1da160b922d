"""Joystick task for Open Duck Mini V2 on MI355X (mirror of playground/open_duck_mini_v2/joystick.py).

Same surface as the reference ``Joystick`` (``joystick.py:105-725``) and its base class
(``base.py:41-291``): ``Joystick(task, config, config_overrides)``, ``reset(rng) -> State``,
``step(state, action) -> State``, ``action_size``, ``observation_size``, ``dt``,
``n_substeps``, ``mj_model``-style accessors and the base-class index maps. Differences
that follow from running a batch of envs in one launch on the GPU:

* the env is batched: ``num_envs`` envs live in one struct-of-arrays state buffer; every
  tensor in ``State`` has a leading env axis (what brax's ``VmapWrapper`` produces),
* ``rng`` is an integer seed; env ``i`` draws from a counter-based threefry stream keyed
  by ``(seed, env_offset + i)`` (shard-invariant), not a JAX key,
* ``step(state, action)`` returns a new ``State`` in new buffers and leaves ``state`` as it was
  (the reference's ``state.replace(...)``, joystick.py:480-481); ``step(state, action,
  inplace=True)`` advances ``state``'s own buffers instead (what a rollout loop that drops the
  previous state wants: brax's jitted unroll donates them the same way),
* physics, obs, rewards and termination all run inside ``libduck.so``
  (``csrc/duck_env_kernels.h`` via ``duck_step``); this module only allocates torch buffers and
  launches.

``wrap_for_brax_training`` / ``domain_randomize`` provide the training-side behaviour the
reference gets from ``mujoco_playground.wrapper`` and ``common/randomize.py``.
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Any, Dict, Optional, Union

import numpy as np
import torch

from . import config as cfgmod
from . import constants
from .cabi import METRIC_NAMES, TASK_JOYSTICK, ModelDescHolder, dr_layout, layout, refmotion_struct
from .config import ConfigDict, default_config  # noqa: F401  (re-exported like the reference module)
from .mjcf import JNT_FREE, Model
from .native import DuckError, check, lib, model_library
from .refmotion import PolyReferenceMotion

USE_IMITATION_REWARD = cfgmod.USE_IMITATION_REWARD
USE_MOTOR_SPEED_LIMITS = cfgmod.USE_MOTOR_SPEED_LIMITS
# duck_set_step_mode (include/duck.h DUCK_STEP_*)
STEP_MODES = {"auto": 0, "throughput": 1, "latency": 2, "paired": 3, "latency_x2": 4}


@dataclass
class Data:
    """The subset of mjx.Data the env exposes: views into the SoA state buffer."""
    qpos: torch.Tensor
    qvel: torch.Tensor
    qacc_warmstart: torch.Tensor
    ctrl: torch.Tensor


@dataclass
class State:
    """mujoco_playground ``State(data, obs, reward, done, metrics, info)`` for a batch."""
    data: Data
    obs: Dict[str, torch.Tensor]
    reward: torch.Tensor
    done: torch.Tensor
    metrics: Dict[str, torch.Tensor]
    info: Dict[str, Any]
    fstate: torch.Tensor = field(repr=False, default=None)
    istate: torch.Tensor = field(repr=False, default=None)

    def replace(self, **kw) -> "State":
        """A new State with the given fields replaced (flax struct.dataclass semantics); the
        tensors themselves are shared, not copied."""
        import dataclasses
        return dataclasses.replace(self, **kw)


class OpenDuckMiniV2Env:
    """Base class (base.py:41-291): model, address maps, accessors."""

    def __init__(self, xml_path: str, config: ConfigDict, config_overrides: Optional[Dict[str, Any]] = None) -> None:
        self._config = cfgmod.apply_overrides(config, config_overrides)
        if xml_path.endswith(".xml"):  # an MJCF scene: compiled here (base.py:53-56 sets the timestep)
            from .mjcf import compile_mjcf
            self._mj_model = compile_mjcf(xml_path, timestep=self._config.sim_dt)
        else:
            self._mj_model = Model.load(xml_path)
        self._xml_path = xml_path
        maps = cfgmod.AddressMaps(self._mj_model)
        self.floating_base_name = maps.floating_base_name
        self.actuator_names = maps.actuator_names
        self.joint_names = maps.joint_names
        self.backlash_joint_names = maps.backlash_joint_names
        self.actuator_joint_ids = maps.actuator_joint_ids
        self.actuator_joint_qpos_addr = maps.actuator_joint_qpos_addr
        self.actuator_qvel_addr = maps.actuator_qvel_addr
        self.backlash_joint_ids = maps.backlash_joint_ids
        self.backlash_joint_qpos_addr = maps.backlash_joint_qpos_addr
        self._floating_base_qpos_addr = maps.floating_base_qpos_addr
        self._floating_base_qvel_addr = maps.floating_base_qvel_addr
        self.backlash_idx_to_add = maps.backlash_idx_to_add

    # --- accessors on batched tensors [N, nq] / [N, nv] (base.py:154-231) ---
    def get_actuator_joints_qpos(self, qpos: torch.Tensor) -> torch.Tensor:
        return qpos[..., self.actuator_joint_qpos_addr]

    def get_actuator_joints_qvel(self, qvel: torch.Tensor) -> torch.Tensor:
        return qvel[..., self.actuator_qvel_addr]

    def get_actuator_backlash_qpos(self, qpos: torch.Tensor) -> torch.Tensor:
        if not self.backlash_joint_qpos_addr:
            return qpos[..., :0]
        return qpos[..., self.backlash_joint_qpos_addr]

    def get_floating_base_qpos(self, qpos: torch.Tensor) -> torch.Tensor:
        a = self._floating_base_qpos_addr
        return qpos[..., a:a + 7]

    def get_floating_base_qvel(self, qvel: torch.Tensor) -> torch.Tensor:
        a = self._floating_base_qvel_addr
        return qvel[..., a:a + 6]

    def get_joint_id_from_name(self, name: str) -> int:
        return self._mj_model.names["jnt"].index(name) if name in self._mj_model.names["jnt"] else -1

    def get_actuator_id_from_name(self, name: str) -> int:
        return self._mj_model.names["actuator"].index(name)

    def get_joint_addr_from_name(self, name: str) -> int:
        return int(self._mj_model.jnt_qposadr[self.get_joint_id_from_name(name)])

    @property
    def xml_path(self) -> str:
        return self._xml_path

    @property
    def action_size(self) -> int:
        return int(self._mj_model.nu)

    @property
    def mj_model(self) -> Model:
        return self._mj_model

    @property
    def dt(self) -> float:
        return self._config.ctrl_dt

    @property
    def sim_dt(self) -> float:
        return self._config.sim_dt

    @property
    def n_substeps(self) -> int:
        return int(round(self._config.ctrl_dt / self._config.sim_dt))


class Joystick(OpenDuckMiniV2Env):
    """Track a joystick command (joystick.py:105-725), batched on one MI355X."""

    TASK = TASK_JOYSTICK
    METRICS = METRIC_NAMES

    def __init__(self, task: str = "flat_terrain", config: ConfigDict = None,
                 config_overrides: Optional[Dict[str, Union[str, int, list]]] = None, num_envs: int = 1,
                 device: Union[str, torch.device] = "cuda:0", use_imitation: Optional[bool] = None,
                 env_offset: int = 0) -> None:
        super().__init__(xml_path=constants.task_to_xml(task), config=config or default_config(),
                         config_overrides=config_overrides)
        self.task = task
        self.num_envs = int(num_envs)
        self.env_offset = int(env_offset)
        self.device = torch.device(device)
        self.use_imitation = USE_IMITATION_REWARD if use_imitation is None else bool(use_imitation)
        self.auto_reset = False
        self.episode_length = int(self._config.episode_length)
        self.dr: Optional[torch.Tensor] = None
        self._step_mode = "auto"
        self._post_init()

    def _post_init(self) -> None:
        m = self._mj_model
        key = m.names["key"].index("home")
        self._init_q = m.key_qpos[key].copy()
        self._default_actuator = m.key_ctrl[key].copy()
        if self.use_imitation:
            self.PRM = PolyReferenceMotion(constants.POLY_COEFFICIENTS)
        jr = m.jnt_range[1:]
        self._lowers, self._uppers = jr[:, 0], jr[:, 1]
        c = (self._lowers + self._uppers) / 2
        r = self._uppers - self._lowers
        self._soft_lowers = c - 0.5 * r * self._config.soft_joint_pos_limit_factor
        self._soft_uppers = c + 0.5 * r * self._config.soft_joint_pos_limit_factor
        self._njoints = m.njnt
        self._actuators = m.nu
        self._torso_body_id = m.id("body", constants.ROOT_BODY)
        self._torso_mass = float(m.body_subtreemass[self._torso_body_id])
        self._site_id = m.id("site", "imu")
        self._feet_site_id = np.array([m.id("site", s) for s in constants.FEET_SITES])
        self._floor_geom_id = m.id("geom", "floor")
        self._feet_geom_id = np.array([m.id("geom", g) for g in constants.FEET_GEOMS])
        self._qpos_noise_scale = cfgmod.qpos_noise_scale(self._config, m.nu)
        self._layout = layout(m.nq, m.nv, m.nu, self.use_imitation, self.TASK)
        self._create_sim()

    def _create_sim(self) -> None:
        m = self._mj_model
        self._desc = ModelDescHolder(m)
        self._cfg_struct = cfgmod.env_config_struct(m, self._config, self.use_imitation, self.auto_reset,
                                                    self.dr is not None, task=self.TASK)
        table = dict(np.load(constants.POLY_COEFFICIENTS, allow_pickle=False))
        self._ref_struct, self._ref_coeffs = refmotion_struct(table)
        handle = C.c_void_p()
        dev = self.device.index if self.device.index is not None else 0
        self._lib = lib(model_library(m))
        check(self._lib.duck_create(C.byref(self._desc.desc), C.byref(self._cfg_struct), C.byref(self._ref_struct),
                                    dev, C.byref(handle)), self._lib)
        self._sim = handle
        self._scratch = None
        if hasattr(self._lib, "duck_set_step_mode"):  # (A/B baselines built before the latency kernel)
            check(self._lib.duck_set_step_mode(self._sim, STEP_MODES[self._step_mode]), self._lib)

    def set_step_mode(self, mode: str) -> None:
        """duck_set_step_mode: "auto" (default), "throughput", "latency", "paired" or "latency_x2". The same stage code
        in a different work split: "throughput" runs 16 envs per workgroup on one team each; "latency"
        splits each substep's stages over four waves per 4 envs (a shorter env-step for small batches,
        e.g. a 4096-env job strong-scaled over 4 or 8 GPUs); "paired" splits them over a pair of waves
        per 4 envs, 8 envs per workgroup (4096 envs over 2 GPUs); "auto" takes latency at <= 4 envs
        per CU and paired at <= 8 -- "latency_x2" instead in the plane-floor scenes without backlash: the latency
        kernel at two workgroups per CU. Every mode gives bit-identical results (include/duck.h)."""
        if mode not in STEP_MODES:
            raise DuckError(f"step mode {mode!r} not in {sorted(STEP_MODES)}")
        if not hasattr(self._lib, "duck_set_step_mode") and mode in ("auto", "throughput"):
            return  # an A/B baseline library without the latency kernel
        self._step_mode = mode
        check(self._lib.duck_set_step_mode(self._sim, STEP_MODES[mode]), self._lib)

    @property
    def step_kernel(self) -> str:
        """The kernel step() launches for this batch: "throughput", "latency", "paired" or "latency_x2"."""
        if not hasattr(self._lib, "duck_step_kernel_for"):
            return "throughput"
        k = self._lib.duck_step_kernel_for(self._sim, self.num_envs)
        check(min(k, 0), self._lib)
        return {1: "throughput", 2: "latency", 3: "paired", 4: "latency_x2"}[k]

    def device_error(self, clear: bool = False) -> int:
        """The handle's sticky device error word (duck_device_error; DUCK_DEVERR_* bits, 0 = none). While
        it is set, reset/step/physics_step raise DuckError (DUCK_EDEVICE): a latency-kernel launch whose
        cross-wave wait gave up has written invalid state (NaN qpos) for its workgroup's envs."""
        out = C.c_uint(0)
        check(self._lib.duck_device_error(self._sim, C.byref(out), int(clear)), self._lib)
        return int(out.value)

    def lat_timeouts(self, reset: bool = False) -> int:
        """Latency-mode event waits that gave up since the last reset (a broken schedule; must be 0)."""
        out = C.c_uint(0)
        check(self._lib.duck_debug_lat_timeouts(self._sim, C.byref(out), int(reset)), self._lib)
        return int(out.value)

    def __del__(self):
        try:
            if getattr(self, "_sim", None):
                self._lib.duck_destroy(self._sim)
        except Exception:
            pass

    def _reconfigure(self) -> None:
        if getattr(self, "_sim", None):
            self._lib.duck_destroy(self._sim)
            self._sim = None
        self._create_sim()

    # ------------------------------------------------------------------
    @property
    def observation_size(self) -> Dict[str, tuple]:
        return {"state": (self._layout.obs_size,), "privileged_state": (self._layout.priv_size,)}

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _views(self, fstate: torch.Tensor, istate: torch.Tensor, obs, priv, reward, done) -> State:
        L = self._layout
        n = self.num_envs
        F = fstate.view(L.nfloat, n)

        def fv(name, k):
            return F[L.off[name]:L.off[name] + k].t()

        I = istate.view(L.nint, n)

        def iv(name, k=1):
            v = I[L.ioff[name]:L.ioff[name] + k].t()
            return v[:, 0] if k == 1 else v

        data = Data(qpos=fv("qpos", L.nq), qvel=fv("qvel", L.nv), qacc_warmstart=fv("qacc_warmstart", L.nv),
                    ctrl=fv("ctrl", L.nu))
        info = {"rng": iv("rng_key", 2), "rng_counter": iv("rng_ctr"), "step": iv("step"),
                "command": fv("command", 7), "last_act": fv("last_act", L.nu),
                "last_last_act": fv("last_last_act", L.nu), "last_last_last_act": fv("last_last_last_act", L.nu),
                "motor_targets": fv("motor_targets", L.nu), "feet_air_time": fv("feet_air_time", 2),
                "last_contact": fv("last_contact", 2), "swing_peak": fv("swing_peak", 2), "push": fv("push", 2),
                "push_step": iv("push_step"), "push_interval_steps": iv("push_interval"),
                "action_history": fv("action_history", 3 * L.nu), "imu_history": fv("imu_history", 9),
                "imitation_i": iv("imitation_i"),
                "current_reference_motion": fv("ref_motion", 40 if self.use_imitation else 0),
                "imitation_phase": fv("imitation_phase", 2)}
        if self.auto_reset:
            info["steps"] = iv("ep_steps")
            info["truncation"] = F[L.off["truncation"]]
        metrics = {name: F[L.off["metrics"] + k] for k, name in enumerate(self.METRICS) if name}
        return State(data=data, obs={"state": obs, "privileged_state": priv}, reward=reward, done=done,
                     metrics=metrics, info=info, fstate=fstate, istate=istate)

    def reset(self, rng: int = 0, mask: Optional[torch.Tensor] = None, state: Optional[State] = None) -> State:
        """Joystick.reset (joystick.py:206-321) for every env (or the envs where mask != 0)."""
        L, n, dev = self._layout, self.num_envs, self.device
        if state is None:
            fstate = torch.zeros(L.nfloat * n, dtype=torch.float32, device=dev)
            istate = torch.zeros(L.nint * n, dtype=torch.int32, device=dev)
            obs = torch.zeros(n, L.obs_size, dtype=torch.float32, device=dev)
            priv = torch.zeros(n, L.priv_size, dtype=torch.float32, device=dev)
            reward = torch.zeros(n, dtype=torch.float32, device=dev)
            done = torch.zeros(n, dtype=torch.float32, device=dev)
            state = self._views(fstate, istate, obs, priv, reward, done)
        mask_ptr = None
        if mask is not None:
            mask = mask.to(device=dev, dtype=torch.uint8).contiguous()
            mask_ptr = mask.data_ptr()
        check(self._lib.duck_reset(self._sim, n, state.fstate.data_ptr(), state.istate.data_ptr(), mask_ptr,
                               int(rng) & 0xFFFFFFFFFFFFFFFF, self.env_offset,
                               self.dr.data_ptr() if self.dr is not None else None,
                               state.obs["state"].data_ptr(), state.obs["privileged_state"].data_ptr(), self._stream()),
              self._lib)
        if mask is None:
            state.reward.zero_()
            state.done.zero_()
        return state

    def step(self, state: State, action: torch.Tensor, inplace: bool = False) -> State:
        """Joystick.step (joystick.py:323-481) for all envs: the next State, in new buffers (``state``
        is left as it was), or with ``inplace=True`` in ``state``'s own buffers (returned)."""
        n = self.num_envs
        if action.numel() != n * self.action_size:
            raise DuckError(f"action must hold {n} x {self.action_size} values, got {tuple(action.shape)}")
        action = action.to(device=self.device, dtype=torch.float32).reshape(n, self.action_size).contiguous()
        if not inplace:
            # the step reads and writes every state row (obs, reward and done are outputs only)
            state = self._views(state.fstate.clone(), state.istate.clone(), torch.empty_like(state.obs["state"]),
                                torch.empty_like(state.obs["privileged_state"]), torch.empty_like(state.reward),
                                torch.empty_like(state.done))
        check(self._lib.duck_step(self._sim, n, state.fstate.data_ptr(), state.istate.data_ptr(),
                              self.dr.data_ptr() if self.dr is not None else None, action.data_ptr(),
                              state.obs["state"].data_ptr(), state.obs["privileged_state"].data_ptr(),
                              state.reward.data_ptr(), state.done.data_ptr(), self._scratch_ptr(), self._stream()),
              self._lib)
        return state

    def _scratch_ptr(self):
        if self._scratch is None:
            nv = self._mj_model.nv
            self._scratch = torch.zeros(self.num_envs * nv * nv, dtype=torch.float32, device=self.device)
        return self._scratch.data_ptr()

    # physics-level entry: mjx_env.step(model, data, ctrl, n_substeps) (joystick.py:420)
    def physics_step(self, qpos: torch.Tensor, qvel: torch.Tensor, qacc_warmstart: torch.Tensor, ctrl: torch.Tensor,
                     n_substeps: int, aux: Optional[torch.Tensor] = None) -> None:
        """In-place physics on SoA tensors [nq, N], [nv, N], [nv, N], [nu, N]."""
        n = qpos.shape[1]
        for t in (qpos, qvel, qacc_warmstart, ctrl):
            if not t.is_contiguous() or t.dtype != torch.float32 or t.device != self.device or t.shape[1] != n:
                raise DuckError("physics_step expects contiguous float32 SoA tensors on the env device")
        scratch = torch.zeros(n * self._mj_model.nv ** 2, dtype=torch.float32, device=self.device)
        check(self._lib.duck_physics_step(self._sim, n, qpos.data_ptr(), qvel.data_ptr(), qacc_warmstart.data_ptr(),
                                      ctrl.data_ptr(), self.dr.data_ptr() if self.dr is not None else None,
                                      int(n_substeps), aux.data_ptr() if aux is not None else None,
                                      scratch.data_ptr(), self._stream()), self._lib)

    def aux_size(self) -> int:
        return int(self._lib.duck_aux_size(self._sim))


def domain_randomize(env: Joystick, rng: int) -> torch.Tensor:
    """randomize.domain_randomize (common/randomize.py:26-146): per-env model values.

    Returns the per-env record (SoA ``[duck_dr_layout.nfloat, num_envs]``) and installs it
    on the env: the same 8 model fields as the reference's ``in_axes`` become per-env.
    """
    m = env.mj_model
    D = dr_layout(m.nbody, m.nu)
    dr = torch.zeros(D["nfloat"] * env.num_envs, dtype=torch.float32, device=env.device)
    check(env._lib.duck_randomize(env._sim, env.num_envs, dr.data_ptr(), int(rng), env.env_offset, env._stream()),
          env._lib)
    env.dr = dr
    env._reconfigure()
    return dr


def wrap_for_brax_training(env: Joystick, episode_length: int = 1000, action_repeat: int = 1,
                           randomization_fn=None, rng: int = 0) -> Joystick:
    """mujoco_playground.wrapper.wrap_for_brax_training: EpisodeWrapper + AutoReset (+ DR).

    AutoReset semantics follow BraxAutoResetWrapper: on done, ``data`` and ``obs`` are
    replaced by the env's first reset state while ``info`` carries on.
    """
    if action_repeat != 1:
        raise DuckError("action_repeat != 1 is not supported (the reference uses 1)")
    env.auto_reset = True
    env.episode_length = int(episode_length)
    env._config.episode_length = int(episode_length)
    if randomization_fn is not None:
        randomization_fn(env, rng)
    env._reconfigure()
    return env
