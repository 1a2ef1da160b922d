"""ctypes mirrors of the C-ABI structs in ``include/duck_model.h`` and ``include/duck_env.h``.

Shared by the product binding (``native.py`` -> ``libduck.so``) and by the test-only
oracle binding (``tests/oracle_ffi.py`` -> ``oracle/liboracle.so``). Nothing here computes
physics; it only lays out host memory for the C side.
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, List

import numpy as np

from .mjcf import Model

_I = C.POINTER(C.c_int)
_D = C.POINTER(C.c_double)


class DuckModelDesc(C.Structure):
    _fields_ = [
        ("nq", C.c_int), ("nv", C.c_int), ("nu", C.c_int), ("nbody", C.c_int), ("njnt", C.c_int),
        ("ngeom", C.c_int), ("nsite", C.c_int), ("nsensor", C.c_int), ("nsensordata", C.c_int), ("npair", C.c_int),
        ("timestep", C.c_double), ("gravity", C.c_double * 3), ("impratio", C.c_double), ("tolerance", C.c_double),
        ("ls_tolerance", C.c_double), ("meaninertia", C.c_double),
        ("iterations", C.c_int), ("ls_iterations", C.c_int), ("eulerdamp", C.c_int),
        ("body_parentid", _I), ("body_rootid", _I), ("body_weldid", _I), ("body_jntnum", _I), ("body_jntadr", _I),
        ("body_dofnum", _I), ("body_dofadr", _I),
        ("body_pos", _D), ("body_quat", _D), ("body_ipos", _D), ("body_iquat", _D), ("body_mass", _D),
        ("body_inertia", _D), ("body_invweight0", _D),
        ("jnt_type", _I), ("jnt_qposadr", _I), ("jnt_dofadr", _I), ("jnt_bodyid", _I), ("jnt_limited", _I),
        ("jnt_pos", _D), ("jnt_axis", _D), ("jnt_range", _D), ("jnt_margin", _D), ("jnt_solref", _D),
        ("jnt_solimp", _D),
        ("dof_bodyid", _I), ("dof_jntid", _I), ("dof_parentid", _I),
        ("dof_armature", _D), ("dof_damping", _D), ("dof_frictionloss", _D), ("dof_invweight0", _D),
        ("dof_solref", _D), ("dof_solimp", _D),
        ("geom_type", _I), ("geom_bodyid", _I), ("geom_dataid", _I),
        ("geom_pos", _D), ("geom_quat", _D), ("geom_rbound", _D), ("geom_size", _D),
        ("pair_geom1", _I), ("pair_geom2", _I), ("pair_condim", _I),
        ("pair_friction", _D), ("pair_solref", _D), ("pair_solimp", _D), ("pair_margin", _D),
        ("hull_nvert", C.c_int), ("hull_nface", C.c_int), ("hull_nedge", C.c_int),
        ("hull_vert", _D), ("hull_face_normal", _D), ("hull_face_offset", _D), ("hull_edge", _I),
        ("hfield_nrow", C.c_int), ("hfield_ncol", C.c_int), ("hfield_size", C.c_double * 4), ("hfield_data", _D),
        ("site_bodyid", _I), ("site_pos", _D), ("site_quat", _D),
        ("actuator_trnid", _I), ("actuator_ctrllimited", _I), ("actuator_forcelimited", _I),
        ("actuator_kp", _D), ("actuator_kv", _D), ("actuator_gear", _D), ("actuator_ctrlrange", _D),
        ("actuator_forcerange", _D),
        ("sensor_type", _I), ("sensor_objid", _I), ("sensor_adr", _I), ("sensor_dim", _I),
        ("qpos0", _D),
    ]


class DuckEnvConfig(C.Structure):
    _fields_ = [
        ("ctrl_dt", C.c_float), ("sim_dt", C.c_float), ("n_substeps", C.c_int),
        ("episode_length", C.c_int), ("auto_reset", C.c_int),
        ("action_scale", C.c_float), ("dof_vel_scale", C.c_float), ("max_motor_velocity", C.c_float),
        ("use_imitation", C.c_int), ("use_motor_speed_limits", C.c_int),
        ("noise_level", C.c_float),
        ("action_min_delay", C.c_int), ("action_max_delay", C.c_int), ("imu_min_delay", C.c_int),
        ("imu_max_delay", C.c_int),
        ("noise_gyro", C.c_float), ("noise_accelerometer", C.c_float), ("noise_gravity", C.c_float),
        ("noise_joint_vel", C.c_float),
        ("qpos_noise_scale", C.c_float * 16),
        ("scale_tracking_lin_vel", C.c_float), ("scale_tracking_ang_vel", C.c_float), ("scale_torques", C.c_float),
        ("scale_action_rate", C.c_float), ("scale_alive", C.c_float), ("scale_imitation", C.c_float),
        ("scale_stand_still", C.c_float),
        ("tracking_sigma", C.c_float),
        ("push_enable", C.c_int),
        ("push_interval_range", C.c_float * 2), ("push_magnitude_range", C.c_float * 2),
        ("lin_vel_x", C.c_float * 2), ("lin_vel_y", C.c_float * 2), ("ang_vel_yaw", C.c_float * 2),
        ("neck_pitch_range", C.c_float * 2), ("head_pitch_range", C.c_float * 2), ("head_yaw_range", C.c_float * 2),
        ("head_roll_range", C.c_float * 2), ("head_range_factor", C.c_float),
        ("default_actuator", C.c_float * 16), ("init_qpos", C.c_float * 40),
        ("actuator_qposadr", C.c_int * 16), ("actuator_qveladr", C.c_int * 16), ("backlash_qposadr", C.c_int * 16),
        ("imu_site", C.c_int), ("left_foot_site", C.c_int), ("right_foot_site", C.c_int),
        ("floor_geom", C.c_int), ("left_foot_geom", C.c_int), ("right_foot_geom", C.c_int),
        ("sens_gyro", C.c_int), ("sens_accelerometer", C.c_int), ("sens_upvector", C.c_int),
        ("sens_local_linvel", C.c_int), ("sens_global_angvel", C.c_int), ("sens_left_foot_linvel", C.c_int),
        ("sens_right_foot_linvel", C.c_int),
        ("domain_randomize", C.c_int),
        ("task", C.c_int), ("scale_orientation", C.c_float), ("scale_head_pos", C.c_float),
    ]


class DuckRefMotion(C.Structure):
    _fields_ = [
        ("n_dx", C.c_int), ("n_dy", C.c_int), ("n_dtheta", C.c_int), ("n_dim", C.c_int), ("n_coef", C.c_int),
        ("nb_steps_in_period", C.c_int),
        ("dxs", C.c_float * 16), ("dys", C.c_float * 16), ("dthetas", C.c_float * 16),
        ("dx_range", C.c_float * 2), ("dy_range", C.c_float * 2), ("dtheta_range", C.c_float * 2),
        ("frames", C.POINTER(C.c_float)), ("coeffs", C.POINTER(C.c_double)),
    ]


class ModelDescHolder:
    """Owns the numpy buffers a :class:`DuckModelDesc` points into."""

    def __init__(self, m: Model):
        self._keep: List[np.ndarray] = []
        d = DuckModelDesc()
        for k in ("nq", "nv", "nu", "nbody", "njnt", "ngeom", "nsite", "nsensor", "nsensordata", "npair"):
            setattr(d, k, int(getattr(m, k)))
        d.timestep = m.opt_timestep
        d.gravity[:] = list(m.opt_gravity)
        d.impratio = m.opt_impratio
        d.tolerance = m.opt_tolerance
        d.ls_tolerance = m.opt_ls_tolerance
        d.meaninertia = m.stat_meaninertia
        d.iterations = m.opt_iterations
        d.ls_iterations = m.opt_ls_iterations
        d.eulerdamp = m.opt_eulerdamp
        for name, typ in DuckModelDesc._fields_:
            if typ is _I or typ is _D:
                src = name
                if name.startswith("hull_"):
                    continue
                if name == "hfield_data":
                    continue
                arr = m.arrays[src]
                setattr(d, name, self._ptr(arr, typ))
        h = m.hulls[0]
        d.hull_nvert, d.hull_nface, d.hull_nedge = len(h.vert), len(h.face_normal), len(h.edge)
        d.hull_vert = self._ptr(h.vert, _D)
        d.hull_face_normal = self._ptr(h.face_normal, _D)
        d.hull_face_offset = self._ptr(h.face_offset, _D)
        d.hull_edge = self._ptr(h.edge, _I)
        d.hfield_nrow, d.hfield_ncol = int(m.hfield_nrow), int(m.hfield_ncol)
        d.hfield_size[:] = list(m.hfield_size)
        d.hfield_data = self._ptr(m.hfield_data if m.hfield_nrow else np.zeros(1), _D)
        self.desc = d

    def _ptr(self, arr, typ):
        if typ is _I:
            a = np.ascontiguousarray(arr, dtype=np.int32)
        else:
            a = np.ascontiguousarray(arr, dtype=np.float64)
        self._keep.append(a)
        return a.ctypes.data_as(typ)


def reference_frames(table: Dict[str, np.ndarray]) -> np.ndarray:
    """Polynomials evaluated (float64) at every phase t = i / nb: [nx, ny, nth, nb, ndim]."""
    nb = int(table["nb_steps_in_period"])
    t = np.arange(nb, dtype=np.float64) / nb
    c = np.asarray(table["coeffs"], dtype=np.float64)  # ascending powers
    out = np.zeros(c.shape[:3] + (nb, c.shape[3]))
    for k in range(c.shape[-1] - 1, -1, -1):  # Horner
        out = out * t[None, None, None, :, None] + c[:, :, :, None, :, k]
    return out


def refmotion_struct(table: Dict[str, np.ndarray]):
    r = DuckRefMotion()
    coeffs = np.ascontiguousarray(table["coeffs"], dtype=np.float64)
    frames = np.ascontiguousarray(reference_frames(table), dtype=np.float32)
    r.n_dx, r.n_dy, r.n_dtheta, r.n_dim, r.n_coef = coeffs.shape
    r.nb_steps_in_period = int(table["nb_steps_in_period"])
    r.dxs[:len(table["dxs"])] = [float(x) for x in table["dxs"]]
    r.dys[:len(table["dys"])] = [float(x) for x in table["dys"]]
    r.dthetas[:len(table["dthetas"])] = [float(x) for x in table["dthetas"]]
    r.dx_range[:] = [float(x) for x in table["dx_range"]]
    r.dy_range[:] = [float(x) for x in table["dy_range"]]
    r.dtheta_range[:] = [float(x) for x in table["dtheta_range"]]
    r.coeffs = coeffs.ctypes.data_as(C.POINTER(C.c_double))
    r.frames = frames.ctypes.data_as(C.POINTER(C.c_float))
    return r, (coeffs, frames)


# --------------------------------------------------------------------------------------
# layouts (mirror of duck_layout_make / duck_dr_layout_make in include/duck_env.h)
# --------------------------------------------------------------------------------------

@dataclass
class Layout:
    nq: int
    nv: int
    nu: int
    imitation: int
    task: int
    off: Dict[str, int]
    ioff: Dict[str, int]
    nfloat: int
    nint: int
    obs_size: int
    priv_size: int


TASK_JOYSTICK, TASK_STANDING = 0, 1


def layout(nq: int, nv: int, nu: int, imitation: bool, task: int = TASK_JOYSTICK) -> Layout:
    imitation = bool(imitation) and task == TASK_JOYSTICK
    if task == TASK_STANDING:  # standing.py:532-570
        obs = 3 + 3 + 7 + 5 * nu + 2
        priv = obs + 15 + 2 * nu + 1 + nu + 2 + 6 + 2
    else:
        obs = 3 + 3 + 7 + 6 * nu + 2 + 2
        priv = obs + 15 + 2 * nu + 1 + nu + 2 + 6 + 2 + (40 if imitation else 0) + 1 + 2
    fields = [("qpos", nq), ("qvel", nv), ("qacc_warmstart", nv), ("ctrl", nu), ("command", 7), ("last_act", nu),
              ("last_last_act", nu), ("last_last_last_act", nu), ("motor_targets", nu), ("feet_air_time", 2),
              ("last_contact", 2), ("swing_peak", 2), ("push", 2), ("action_history", 3 * nu), ("imu_history", 9),
              ("ref_motion", 40), ("imitation_phase", 2), ("metrics", 8), ("reward", 1), ("done", 1),
              ("truncation", 1), ("first_qpos", nq), ("first_qvel", nv), ("first_qacc_warmstart", nv),
              ("first_ctrl", nu), ("first_obs", obs), ("first_priv", priv)]
    off, o = {}, 0
    for k, n in fields:
        off[k] = o
        o += n
    ifields = [("rng_key", 2), ("rng_ctr", 1), ("step", 1), ("push_step", 1), ("push_interval", 1),
               ("imitation_i", 1), ("ep_steps", 1)]
    ioff, io = {}, 0
    for k, n in ifields:
        ioff[k] = io
        io += n
    return Layout(nq, nv, nu, int(imitation), int(task), off, ioff, o, io, obs, priv)


def dr_layout(nbody: int, nu: int) -> Dict[str, int]:
    out, o = {}, 0
    for k, n in [("floor_friction", 1), ("base_ipos", 3), ("body_mass", nbody), ("frictionloss", nu),
                 ("armature", nu), ("qpos0", nu), ("kp", nu)]:
        out[k] = o
        o += n
    out["nfloat"] = o
    return out


METRIC_NAMES = ["reward/tracking_lin_vel", "reward/tracking_ang_vel", "cost/torques", "cost/action_rate",
                "reward/alive", "reward/imitation", "cost/stand_still", "swing_peak"]
# standing.py:290-297 + :584-606 (slot 6 unused; swing_peak stays in slot 7)
STANDING_METRIC_NAMES = ["cost/orientation", "cost/torques", "cost/action_rate", "reward/alive", "cost/stand_still",
                         "cost/head_pos", None, "swing_peak"]


# --------------------------------------------------------------------------------------
# model fingerprint (mirror of duck_model_fingerprint in csrc/duck_capi.hip)
# --------------------------------------------------------------------------------------

def _fp_fields(d: DuckModelDesc):
    """(kind, name, count) in the hash order of duck_model_fingerprint."""
    nb, nj, nv, ng, np_, ns, nu = d.nbody, d.njnt, d.nv, d.ngeom, d.npair, d.nsite, d.nu
    out = []
    out += [("i", n, nb) for n in ("body_parentid", "body_rootid", "body_weldid", "body_jntnum", "body_jntadr",
                                   "body_dofnum", "body_dofadr")]
    out += [("f", "body_pos", 3 * nb), ("f", "body_quat", 4 * nb), ("f", "body_ipos", 3 * nb),
            ("f", "body_iquat", 4 * nb), ("f", "body_mass", nb), ("f", "body_inertia", 3 * nb),
            ("f", "body_invweight0", 2 * nb)]
    out += [("i", n, nj) for n in ("jnt_type", "jnt_qposadr", "jnt_dofadr", "jnt_bodyid", "jnt_limited")]
    out += [("f", "jnt_pos", 3 * nj), ("f", "jnt_axis", 3 * nj), ("f", "jnt_range", 2 * nj), ("f", "jnt_margin", nj),
            ("f", "jnt_solref", 2 * nj), ("f", "jnt_solimp", 5 * nj)]
    out += [("i", n, nv) for n in ("dof_bodyid", "dof_jntid", "dof_parentid")]
    out += [("f", n, nv) for n in ("dof_armature", "dof_damping", "dof_frictionloss", "dof_invweight0")]
    out += [("f", "dof_solref", 2 * nv), ("f", "dof_solimp", 5 * nv)]
    out += [("i", n, ng) for n in ("geom_type", "geom_bodyid", "geom_dataid")]
    out += [("f", "geom_pos", 3 * ng), ("f", "geom_quat", 4 * ng), ("f", "geom_rbound", ng), ("f", "geom_size", 3 * ng)]
    out += [("i", n, np_) for n in ("pair_geom1", "pair_geom2", "pair_condim")]
    out += [("f", "pair_friction", 5 * np_), ("f", "pair_solref", 2 * np_), ("f", "pair_solimp", 5 * np_),
            ("f", "pair_margin", np_)]
    return out


def model_fingerprint(m: Model) -> int:
    """Identity of a compiled kernel specialisation: FNV-1a 64 over the float32-rounded model values
    the generated header bakes (the same bytes duck_model_fingerprint hashes from a duck_model_desc)."""
    h = ModelDescHolder(m)
    d = h.desc
    buf = []
    buf.append(np.array([d.nq, d.nv, d.nu, d.nbody, d.njnt, d.ngeom, d.nsite, d.nsensor, d.nsensordata, d.npair,
                         d.iterations, d.ls_iterations, d.eulerdamp], dtype=np.int32).tobytes())
    buf.append(np.array([d.timestep, *d.gravity, d.impratio, d.tolerance, d.ls_tolerance, d.meaninertia],
                        dtype=np.float32).tobytes())

    def arr(kind, name, n):
        if n == 0:
            return b""
        p = getattr(d, name)
        a = np.ctypeslib.as_array(p, shape=(n,))
        return a.astype(np.int32 if kind == "i" else np.float32).tobytes()

    for kind, name, n in _fp_fields(d):
        buf.append(arr(kind, name, n))
    buf.append(np.array([d.hull_nvert, d.hull_nface, d.hull_nedge, d.hfield_nrow, d.hfield_ncol],
                        dtype=np.int32).tobytes())
    buf.append(arr("f", "hull_vert", 3 * d.hull_nvert))
    buf.append(arr("f", "hull_face_normal", 3 * d.hull_nface))
    buf.append(arr("f", "hull_face_offset", d.hull_nface))
    buf.append(arr("i", "hull_edge", 2 * d.hull_nedge))
    buf.append(np.array(list(d.hfield_size), dtype=np.float32).tobytes())
    ns, nu, nsen = d.nsite, d.nu, d.nsensor
    buf.append(arr("i", "site_bodyid", ns) + arr("f", "site_pos", 3 * ns) + arr("f", "site_quat", 4 * ns))
    for n in ("actuator_trnid", "actuator_ctrllimited", "actuator_forcelimited"):
        buf.append(arr("i", n, nu))
    for n in ("actuator_kp", "actuator_kv", "actuator_gear"):
        buf.append(arr("f", n, nu))
    buf.append(arr("f", "actuator_ctrlrange", 2 * nu) + arr("f", "actuator_forcerange", 2 * nu))
    for n in ("sensor_type", "sensor_objid", "sensor_adr", "sensor_dim"):
        buf.append(arr("i", n, nsen))
    buf.append(arr("f", "qpos0", d.nq))
    h64 = 1469598103934665603
    for c in b"".join(buf):
        h64 = ((h64 ^ c) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h64
