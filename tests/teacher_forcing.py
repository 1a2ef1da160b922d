"""Teacher-forced env parity: one Joystick.step of libduck.so from the oracle's own state.

Test infrastructure (imports the oracle). Free-running fp32 and fp64 trajectories of a contact
system separate within a few env-steps, so long free-running comparisons can only be loose.
Here the oracle is the trajectory: before every env-step its fp64 state is rounded to fp32 and
uploaded into the GPU's ``fstate``/``istate`` (and the oracle continues from the same rounded
state), both take the same action, and the two results are compared field by field -- qpos,
qvel, qacc_warmstart, every info field, obs, privileged obs, reward, done and the integer
bookkeeping. The error of one env-step is then the error of the kernel, not of a chaotic
trajectory.

Outliers are classified, not tolerated blindly (`explain`): the GPU replays the outlier's env-step
substep by substep and the oracle takes every substep from the GPU's own input. If each substep
agrees (or the GPU's result is a branch the oracle also takes under a 1e-6 input perturbation),
the kernel is right at every state it visited and the env-step difference is the oracle's own
sensitivity, amplified over 10 substeps (a contact row or friction edge switching, a line-search
tie): "sensitive". Anything else is a "defect".
"""

from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import numpy as np
import torch

from open_duck_playground_amd.joystick import Joystick, domain_randomize, wrap_for_brax_training
from open_duck_playground_amd.mjcf import Hull, Model
from tests.oracle_ffi import OracleBatch, OracleModel

# per-env error = max over a field group of |gpu - oracle| / (1 + |oracle|)
GROUPS = ("qpos", "qvel", "qacc_warmstart", "info", "obs", "priv", "reward")
INT_FIELDS = ("rng_key", "rng_ctr", "step", "push_step", "push_interval", "imitation_i", "ep_steps")


@dataclass
class StepStats:
    err: Dict[str, np.ndarray]          # group -> [n] relative error
    done_mismatch: np.ndarray           # [n] bool
    int_mismatch: np.ndarray            # [n] bool


@dataclass
class Report:
    steps: List[StepStats] = field(default_factory=list)
    tol: Dict[str, float] = field(default_factory=dict)
    pre: list = field(default_factory=list)   # per step (fs, is, action) before the step (keep_states)
    post: list = field(default_factory=list)  # per step the GPU's fstate after the step (keep_states)
    reset: dict = field(default_factory=dict)  # the strict post-reset comparison (reset_stats)
    env: object = None
    models: object = None

    def outliers(self, s: StepStats) -> np.ndarray:
        bad = np.zeros_like(s.done_mismatch)
        for g in GROUPS:
            bad |= s.err[g] > self.tol[g]
        return bad

    def summary(self) -> dict:
        n_env_steps = sum(len(s.done_mismatch) for s in self.steps)
        out = sum(int(self.outliers(s).sum()) for s in self.steps)
        q = {}
        for g in GROUPS:
            e = np.concatenate([s.err[g] for s in self.steps])
            q[g] = (float(np.median(e)), float(np.quantile(e, 0.99)), float(e.max()))
        return {"env_steps": n_env_steps, "outliers": out,
                "good_frac": 1 - out / max(n_env_steps, 1), "err_median_p99_max": q}


def default_tol() -> Dict[str, float]:
    return {"qpos": 1e-4, "qvel": 2e-3, "qacc_warmstart": 2e-2, "info": 2e-3, "obs": 2e-3, "priv": 2e-3,
            "reward": 2e-3}


def _group_slices(L):
    o = L.off
    info = [(o["command"], o["metrics"] + 8)]   # command .. metrics (incl. motor targets, histories, ref)
    return {"qpos": [(o["qpos"], o["qpos"] + L.nq)], "qvel": [(o["qvel"], o["qvel"] + L.nv)],
            "qacc_warmstart": [(o["qacc_warmstart"], o["qacc_warmstart"] + L.nv)],
            "info": info + [(o["ctrl"], o["ctrl"] + L.nu), (o["truncation"], o["truncation"] + 1)]}


def _rel(a, b):
    return np.abs(a - b) / (1 + np.abs(b))


def _fs_err(L, fa, fb, n):
    A = fa.reshape(L.nfloat, n)
    B = fb.reshape(L.nfloat, n)
    out = {}
    for g, sl in _group_slices(L).items():
        out[g] = np.max(np.concatenate([_rel(A[a:b], B[a:b]) for a, b in sl], axis=0), axis=0)
    return out


def run(task: str, imitation: bool, n: int, steps: int, device, seed: int = 7, dr: bool = False,
        auto_reset: bool = False, episode_length: int = 1000, overrides: Optional[dict] = None,
        force_push: bool = False, force_resample: bool = False, env_cls=Joystick, action_seed: int = 0,
        keep_states: bool = False, oracle_edit: Optional[Callable[[Model], Model]] = None,
        step_mode: str = "auto") -> Report:
    """``oracle_edit`` hands the oracle a deliberately wrong model (a copy of the GPU's, edited; the
    GPU keeps the nominal one): the injected-defect test of ``explain`` (DEFECTS). ``step_mode``:
    Joystick.set_step_mode ("auto" runs the latency kernel at these batch sizes, <= 4 envs per CU)."""
    kw = {} if env_cls is not Joystick else {"use_imitation": imitation}
    env = env_cls(task, num_envs=n, device=device, config_overrides=overrides, **kw)
    if auto_reset:
        env = wrap_for_brax_training(env, episode_length=episode_length,
                                     randomization_fn=domain_randomize if dr else None, rng=seed + 1)
    elif dr:
        domain_randomize(env, rng=seed + 1)
    env.set_step_mode(step_mode)
    st = env.reset(rng=seed)
    om_model = oracle_edit(copy_model(env.mj_model)) if oracle_edit is not None else env.mj_model
    base = OracleModel(om_model)
    models = [OracleModel(om_model, dr=base.dr_sample(seed + 1, e)) for e in range(n)] if dr else base
    cfg = env._cfg_struct                      # the exact struct duck_create received
    L = env._layout
    ob = OracleBatch(models, cfg, n)
    ob.reset(seed=seed)
    rng = np.random.default_rng(action_seed)
    rep = Report(tol=default_tol(), env=env, models=models)
    torch.cuda.synchronize()
    rep.reset = reset_stats(L, st, ob, n)
    I = lambda name: L.ioff[name]  # noqa: E731
    for t in range(steps):
        isv = ob.is_.reshape(L.nint, n)
        if t == 0 and force_push:        # every third env pushed on this step (push_step+1 == interval)
            sel = np.arange(n) % 3 == 0
            isv[I("push_step"), sel] = np.maximum(isv[I("push_interval"), sel] - 1, 0)
        if t == 0 and force_resample:    # every fourth env past step 500: command resample + step reset
            sel = np.arange(n) % 4 == 1
            isv[I("step"), sel] = 500
        ob.fs[:] = ob.fs.astype(np.float32).astype(np.float64)
        st.fstate.copy_(torch.from_numpy(ob.fs.astype(np.float32)))
        st.istate.copy_(torch.from_numpy(ob.is_.copy()))
        a = rng.uniform(-1, 1, (n, env.action_size)).astype(np.float32)
        if keep_states:
            rep.pre.append((ob.fs.copy(), ob.is_.copy(), a.copy()))
        st = env.step(st, torch.from_numpy(a).to(st.fstate.device))
        ob.step(a.astype(np.float64))
        torch.cuda.synchronize()
        gf = st.fstate.cpu().numpy().astype(np.float64)
        gi = st.istate.cpu().numpy()
        if keep_states:
            rep.post.append(gf.copy())
        err = _fs_err(L, gf, ob.fs, n)
        obs = st.obs["state"].cpu().numpy().astype(np.float64)
        priv = st.obs["privileged_state"].cpu().numpy().astype(np.float64)
        err["obs"] = _rel(obs, ob.obs).max(axis=1)
        err["priv"] = _rel(priv, ob.priv).max(axis=1)
        err["reward"] = _rel(st.reward.cpu().numpy().astype(np.float64), ob.rew)
        done_mm = st.done.cpu().numpy() != ob.done
        GI, OI = gi.reshape(L.nint, n), ob.is_.reshape(L.nint, n)
        int_mm = np.zeros(n, dtype=bool)
        for name in INT_FIELDS:
            if name in L.ioff:
                int_mm |= GI[L.ioff[name]] != OI[L.ioff[name]]
        rep.steps.append(StepStats(err=err, done_mismatch=done_mm, int_mismatch=int_mm))
    return rep


def reset_stats(L, st, ob, n: int) -> dict:
    """Joystick.reset (joystick.py:206-321) strictly, field by field: every fstate row of every env
    (state, info, the auto-reset snapshot) against oracle_env_reset at the teacher-forced bar (qpos
    rows 1e-4, qacc_warmstart rows 2e-2, every other row 2e-3, relative to 1 + |oracle|), obs and
    privileged obs at 2e-3, every istate word exact. Returns per-env worst row error / its bar
    ("norm", > 1 fails), the worst row's name, and the integer / obs mismatches."""
    A = st.fstate.cpu().numpy().astype(np.float64).reshape(L.nfloat, n)
    B = ob.fs.reshape(L.nfloat, n)
    tol = np.full(L.nfloat, 2e-3)
    name = np.empty(L.nfloat, dtype=object)
    bounds = sorted(L.off.items(), key=lambda kv: kv[1]) + [("end", L.nfloat)]
    for (k, a), (_, b) in zip(bounds[:-1], bounds[1:]):
        name[a:b] = k
        if k in ("qpos", "first_qpos"):
            tol[a:b] = 1e-4
        elif k in ("qacc_warmstart", "first_qacc_warmstart"):
            tol[a:b] = 2e-2
    r = _rel(A, B) / tol[:, None]
    worst = r.argmax(axis=0)
    obs = st.obs["state"].cpu().numpy().astype(np.float64)
    priv = st.obs["privileged_state"].cpu().numpy().astype(np.float64)
    oerr = np.maximum(_rel(obs, ob.obs).max(axis=1), _rel(priv, ob.priv).max(axis=1)) / 2e-3
    GI, OI = st.istate.cpu().numpy().reshape(L.nint, n), ob.is_.reshape(L.nint, n)
    return {"norm": np.maximum(r.max(axis=0), oerr), "worst_row": name[worst],
            "int_mismatch": np.any(GI != OI, axis=0), "fs_norm": r.max(axis=0), "obs_norm": oerr,
            "gpu_fs": A.copy(), "ora_fs": B.copy()}


def explain_reset(rep: Report, e: int, seed: int = 0) -> dict:
    """Why env e's reset differs: the reset ends with mjx.forward (mjx_env.init, joystick.py:258),
    whose constrained qacc (stored as qacc_warmstart; the accelerometer in obs) can take another
    contact branch from fp32-sized differences of the sampled state. "sensitive" when the oracle's
    forward from its reset state, perturbed by 1e-6 / 1e-5, lands on the GPU's qacc (a branch the
    oracle also takes) and every integer word matches; otherwise "defect"."""
    env, m = rep.env, rep.env.mj_model
    L, o = env._layout, env._layout.off
    G, B = rep.reset["gpu_fs"][:, e], rep.reset["ora_fs"][:, e]
    if rep.reset["int_mismatch"][e]:
        return {"kind": "defect", "why": "integer words"}
    om = rep.models[e] if isinstance(rep.models, list) else rep.models
    x = np.concatenate([B[o["qpos"]:o["qpos"] + m.nq], B[o["qvel"]:o["qvel"] + m.nv], np.zeros(m.nv),
                        B[o["ctrl"]:o["ctrl"] + m.nu]])
    target = np.concatenate([G[o["qpos"]:o["qpos"] + m.nq], G[o["qvel"]:o["qvel"] + m.nv],
                             G[o["qacc_warmstart"]:o["qacc_warmstart"] + m.nv], G[o["ctrl"]:o["ctrl"] + m.nu]])

    def fwd(y):
        q, v, w, c = _split(m, y)
        d = om.new_data(qpos=q, qvel=v, ctrl=c, warm=w)
        om.forward(d)
        return np.concatenate([q, v, d.arr("qacc", m.nv), c])
    d0 = _state_rel(m, fwd(x), target)
    rng = np.random.default_rng(seed)
    k = m.nq + m.nv
    for lev in (1e-6, 1e-5):
        for _ in range(24):
            y = x.copy()
            y[:k] *= 1 + lev * rng.choice([-1.0, 1.0], size=k)
            y[:k] += 1e-3 * lev * rng.choice([-1.0, 1.0], size=k)
            if _state_rel(m, fwd(y), target) < 0.25 * d0:
                return {"kind": "sensitive", "flip": lev, "forward_err": d0}
    return {"kind": "defect", "why": "forward", "forward_err": d0}


def _short_push():
    # pushes every 1-3 env-steps (reset draws the interval from this range): the push path runs
    return {"push_config.interval_range": [0.02, 0.06]}


# name -> run() arguments; every scene the kernels are built for, the Standing task, the training
# wrappers with a 3-step episode (auto-reset restore on the GPU vs the oracle), pushes and the
# 500-step command resample
CASES = {
    "flat": dict(task="flat_terrain", imitation=False, force_push=True, force_resample=True),
    "flat_imitation": dict(task="flat_terrain", imitation=True, force_push=True, force_resample=True),
    "flat_backlash_imitation": dict(task="flat_terrain_backlash", imitation=True, force_push=True),
    "rough_dr": dict(task="rough_terrain", imitation=False, dr=True, force_push=True),
    "rough_backlash_dr": dict(task="rough_terrain_backlash", imitation=False, dr=True, force_resample=True),
    "flat_autoreset_pushes": dict(task="flat_terrain", imitation=False, auto_reset=True, episode_length=3,
                                  overrides=_short_push()),
    "rough_backlash_dr_autoreset": dict(task="rough_terrain_backlash", imitation=False, dr=True, auto_reset=True,
                                        episode_length=3, overrides=_short_push()),
    "flat_zero_push_interval": dict(task="flat_terrain", imitation=False,
                                    overrides={"push_config.interval_range": [0.0, 0.009]}),
    # an edited MJCF scene on its own compiled kernels (native.model_library)
    "edited_scene": dict(task=os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "models",
                                           "flat_terrain_edited.npz"), imitation=False, force_push=True,
                         force_resample=True),
    "standing": dict(task="flat_terrain", imitation=False, force_push=True, force_resample=True, standing=True),
    # the throughput kernel (16 envs per workgroup) at the same size; the cases above run the latency
    # kernel ("auto" at <= 4 envs per CU)
    "flat_throughput_kernel": dict(task="flat_terrain", imitation=True, force_push=True, force_resample=True,
                                   step_mode="throughput"),
    "rough_backlash_dr_throughput_kernel": dict(task="rough_terrain_backlash", imitation=False, dr=True,
                                                force_push=True, step_mode="throughput"),
    # the paired latency kernel (each substep's stages over a pair of waves per 4 envs)
    "flat_paired_kernel": dict(task="flat_terrain", imitation=True, force_push=True, force_resample=True,
                               step_mode="paired"),
    # the latency kernel at two workgroups per CU (round 6; plane-floor scenes without backlash)
    "flat_latency_x2_kernel": dict(task="flat_terrain", imitation=True, force_push=True, force_resample=True,
                                   step_mode="latency_x2"),
    "rough_backlash_dr_paired_kernel": dict(task="rough_terrain_backlash", imitation=False, dr=True,
                                            force_push=True, step_mode="paired"),
}


def copy_model(m: Model) -> Model:
    return Model(name=m.name, arrays={k: v.copy() for k, v in m.arrays.items()}, names=dict(m.names),
                 hulls=[Hull(vert=h.vert.copy(), face_normal=h.face_normal.copy(), face_offset=h.face_offset.copy(),
                             face_vert=[list(f) for f in h.face_vert], edge=h.edge.copy()) for h in m.hulls])


def _floor_friction(m: Model) -> Model:      # the contact pairs' sliding friction x 1.02
    m.arrays["pair_friction"][:, :2] *= 1.02
    return m


def _one_kp(m: Model) -> Model:              # the left knee servo's kp x 1.005
    m.arrays["actuator_kp"][3] *= 1.005
    return m


def _solref(m: Model) -> Model:              # the contact pairs' solref time constant x 1.02
    m.arrays["pair_solref"][:, 0] *= 1.02
    return m


def _foot_hull(m: Model) -> Model:           # the foot hull scaled by 1.0005 about its mesh origin (~25 um)
    m.hulls = [Hull(vert=h.vert * 1.0005, face_normal=h.face_normal, face_offset=h.face_offset * 1.0005,
                    face_vert=h.face_vert, edge=h.edge) for h in m.hulls]
    return m


def _servo_damping(m: Model) -> Model:       # every hinge's damping x 1.01 (small, smooth force error)
    m.arrays["dof_damping"][6:] *= 1.01
    return m


def _one_kp_small(m: Model) -> Model:        # the left knee servo's kp x 1.001
    m.arrays["actuator_kp"][3] *= 1.001
    return m


# injected defects (name -> (case, oracle model edit, oracle knob)): the oracle runs a deliberately wrong
# model (edit) or a wrong contact generation (knob: oracle_set_hf_defect(which, value), a test aid of
# the oracle; the kernel keeps the declared rules) while the GPU runs the nominal one, so an outlier
# the defect induces IS a defect and explain() must say so (test_explain_has_teeth). The knob defects
# change only contact generation on the height field -- where sat_tie, onset, onset_selection and
# dup_selection fire: round 4's point band switched back on, the support features' witness band x 1.5,
# the deepest-prism tie x 100 (1e-4 m; at x 10 = 1e-5 m the defect sits at the reach of flip_level's 1e-5
# input perturbation, and 4 of 23 differing substeps were flips, none a contact rule: DESIGN.md §5), and the
# 4-slot manifold started from the second-deepest prism contact
DEFECTS = {
    "floor_friction_x1.02": ("flat", _floor_friction, None),
    "actuator_kp_x1.005": ("flat", _one_kp, None),
    "actuator_kp_x1.001": ("flat", _one_kp_small, None),
    "dof_damping_x1.01": ("flat", _servo_damping, None),
    "contact_solref_x1.02": ("flat", _solref, None),
    "foot_hull_x1.0005_hfield": ("rough_dr", _foot_hull, None),
    "hf_point_band_on": ("rough_dr", None, (0, 1.0)),
    "hf_witness_band_x1.5": ("rough_dr", None, (1, 1.5)),
    "hf_depth_tie_x100": ("rough_dr", None, (2, 100.0)),
    "hf_manifold_second_deepest": ("rough_dr", None, (3, 1.0)),
}


@contextlib.contextmanager
def oracle_knob(knob):
    """An injected contact-generation defect (DEFECTS' knob) in force inside the block, process-wide:
    the batched oracle of run() and the single-env oracle of explain() both run it."""
    if knob is None:
        yield
        return
    from tests.oracle_ffi import lib
    which, value = knob
    old = lib().oracle_get_hf_defect(which)
    lib().oracle_set_hf_defect(which, value)
    try:
        yield
    finally:
        lib().oracle_set_hf_defect(which, old)


def nominal_agrees(rep: "Report", t: int, e: int, knob) -> bool:
    """Is env e's env-step t an outlier only because of the injected knob defect? The oracle with the
    declared rules (the knob switched off), from the same teacher-forced pre-state and action, lands
    inside every teacher-forcing bar on the GPU's result."""
    from tests.oracle_ffi import OracleEnv, lib
    env, L, n = rep.env, rep.env._layout, rep.env.num_envs
    fs, is_, a = rep.pre[t]
    om = rep.models[e] if isinstance(rep.models, list) else rep.models
    which, _ = knob
    old = lib().oracle_get_hf_defect(which)
    lib().oracle_set_hf_defect(which, (0.0, 1.0, 1.0, 0.0)[which])
    try:
        oe = OracleEnv(om, env._cfg_struct)
        oe.fs[:] = fs.reshape(L.nfloat, n)[:, e]
        oe.is_[:] = is_.reshape(L.nint, n)[:, e]
        oe.step(a[e].astype(np.float64))
    finally:
        lib().oracle_set_hf_defect(which, old)
    G = rep.post[t].reshape(L.nfloat, n)[:, e:e + 1]
    err = _fs_err(L, G.ravel(), oe.fs.reshape(L.nfloat, 1).ravel(), 1)
    return all(err[g][0] <= rep.tol[g] for g in err)


def run_case(name: str, device, n: int = 256, steps: int = 6, **extra) -> Report:
    kw = dict(CASES[name], **extra)
    if kw.pop("standing", False):
        from open_duck_playground_amd.standing import Standing
        kw["env_cls"] = Standing
    return run(n=n, steps=steps, device=device, **kw)


# ---------------------------------------------------------------------------------------------
# outlier explanation at substep resolution
# ---------------------------------------------------------------------------------------------

def substep_trace(rep: Report, e: int, t: int):
    """The oracle's env-step t of env e with every substep's input state (qpos, qvel,
    qacc_warmstart, ctrl); row n_substeps is the final state. Needs keep_states=True."""
    import ctypes as C
    from tests.oracle_ffi import OracleEnv, lib
    env, L = rep.env, rep.env._layout
    m, n = env.mj_model, env.num_envs
    fs, is_, a = rep.pre[t]
    om = rep.models[e] if isinstance(rep.models, list) else rep.models
    oe = OracleEnv(om, env._cfg_struct)
    oe.fs[:] = fs.reshape(L.nfloat, n)[:, e]
    oe.is_[:] = is_.reshape(L.nint, n)[:, e]
    tr = np.zeros((env.n_substeps + 1, m.nq + 2 * m.nv + m.nu))
    lib().oracle_set_trace(tr.ctypes.data_as(C.POINTER(C.c_double)))
    try:
        oe.step(a[e].astype(np.float64))
    finally:
        lib().oracle_set_trace(None)
    o = L.off
    tr[-1, :m.nq] = oe.fs[o["qpos"]:o["qpos"] + m.nq]
    tr[-1, m.nq:m.nq + m.nv] = oe.fs[o["qvel"]:o["qvel"] + m.nv]
    tr[-1, m.nq + m.nv:m.nq + 2 * m.nv] = oe.fs[o["qacc_warmstart"]:o["qacc_warmstart"] + m.nv]
    tr[-1, m.nq + 2 * m.nv:] = tr[-2, m.nq + 2 * m.nv:]
    return om, tr


def _split(m, x):
    return x[:m.nq], x[m.nq:m.nq + m.nv], x[m.nq + m.nv:m.nq + 2 * m.nv], x[m.nq + 2 * m.nv:]


def gpu_substep(env, e: int, x: np.ndarray) -> np.ndarray:
    """One substep (duck_physics_step, nsub=1) of env column e from state x; returns the next state
    in trace layout (qacc_warmstart = this substep's qacc). Every column carries x (DR is per column)."""
    m, n, dev = env.mj_model, env.num_envs, env.device
    T = lambda y: torch.tensor(np.tile(y.astype(np.float32)[:, None], (1, n)), device=dev).contiguous()  # noqa: E731
    tq, tv, tw, tc = (T(y) for y in _split(m, x))
    env.physics_step(tq, tv, tw, tc, 1)
    torch.cuda.synchronize()
    return np.concatenate([tq[:, e].cpu().numpy(), tv[:, e].cpu().numpy(), tw[:, e].cpu().numpy(),
                           tc[:, e].cpu().numpy()]).astype(np.float64)


def oracle_substep(om, x: np.ndarray) -> np.ndarray:
    m = om.m
    q, v, w, c = _split(m, x)
    d = om.new_data(qpos=q, qvel=v, ctrl=c, warm=w)
    om.step(d, 1)
    return np.concatenate([d.arr("qpos", m.nq), d.arr("qvel", m.nv), d.arr("qacc_warmstart", m.nv),
                           d.arr("ctrl", m.nu)])


def oracle_substep_with_contacts(om, x: np.ndarray, ga: dict) -> np.ndarray:
    """oracle_substep with the contact set replaced, after collision, by the GPU's (parse_aux dict ga
    of one env: con_dist, con_pos, con_normal; oracle_set_con_override)."""
    import ctypes as C
    from tests.oracle_ffi import lib
    ncon = 4 * om.m.npair
    buf = np.zeros((ncon, 7))
    buf[:, 0] = ga["con_dist"][0][:ncon]
    buf[:, 1:4] = np.asarray(ga["con_pos"][0]).reshape(-1, 3)[:ncon]
    buf[:, 4:7] = np.asarray(ga["con_normal"][0]).reshape(-1, 3)[:ncon]
    buf = np.ascontiguousarray(buf.ravel())
    lib().oracle_set_con_override(buf.ctypes.data_as(C.POINTER(C.c_double)))
    try:
        return oracle_substep(om, x)
    finally:
        lib().oracle_set_con_override(None)


def _state_rel(m, a, b):
    """max relative error over qvel and qacc (qacc_warmstart) of two trace rows."""
    sl = slice(m.nq, m.nq + 2 * m.nv)
    return float(np.max(np.abs(a[sl] - b[sl])) / (1 + np.max(np.abs(b[sl]))))


def flip_level(om, x: np.ndarray, target: np.ndarray, rng, levels=(1e-6, 1e-5)) -> Optional[float]:
    """Smallest relative input perturbation at which the oracle's substep from x lands on target
    (closer than a quarter of the unperturbed distance): the target is one of the oracle's own
    branches at this state."""
    m = om.m
    d0 = _state_rel(m, oracle_substep(om, x), target)
    k = m.nq + 2 * m.nv
    for lev in levels:
        for _ in range(24):
            y = x.copy()
            y[:k] *= 1 + lev * rng.choice([-1.0, 1.0], size=k)
            y[:k] += 1e-3 * lev * rng.choice([-1.0, 1.0], size=k)
            if _state_rel(m, oracle_substep(om, y), target) < 0.25 * d0:
                return lev
    return None


def backward_error_landing(om, x: np.ndarray, target: np.ndarray, level: float = 1e-6,
                           contacts: Optional[tuple] = None) -> Optional[dict]:
    """Backward error of the GPU's substep: is there an input within `level` of x -- every qpos,
    qvel and qacc_warmstart coordinate moved by at most level * |x_i| + 1e-3 level, the size
    flip_level perturbs by -- from which the oracle's substep lands on target (closer than a quarter
    of the unperturbed distance)? Found by a bounded least-squares fit of target - f(x) to the
    oracle's finite-difference Jacobian (one column per input coordinate), then checked by running
    the oracle at the fitted input (the landing is real, not a linear prediction). The fit has more
    free inputs than outputs, so landing alone could absorb a small systematic force error; with
    `contacts` = the GPU's (con_dist, con_pos) at x the fitted input must also reproduce the GPU's
    contact set -- the same active slots, depths within 2e-6 m, points within 1e-4 m -- so the
    explanation is "the kernel computed this substep's contacts and everything after them at a
    nearby state", not a refit of the dynamics. A continuous sensitivity of the state (no branch
    flips) passes it; a model defect -- a systematic force error no fp32-sized input change produces --
    does not (test_explain_has_teeth, also at kp x 1.001 and damping x 1.01). Returns the fit
    (landed distance, max_coord = the largest input move as a fraction of its box) or None."""
    from scipy.optimize import lsq_linear
    m = om.m
    k = m.nq + 2 * m.nv
    sl = slice(m.nq, m.nq + 2 * m.nv)
    base = oracle_substep(om, x)
    d0 = _state_rel(m, base, target)
    h = level * np.abs(x[:k]) + 1e-3 * level
    J = np.empty((2 * m.nv, k))
    for i in range(k):
        y = x.copy()
        y[i] += h[i]
        J[:, i] = oracle_substep(om, y)[sl] - base[sl]
    fit = lsq_linear(J, target[sl] - base[sl], bounds=(-1.0, 1.0))
    y = x.copy()
    y[:k] += fit.x * h
    d = _state_rel(m, oracle_substep(om, y), target)
    if not d < 0.25 * d0:
        return None
    if contacts is not None:
        gd, gp = contacts
        q, v, w, c = _split(m, y)
        dd = om.new_data(qpos=q, qvel=v, ctrl=c, warm=w)
        om.forward(dd)
        od, op = _contacts(m, dd.arr("con_dist", 4 * m.npair), np.ctypeslib.as_array(dd.con_pos))
        act = (gd < 0) | (od < 0)
        if ((gd < 0) != (od < 0)).any() or (np.abs(gd - od)[act] > 2e-6).any() or \
                (np.abs(gp - op)[act].max(initial=0.0) > 1e-4):
            return None
    return {"landed": d, "unperturbed": d0, "max_coord": float(np.abs(fit.x).max())}


def _contacts(m, dist, pos):
    return np.asarray(dist, dtype=np.float64)[:4 * m.npair], np.asarray(pos, dtype=np.float64).reshape(-1, 3)[:4 * m.npair]


def oracle_contact_aux(om, x: np.ndarray) -> dict:
    """The oracle's contact set at x in parse_aux's layout for one env (con_dist, con_pos, con_normal):
    a stand-in for the GPU's in the CPU tests of the rules (test_explain_rules.py)."""
    m = om.m
    q, v, w, c = _split(m, x)
    d = om.new_data(qpos=q, qvel=v, ctrl=c, warm=w)
    om.forward(d)
    nc = 4 * m.npair
    return {"con_dist": d.arr("con_dist", nc)[None].copy(),
            "con_pos": np.ctypeslib.as_array(d.con_pos)[:nc].reshape(1, -1).copy(),
            "con_normal": np.ctypeslib.as_array(d.con_frame)[:nc, :3].reshape(1, -1).copy()}


def gpu_contact_aux(env, e: int, x: np.ndarray) -> dict:
    """The GPU's contact set at x (the forward of duck_physics_step with nsub = 0), env e's column."""
    from tests.helpers import parse_aux
    m, n = env.mj_model, env.num_envs
    T = lambda y: torch.tensor(np.tile(y.astype(np.float32)[:, None], (1, n)), device=env.device).contiguous()  # noqa: E731
    tq, tv, tw, tc = (T(y) for y in _split(m, x))
    aux = torch.zeros(env.aux_size() * n, dtype=torch.float32, device=env.device).view(-1, n)
    env.physics_step(tq, tv, tw, tc, 0, aux)
    torch.cuda.synchronize()
    return parse_aux(m, aux[:, e].cpu().numpy().astype(np.float64)[:, None])


def declared_difference(env, e: int, om, x: np.ndarray, g: np.ndarray, sub_tol: float, onset: float = 1e-6,
                        info: Optional[dict] = None, ga: Optional[dict] = None):
    """A substep where the GPU and the oracle differ beyond sub_tol from the same input, explained by
    one of the kernel's declared fp32 behaviours, or None:
    "ls_floor": the oracle with the kernel's line-search stop (slope below 1e-6 of the start; DESIGN.md
    §5 item 7) lands on the GPU's result (within sub_tol);
    "backward_error": the oracle from an input within 1e-6 of the GPU's input lands on the GPU's result
    and reproduces the GPU's contact set there (backward_error_landing: the kernel's fp32 substep is the
    exact substep of a nearby input; `info` receives the fit, max_coord included);
    "onset": the two contact sets differ only in slots that are, on each side, inactive or active
    within `onset` (m) of zero depth -- which prisms of a height field touch at the onset is decided
    below fp32 resolution.
    "sat_tie": two separating axes of one height-field prism overlap within 1e-6 m (the kernel's fp32
    error bound on an overlap), and the oracle resolving such ties to the other axis -- the last one in
    the band (oracle_set_hf_tie_last) or the first (oracle_set_hf_tie_first) -- lands on the GPU's result;
    "dup_selection": the same, around two prisms reporting one contact (the shared edge it lies on):
    equal in fp64, a few ulp apart in fp32, so the 4-point selection's choice is decided below fp32;
    "onset_selection": the manifold chose other prism contacts around an onset-depth prism -- every GPU
    slot of the differing pairs is one of the oracle's own prism contacts (oracle_hfield_contacts) or
    at the onset depth, and the oracle continued from the GPU's slots lands on the GPU's result
    (round 3's "onset_cascade" checked only the landing: a collision bug in a shallow pair would have
    passed). Round 3's "conditioning" rule -- the oracle merely moving by the GPU's difference under 1e-6
    perturbations, without landing on it -- is gone: a rule that does not require landing cannot tell
    a defect from a sensitive state, tests/test_gpu_teacher_forced.py::test_explain_has_teeth.)
    `ga`: the GPU's contact set at x (gpu_contact_aux; computed here when None -- the CPU tests of the
    rules pass an oracle's, oracle_contact_aux)."""
    from tests.oracle_ffi import lib
    m = om.m
    lib().oracle_set_ls_floor(1e-6)
    try:
        r = oracle_substep(om, x)
    finally:
        lib().oracle_set_ls_floor(0.0)
    if _state_rel(m, g, r) <= sub_tol:
        return "ls_floor"
    if ga is None:
        ga = gpu_contact_aux(env, e, x)
    gd, gp = _contacts(m, ga["con_dist"][0], ga["con_pos"][0])
    # backward error: the oracle from an fp32-sized perturbation of the input lands on the GPU's result
    # and has the GPU's contacts there
    be = backward_error_landing(om, x, g, contacts=(gd, gp))
    if be is not None:
        if info is not None:
            info["backward_error"] = be
        return "backward_error"
    # a height-field prism whose two best separating axes overlap within 1e-6 m (the kernel's fp32 error
    # bound on an overlap: tied at its precision): the oracle resolving such ties to the other axis
    # lands on the GPU
    for tie in (lib().oracle_set_hf_tie_last, lib().oracle_set_hf_tie_first):
        tie(1e-6)
        try:
            r = oracle_substep(om, x)
        finally:
            tie(0.0)
        if _state_rel(m, g, r) <= sub_tol:
            return "sat_tie"
    q, v, w, c = _split(m, x)
    d = om.new_data(qpos=q, qvel=v, ctrl=c, warm=w)
    om.forward(d)
    od, op = _contacts(m, d.arr("con_dist", 4 * m.npair), np.ctypeslib.as_array(d.con_pos))
    differ = ((gd < 0) != (od < 0)) | ((gd < 0) & (od < 0) & (np.abs(gp - op).max(axis=1) > 1e-4))
    # every differing slot is, on each side, inactive or active at the onset depth
    at_onset = ((gd >= 0) | (np.abs(gd) <= onset)) & ((od >= 0) | (np.abs(od) <= onset))
    if differ.any() and at_onset[differ].all():
        return "onset"
    # the 4-slot manifold's choice among the prism contacts of a height-field pair, decided below fp32
    # resolution: an onset-depth prism (in or out of the candidates at fp32), or candidates whose scores
    # tie within fp32 noise (two prisms reporting one contact on their shared edge: equal in fp64, a few
    # ulp apart in fp32). Accepted only if (a) for every differing pair, the oracle's own selection
    # (manifold_select = collide_hfield_convex's, oracle_hfield_select) over its own candidates
    # (oracle_hfield_contacts) reproduces the GPU's 4 slots -- same active slots, points within 1e-4 m,
    # depths within 2e-6 m -- in one of 256 trials that move every candidate by fp32-sized noise
    # (points 2e-5 m, depths 2e-7 m: the kernel's contact-point and depth errors) and drop onset-depth
    # candidates / add the GPU's onset-depth slots at random, and (b) the oracle continued from the
    # GPU's slots lands on the GPU's result (everything after collision agrees). "onset_selection"
    # when the reproducing trial needed an onset-depth candidate dropped or added, else "dup_selection".
    # (Round 4 accepted any GPU slot set whose slots were all among the oracle's candidates, given an
    # onset-depth or duplicate candidate: a manifold started from the second-deepest prism passed 14 of
    # 37 times, test_explain_rules.py::test_contact_rules_reject_contact_generation_defects.)
    pair_differs = differ.reshape(m.npair, 4).any(axis=1)
    if pair_differs.any():
        how = _selection_reproduced(m, om, d, ga, pair_differs, onset)
        if how is not None and _state_rel(m, g, oracle_substep_with_contacts(om, x, ga)) <= sub_tol:
            return how
    return None


def manifold_select(dep: np.ndarray, pt: np.ndarray, nrm: np.ndarray) -> List[int]:
    """The candidate indices of the 4 slots of a height-field pair: the oracle's own choice
    (oracle_hfield_select = collide_hfield_convex's hf_select: from the first candidate in strip order
    within HF_DEPTH_TIE of the deepest, mjx's _manifold_points), with whatever injected defect knob is
    in force -- the rules replay the oracle's procedure, not a copy of the declared one. Frame-free, so
    world-frame candidates give the oracle's choice (test_explain_rules.py::test_manifold_select_is_the_oracles)."""
    import ctypes as C
    from tests.oracle_ffi import lib
    dep, pt, nrm = (np.ascontiguousarray(a, dtype=np.float64) for a in (dep, pt, nrm))
    idx = np.zeros(4, dtype=np.int32)
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    if lib().oracle_hfield_select(dp(dep), dp(pt), dp(nrm), len(dep), idx.ctypes.data_as(C.POINTER(C.c_int32))) != 0:
        raise ValueError(f"{len(dep)} candidates")
    return [int(i) for i in idx]


def _slots_of(sel: List[int], dep: np.ndarray, pt: np.ndarray):
    """(depth or None when inactive, point) per slot: repeats stay inactive (plane_convex's rule)"""
    return [(dep[k] if k not in sel[:i] else None, pt[k]) for i, k in enumerate(sel)]


def _selection_reproduced(m, om, d, ga, pair_differs, onset, trials: int = 256, seed: int = 0) -> Optional[str]:
    import ctypes as C
    from tests.oracle_ffi import lib
    floor = m.id("geom", "floor")
    gd = np.asarray(ga["con_dist"][0], dtype=np.float64)
    gp = np.asarray(ga["con_pos"][0], dtype=np.float64).reshape(-1, 3)
    gn = np.asarray(ga["con_normal"][0], dtype=np.float64).reshape(-1, 3)
    rng = np.random.default_rng(seed)
    used_onset = False
    for p in np.nonzero(pair_differs)[0]:
        g1, g2 = int(m.pair_geom1[p]), int(m.pair_geom2[p])
        if floor not in (g1, g2):
            return None                        # only height-field pairs choose among prism contacts
        foot = g2 if g1 == floor else g1
        dep, nrm, pt = np.zeros(128), np.zeros(3 * 128), np.zeros(3 * 128)
        k = lib().oracle_hfield_contacts(om.ptr, C.byref(d), floor, foot, 128, dep.ctypes.data_as(C.POINTER(C.c_double)),
                                         nrm.ctypes.data_as(C.POINTER(C.c_double)), pt.ctypes.data_as(C.POINTER(C.c_double)))
        dep, nrm, pt = dep[:k], nrm[:3 * k].reshape(k, 3), pt[:3 * k].reshape(k, 3)
        sl = range(4 * p, 4 * p + 4)
        want = [(-gd[s] if gd[s] < 0 else None, gp[s]) for s in sl]
        # the GPU's onset-depth slots the oracle does not hold: candidates a trial may add
        extra = [s for s in sl if -onset <= gd[s] < 0 and
                 not ((np.abs(pt - gp[s]).max(axis=1) <= 1e-4) & (np.abs(dep + gd[s]) <= 2e-6)).any()]
        is_onset = dep <= onset
        found = None
        for t in range(trials):
            keep = ~is_onset | (rng.random(k) < 0.5) if t else np.ones(k, dtype=bool)
            add = [s for s in extra if t and rng.random() < 0.5]
            D = np.concatenate([dep[keep], [-gd[s] for s in add]])
            P = np.concatenate([pt[keep], gp[add].reshape(-1, 3)])
            N = np.concatenate([nrm[keep], gn[add].reshape(-1, 3)])
            if len(D) == 0:
                continue
            if t:
                D = D + rng.uniform(-2e-7, 2e-7, len(D))
                P = P + rng.uniform(-2e-5, 2e-5, P.shape)
            got = _slots_of(manifold_select(D, P, N), D, P)
            if all((w[0] is None) == (h[0] is None) and
                   (w[0] is None or (abs(w[0] - h[0]) <= 2e-6 and np.abs(w[1] - h[1]).max() <= 1e-4))
                   for w, h in zip(want, got)):
                found = (not keep.all()) or bool(add)
                break
        if found is None:
            return None
        used_onset |= found
    return "onset_selection" if used_onset else "dup_selection"


def rule_of(x: dict) -> List[str]:
    """The rules an explain() result used: one per flipped substep ("flip1e-06", "ls_floor", ...),
    plus "gpu_flip1e-07" when step_kernel's result needed the chain ensemble, or ["agree"] when every
    substep agreed to sub_tol; ["defect"] for a defect."""
    if x["kind"] != "sensitive":
        return ["defect"]
    out = [lev if isinstance(lev, str) else f"flip{lev:.0e}" for _, lev in x.get("flips", [])]
    if "gpu_flip" in x:
        out.append(f"gpu_flip{x['gpu_flip'][0]:.0e}")
    return out or ["agree"]


def gpu_chain_ensemble(env, e: int, x: np.ndarray, rel: float, seed: int = 0) -> np.ndarray:
    """The physics kernel's chain of env.n_substeps single substeps from x in every column at once:
    column 0 unperturbed, the others with x's state perturbed by a random relative rel (and 1e-3
    rel absolute), all with env e's DR record. Returns [num_envs, trace width] final states."""
    m, n, dev = env.mj_model, env.num_envs, env.device
    rng = np.random.default_rng(seed)
    k = m.nq + 2 * m.nv
    X = np.tile(x[:, None], (1, n))
    X[:k, 1:] *= 1 + rel * rng.choice([-1.0, 1.0], size=(k, n - 1))
    X[:k, 1:] += 1e-3 * rel * rng.choice([-1.0, 1.0], size=(k, n - 1))
    q, v, w, c = _split(m, X)
    T = lambda y: torch.tensor(y.astype(np.float32), device=dev).contiguous()  # noqa: E731
    tq, tv, tw, tc = T(q), T(v), T(w), T(c)
    saved = env.dr
    try:
        if saved is not None:
            env.dr = saved.view(-1, n)[:, e:e + 1].expand(-1, n).contiguous().view(-1)
        for _ in range(env.n_substeps):
            env.physics_step(tq, tv, tw, tc, 1)
        torch.cuda.synchronize()
    finally:
        env.dr = saved
    return np.concatenate([tq.cpu().numpy(), tv.cpu().numpy(), tw.cpu().numpy(), tc.cpu().numpy()]).astype(np.float64).T


def explain(rep: Report, t: int, e: int, sub_tol: float = 1e-4, seed: int = 0) -> dict:
    """Why env e differs after env-step t. The GPU replays the env-step as a chain of single
    substeps (physics_kernel) from the oracle's substep-0 input, each from its own previous output;
    at every substep the oracle takes the same substep from the GPU's (fp32) input. If every substep
    agrees to sub_tol (or the GPU's result is a branch a 1e-6/1e-5 input perturbation of the oracle
    also takes), the physics kernel is right at every state it visited. That explains step_kernel's
    outlier only if the chain lands where step_kernel did (a different code object: its substeps
    are inlined): the chain's final state must be closer to step_kernel's output than a quarter of
    step_kernel's distance from the oracle (and within 1e-3). Then the env-step difference is the
    oracle's own sensitivity to fp32-sized input differences, amplified over the 10 substeps:
    "sensitive". Otherwise "defect". Needs keep_states=True."""
    env = rep.env
    m = env.mj_model
    om, tr = substep_trace(rep, e, t)
    rng = np.random.default_rng(seed)
    x = tr[0].astype(np.float32).astype(np.float64)
    per, flips, details = [], [], {}
    for s in range(env.n_substeps):
        g = gpu_substep(env, e, x)
        r = oracle_substep(om, x)
        err = _state_rel(m, g, r)
        per.append(err)
        if err > sub_tol:
            lev = flip_level(om, x, g, rng)
            if lev is None:
                why = declared_difference(env, e, om, x, g, sub_tol, info=details.setdefault(s, {}))
                if why is None:
                    return {"kind": "defect", "substep": s, "substep_err": per}
                lev = why
            flips.append((s, lev))
        x = g
    chain_vs_oracle = _state_rel(m, x, tr[-1])
    # step_kernel's own result for this env-step (qpos, qvel, qacc_warmstart; ctrl as traced)
    L, n = env._layout, env.num_envs
    G = rep.post[t].reshape(L.nfloat, n)[:, e]
    o = L.off
    step_out = np.concatenate([G[o["qpos"]:o["qpos"] + m.nq], G[o["qvel"]:o["qvel"] + m.nv],
                               G[o["qacc_warmstart"]:o["qacc_warmstart"] + m.nv], tr[-1, m.nq + 2 * m.nv:]])
    chain_vs_step = _state_rel(m, x, step_out)
    step_vs_oracle = _state_rel(m, step_out, tr[-1])
    res = {"substep_err": per, "flips": flips, "chain_vs_oracle": chain_vs_oracle, "chain_vs_step": chain_vs_step,
           "step_vs_oracle": step_vs_oracle, "details": {k: v for k, v in details.items() if v}}
    bar = min(0.25 * step_vs_oracle, 1e-3)
    if chain_vs_step > bar:
        # the two code objects round differently (step_kernel inlines the substeps): step_kernel's
        # result is still the physics kernel's own at this state if a fp32-sized perturbation of the
        # chain's input lands there (the GPU-side counterpart of flip_level)
        x0 = tr[0].astype(np.float32).astype(np.float64)
        for lev in (1e-7, 1e-6):
            ens = gpu_chain_ensemble(env, e, x0, lev, seed)
            d = np.array([_state_rel(m, y, step_out) for y in ens[1:]])
            res["gpu_flip"] = (lev, int((d <= bar).sum()), len(d))
            if (d <= bar).any():
                return {"kind": "sensitive", **res}
        return {"kind": "defect", "substep": "step_kernel != physics_kernel chain", **res}
    return {"kind": "sensitive", **res}
