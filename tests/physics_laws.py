"""Newton-Euler laws of the whole robot, measured without the engine's own dynamics code.

The physics pipeline (mjx.step restated by the oracle and the HIP kernels) has no reference
test to pin it (DESIGN.md "Parity"). This module supplies an independent, size-independent
check: for a robot in flight (no floor contact), every force the pipeline may apply besides
gravity — actuators (joint torques), joint damping, armature, dof friction loss, joint limits,
foot/foot contact — acts between bodies of the robot. So whatever qacc the engine returns,
the centroidal momentum h = (P, L_com) of the robot must obey

    dP/dt = m_total * g,        dL_com/dt = 0     (gravity has no moment about the com).

Here h is computed from body POSITIONS ONLY (a batched forward-kinematics written for this
check, vectorised over envs) along the path q(t) = q (+) (v t + a t^2 / 2), and its time
derivative is taken by finite differences: no cdof, no composite inertia, no RNE, no mass
matrix. A wrong mass matrix, bias force, actuator transmission or solver row breaks it.

One condition makes the law exact for MuJoCo's Newton solver with iterations = 1: the solve
must start from qacc_smooth. From there qacc = qs + alpha H^-1 J' f(qs) with H = M + J'DJ, and
M H^-1 J' = J' (I + D J M^-1 J')^-1, so M qacc - qfrc_smooth lies in the span of the
constraint rows (internal forces). If instead the warm start wins the start-point comparison
and the line search returns alpha != 1, the implied force has a component outside that span
(an unconverged iterate, faithful to the reference, not a physics law). The checks therefore
pass qacc_warmstart = qacc_smooth, so both start candidates coincide.
"""

import numpy as np

from open_duck_playground_amd.mjcf import Model


def _qmul(a, b):
    w1, x1, y1, z1 = np.moveaxis(a, -1, 0)
    w2, x2, y2, z2 = np.moveaxis(b, -1, 0)
    return np.stack([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2], -1)


def _qmat(q):
    q = q / np.linalg.norm(q, axis=-1, keepdims=True)
    w, x, y, z = np.moveaxis(q, -1, 0)
    return np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                     2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                     2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], -1).reshape(q.shape[:-1] + (3, 3))


def _axis_quat(axis, angle):
    """[n] angles about a fixed unit axis -> [n, 4]."""
    h = 0.5 * angle
    return np.concatenate([np.cos(h)[:, None], np.sin(h)[:, None] * np.asarray(axis)[None, :]], 1)


def _rotvec_quat(r):
    """[n, 3] rotation vectors -> [n, 4] (exact exponential map)."""
    th = np.linalg.norm(r, axis=1)
    s = np.where(th > 1e-12, np.sin(0.5 * th) / np.where(th > 1e-12, th, 1.0), 0.5)
    return np.concatenate([np.cos(0.5 * th)[:, None], s[:, None] * r], 1)


def body_frames(m: Model, qpos: np.ndarray):
    """Batched forward kinematics: qpos [n, nq] -> body com positions [n, nb, 3] and
    inertia-frame rotations [n, nb, 3, 3] (MuJoCo conventions: free joint qpos = world pos +
    quat (w,x,y,z); hinge rotates by q - qpos0 about its body-frame axis through jnt_pos)."""
    n, nb = qpos.shape[0], m.nbody
    xpos = np.zeros((n, nb, 3))
    xquat = np.zeros((n, nb, 4))
    xquat[:, 0, 0] = 1.0
    for i in range(1, nb):
        p, ja, jn = m.body_parentid[i], m.body_jntadr[i], m.body_jntnum[i]
        if jn and m.jnt_type[ja] == 0:
            a = m.jnt_qposadr[ja]
            xpos[:, i] = qpos[:, a:a + 3]
            xquat[:, i] = qpos[:, a + 3:a + 7] / np.linalg.norm(qpos[:, a + 3:a + 7], axis=1, keepdims=True)
            continue
        Rp = _qmat(xquat[:, p])
        xpos[:, i] = xpos[:, p] + Rp @ m.body_pos[i]
        q = _qmul(xquat[:, p], np.broadcast_to(m.body_quat[i], (n, 4)))
        for j in range(ja, ja + jn):
            assert m.jnt_type[j] == 3, "hinge joints only below the root"
            anchor = _qmat(q) @ m.jnt_pos[j] + xpos[:, i]
            a = m.jnt_qposadr[j]
            q = _qmul(q, _axis_quat(m.jnt_axis[j], qpos[:, a] - m.qpos0[a]))
            xpos[:, i] = anchor - _qmat(q) @ m.jnt_pos[j]
        xquat[:, i] = q
    R = _qmat(xquat)
    com = xpos + np.einsum("nbij,bj->nbi", R, m.body_ipos)
    Ri = R @ _qmat(m.body_iquat)[None]
    return com, Ri


def path_qpos(m: Model, qpos, qvel, qacc, t):
    """q(t) = q (+) (v t + a t^2/2): world-frame translation, body-frame rotation vector for
    the free joint (its qvel[3:6] is the local angular velocity), additive hinges."""
    q = qpos.copy()
    dq = qvel * t + 0.5 * qacc * t * t
    for j in range(m.njnt):
        a, d = m.jnt_qposadr[j], m.jnt_dofadr[j]
        if m.jnt_type[j] == 0:
            q[:, a:a + 3] += dq[:, d:d + 3]
            q[:, a + 3:a + 7] = _qmul(qpos[:, a + 3:a + 7], _rotvec_quat(dq[:, d + 3:d + 6]))
        else:
            q[:, a] += dq[:, d]
    return q


def _momenta(m: Model, qpos, qvel, qacc, t, delta=1e-5):
    """Per-body linear momentum and angular momentum about the robot com at time t."""
    c0, R0 = body_frames(m, path_qpos(m, qpos, qvel, qacc, t))
    cp, Rp = body_frames(m, path_qpos(m, qpos, qvel, qacc, t + delta))
    cm, Rm = body_frames(m, path_qpos(m, qpos, qvel, qacc, t - delta))
    mass = m.body_mass
    vel = (cp - cm) / (2 * delta)
    W = (Rp - Rm) / (2 * delta) @ np.swapaxes(R0, -1, -2)  # dR/dt R^T = [omega]
    om = 0.5 * np.stack([W[..., 2, 1] - W[..., 1, 2], W[..., 0, 2] - W[..., 2, 0], W[..., 1, 0] - W[..., 0, 1]], -1)
    Iw = R0 @ (m.body_inertia[None, :, :, None] * np.swapaxes(R0, -1, -2))  # R diag(I) R^T
    ctot = np.einsum("b,nbi->ni", mass, c0) / mass.sum()
    P = mass[None, :, None] * vel
    L = np.einsum("nbij,nbj->nbi", Iw, om) + np.cross(c0 - ctot[:, None], P)
    return P, L


def centroidal_residual(m: Model, qpos, qvel, qacc, eps=1e-3):
    """Relative residuals of dP/dt = m g and dL_com/dt = 0 for each env ([n] each).

    Fourth-order central differences in time (step eps) of the momenta along the path; each
    residual is normalised by the sum over bodies of the magnitudes of their own momentum
    rates (plus m|g| for the force), so 1e-6 means the laws hold to 6 digits of the
    accelerations actually present."""
    w = {-2: 1.0, -1: -8.0, 1: 8.0, 2: -1.0}
    dP = dL = 0.0
    for k, c in w.items():
        P, L = _momenta(m, qpos, qvel, qacc, k * eps)
        dP = dP + c * P
        dL = dL + c * L
    dP, dL = dP / (12 * eps), dL / (12 * eps)  # [n, nb, 3] per-body rates
    mg = m.body_mass.sum() * np.asarray(m.opt_gravity)
    fres = np.linalg.norm(dP.sum(1) - mg, axis=1) / (np.linalg.norm(dP, axis=2).sum(1) + np.linalg.norm(mg))
    mres = np.linalg.norm(dL.sum(1), axis=1) / (np.linalg.norm(dL, axis=2).sum(1) + 1e-9)
    return fres, mres


def flight_states(m: Model, n: int, seed: int, vel=1.0):
    """Random robots in flight: base 3 m up, any orientation, joints anywhere in (and
    slightly beyond) their ranges, random velocities and servo targets (actuators, limits
    and dof friction all active; feet may touch each other)."""
    rng = np.random.default_rng(seed)
    qpos = np.tile(m.qpos0, (n, 1))
    qpos[:, 2] = 3.0
    qv = rng.normal(size=(n, 4))
    qpos[:, 3:7] = qv / np.linalg.norm(qv, axis=1, keepdims=True)
    for j in range(1, m.njnt):
        a = m.jnt_qposadr[j]
        lo, hi = m.jnt_range[j] if m.jnt_limited[j] else (-1.0, 1.0)
        span = hi - lo
        qpos[:, a] = rng.uniform(lo - 0.05 * span, hi + 0.05 * span, n)
    qvel = rng.uniform(-vel, vel, (n, m.nv))
    lo, hi = m.actuator_ctrlrange[:, 0], m.actuator_ctrlrange[:, 1]
    ctrl = rng.uniform(lo, hi, (n, m.nu))
    return qpos, qvel, ctrl
