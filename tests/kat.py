"""Known-answer physics experiments on the robot, run on either backend (oracle or HIP kernels).

Test infrastructure. Each experiment poses a situation with a closed-form answer, drives the
engine with it, and measures the result with tools independent of the engine's own dynamics
code (tests/physics_laws.py: momenta and energies from body positions only):

* slope (Coulomb friction): on a floor with friction mu sloping by theta, a robot
  at rest sticks when tan(theta) < mu -- the floor then carries F_t / F_n = tan(theta) -- and
  slides when tan(theta) > mu with centre-of-mass acceleration g (sin(theta) - mu cos(theta)) and
  F_t / F_n = mu (pyramidal cone, sliding along a cone edge)
* stiction band (dof frictionloss 0.068 Nm, open_duck_mini_v2.xml:47): a servo preloaded with
  torque tau on a joint of a robot in flight comes to rest where |kp (ctrl - q)| <= frictionloss
* backlash stop (open_duck_mini_v2_backlash.xml:53-56): servo torque drives the backlash hinges
  into their +-0.00873 rad limits, where the soft limit holds them within the solimp width
* penetration (solref (0.02, 1), solimp (0.9, 0.95, 0.001, 0.5, 2)): at rest on the flat floor
  every contact edge row carries f = k d(r)^2 |r| / ((1 - d(r)) A), so the depths the engine
  reports must add up to the robot's weight through the documented impedance law
* energy: without damping, friction or servos, a robot in flight conserves kinetic + potential
  energy up to the O(dt) oscillation of semi-implicit Euler
"""

from __future__ import annotations

import numpy as np

from open_duck_playground_amd.mjcf import Model
from tests.physics_laws import _qmat, body_frames, path_qpos

G = 9.81


# ----------------------------------------------------------------------------------------------
# measurement (positions only)
# ----------------------------------------------------------------------------------------------

def _body_motion(m: Model, qpos, qvel, qacc, t, delta=1e-5):
    c0, R0 = body_frames(m, path_qpos(m, qpos, qvel, qacc, t))
    cp, Rp = body_frames(m, path_qpos(m, qpos, qvel, qacc, t + delta))
    cm, Rm = body_frames(m, path_qpos(m, qpos, qvel, qacc, t - delta))
    vel = (cp - cm) / (2 * delta)
    W = (Rp - Rm) / (2 * delta) @ np.swapaxes(R0, -1, -2)
    om = 0.5 * np.stack([W[..., 2, 1] - W[..., 1, 2], W[..., 0, 2] - W[..., 2, 0], W[..., 1, 0] - W[..., 0, 1]], -1)
    return c0, R0, vel, om


def com_velocity(m: Model, qpos, qvel):
    _, _, vel, _ = _body_motion(m, qpos, qvel, np.zeros_like(qvel), 0.0)
    return np.einsum("b,nbi->ni", m.body_mass, vel) / m.body_mass.sum()


def external_force(m: Model, qpos, qvel, qacc, eps=1e-3):
    """Total force on the robot besides gravity, dP/dt - m g ([n, 3]): the floor's contact force.
    Fourth-order central differences of the momentum along q(t) = q (+) (v t + a t^2 / 2)."""
    w = {-2: 1.0, -1: -8.0, 1: 8.0, 2: -1.0}
    dP = 0.0
    for k, c in w.items():
        _, _, vel, _ = _body_motion(m, qpos, qvel, qacc, k * eps)
        dP = dP + c * np.einsum("b,nbi->ni", m.body_mass, vel)
    return dP / (12 * eps) - m.body_mass.sum() * np.asarray(m.opt_gravity)[None]


def energy(m: Model, qpos, qvel):
    """Kinetic + gravitational potential energy from body positions only ([n])."""
    c, R, vel, om = _body_motion(m, qpos, qvel, np.zeros_like(qvel), 0.0)
    Iw = R @ (m.body_inertia[None, :, :, None] * np.swapaxes(R, -1, -2))
    ke = 0.5 * (m.body_mass[None] * (vel ** 2).sum(-1)).sum(1) + 0.5 * np.einsum("nbi,nbij,nbj->n", om, Iw, om)
    pe = -np.einsum("b,nbi,i->n", m.body_mass, c, np.asarray(m.opt_gravity))
    return ke + pe


# ----------------------------------------------------------------------------------------------
# backends: batched [n, k] states in, [n, k] states out
# ----------------------------------------------------------------------------------------------

class OracleBackend:
    def __init__(self, m: Model):
        from tests.oracle_ffi import OracleModel
        self.m = m
        self.om = OracleModel(m)

    def run(self, qpos, qvel, warm, ctrl, nsub):
        """nsub substeps from each state; returns (qpos, qvel, warm, qacc of a forward at the end,
        contact distances of that forward)."""
        m = self.m
        out = [np.zeros_like(qpos), np.zeros_like(qvel), np.zeros_like(warm), np.zeros_like(qvel),
               np.zeros((len(qpos), 4 * m.npair))]
        for e in range(len(qpos)):
            d = self.om.new_data(qpos=qpos[e], qvel=qvel[e], ctrl=ctrl[e], warm=warm[e])
            if nsub:
                self.om.step(d, nsub)
            self.om.forward(d)
            out[0][e], out[1][e] = d.arr("qpos", m.nq), d.arr("qvel", m.nv)
            out[2][e], out[3][e] = d.arr("qacc_warmstart", m.nv), d.arr("qacc", m.nv)
            out[4][e] = d.arr("con_dist", 4 * m.npair)
        return out


class GpuBackend:
    def __init__(self, m_or_task, device="cuda:0"):
        import torch
        from open_duck_playground_amd.joystick import Joystick
        self.torch = torch
        task = m_or_task
        self.env = Joystick(task, num_envs=1, device=device, use_imitation=False)
        self.m = self.env.mj_model
        self.device = device

    def run(self, qpos, qvel, warm, ctrl, nsub):
        from tests.helpers import parse_aux
        torch, m, n = self.torch, self.m, len(qpos)
        T = lambda a: torch.tensor(np.ascontiguousarray(a.T), dtype=torch.float32, device=self.device)  # noqa: E731
        tq, tv, tw, tc = T(qpos), T(qvel), T(warm), T(ctrl)
        if nsub:
            self.env.physics_step(tq, tv, tw, tc, nsub)
        aux = torch.zeros(self.env.aux_size() * n, dtype=torch.float32, device=self.device).view(-1, n)
        self.env.physics_step(tq, tv, tw, tc, 0, aux)  # mjx.forward at the end state
        torch.cuda.synchronize()
        g = parse_aux(m, aux.cpu().numpy().astype(np.float64))
        back = lambda t: t.cpu().numpy().T.astype(np.float64)  # noqa: E731
        return [back(tq), back(tv), back(tw), g["qacc"], g["con_dist"]]


def home(m: Model, n: int = 1):
    k = m.names["key"].index("home")
    return np.tile(m.key_qpos[k], (n, 1)), np.zeros((n, m.nv)), np.tile(m.key_ctrl[k], (n, 1))


def actuator_maps(m: Model):
    return (np.array([m.jnt_qposadr[j] for j in m.actuator_trnid]),
            np.array([m.jnt_dofadr[j] for j in m.actuator_trnid]))


# ----------------------------------------------------------------------------------------------
# experiments
# ----------------------------------------------------------------------------------------------

def slope(backend, chunks=20, chunk=25):
    """Robot released at the home pose on the model's slope (gravity tilted about x, floor friction
    mu). Returns times, com velocity along the slope, floor force ratio F_t/F_n and F_n / (m g)."""
    m = backend.m
    q, v, c = home(m)
    w = np.zeros_like(v)
    g = np.asarray(m.opt_gravity)
    down = np.array([0.0, np.sign(g[1]) or 1.0, 0.0])
    rows = []
    for k in range(chunks):
        q, v, w, qa, _ = backend.run(q, v, w, c, chunk)
        F = external_force(m, q, v, qa)[0]
        vc = com_velocity(m, q, v)[0]
        rows.append(((k + 1) * chunk * m.opt_timestep, vc @ down, np.hypot(F[0], F[1]) / max(F[2], 1e-9),
                     F[2] / (m.body_mass.sum() * np.linalg.norm(g))))
    return np.array(rows)


def stiction(backend, act: int, taus, nsub=150):
    """Robot in flight at the home pose, every servo at its joint's position except actuator `act`,
    preloaded by tau (ctrl = q + tau / kp). Returns the joint displacement times kp per tau and the
    final joint speed."""
    m = backend.m
    qadr, dadr = actuator_maps(m)
    n = len(taus)
    q, v, c = home(m, n)
    q[:, 2] = 3.0
    c = q[:, qadr].copy()
    kp = float(m.actuator_kp[act])
    c[:, act] += np.asarray(taus) / kp
    q1, v1, _, _, _ = backend.run(q, v, np.zeros_like(v), c, nsub)
    return (q1[:, qadr[act]] - q[:, qadr[act]]) * kp, v1[:, dadr[act]], kp


def backlash_stop(backend, tau=1.0, nsub=100):
    """Robot in flight; every leg servo preloaded by +tau. Returns backlash joint positions [n_bl]
    and speeds, and the joint range."""
    m = backend.m
    qadr, _ = actuator_maps(m)
    q, v, c = home(m)
    q[:, 2] = 3.0
    c = q[:, qadr].copy()
    names = m.names["jnt"]
    legs = [a for a, j in enumerate(m.actuator_trnid) if (names[j] + "_backlash") in names]
    c[0, legs] += tau / m.actuator_kp[legs]
    bl = [names.index(names[m.actuator_trnid[a]] + "_backlash") for a in legs]
    q1, v1, _, _, _ = backend.run(q, v, np.zeros_like(v), c, nsub)
    qa = np.array([m.jnt_qposadr[j] for j in bl])
    da = np.array([m.jnt_dofadr[j] for j in bl])
    return q1[0, qa], v1[0, da], m.jnt_range[bl]


def impedance(m: Model, pos, solref, solimp):
    """MuJoCo's documented impedance law (mj_makeImpedance): stiffness K, damping B and d(r)."""
    timeconst, dampratio = max(solref[0], 2 * m.opt_timestep), solref[1]
    dmin, dmax, width, mid, power = solimp
    K = 1.0 / (dmax ** 2 * timeconst ** 2 * dampratio ** 2)
    B = 2.0 / (dmax * timeconst)
    x = np.minimum(np.abs(pos) / width, 1.0)
    y = np.where(x < mid, x ** power / mid ** (power - 1), 1 - (1 - x) ** power / (1 - mid) ** (power - 1))
    return K, B, dmin + y * (dmax - dmin)


def resting_weight_from_depths(m: Model, dist):
    """Sum over active contacts of the normal force the impedance law assigns to a contact at rest
    with depth r: 4 edge rows, each f = K d^2 |r| / ((1 - d) A) with the pyramidal edge's diagonal
    A = 2 mu^2 (1 + mu^2) w_foot / impratio (w_foot: the foot body's translational invweight0;
    MJX _instantiate_contact). Returned in units of the robot's weight m g."""
    total = 0.0
    for p in range(m.npair):
        mu = float(m.pair_friction[p][0])
        b1, b2 = m.geom_bodyid[m.pair_geom1[p]], m.geom_bodyid[m.pair_geom2[p]]
        w = m.body_invweight0[b1][0] + m.body_invweight0[b2][0]
        A = 2 * mu * mu * (1 + mu * mu) * w / m.opt_impratio
        r = dist[4 * p:4 * p + 4] - m.pair_margin[p]
        r = r[r < 0]
        K, _, d = impedance(m, r, m.pair_solref[p], m.pair_solimp[p])
        total += (4 * K * d * d * np.abs(r) / ((1 - d) * A)).sum()
    return total / (m.body_mass.sum() * np.linalg.norm(m.opt_gravity))


def settle(backend, seconds=1.5, chunk=250):
    m = backend.m
    q, v, c = home(m)
    w = np.zeros_like(v)
    for _ in range(int(round(seconds / (chunk * m.opt_timestep)))):
        q, v, w, qa, dist = backend.run(q, v, w, c, chunk)
    return q[0], v[0], qa[0], dist[0]


def flight_energy(backend, seconds=1.0, chunk=25, seed=0, vel=2.0):
    """Robot in flight (no contacts, joints inside their ranges) with random velocities; energy at
    every chunk boundary."""
    m = backend.m
    rng = np.random.default_rng(seed)
    q, v, c = home(m)
    q[:, 2] = 20.0                   # no floor contact within the second
    v = rng.uniform(-vel, vel, v.shape)
    v[:, 6:] *= 0.3                  # joints stay well inside their ranges over a second
    w = np.zeros_like(v)
    E = [energy(m, q, v)[0]]
    for _ in range(int(round(seconds / (chunk * m.opt_timestep)))):
        q, v, w, _, _ = backend.run(q, v, w, c, chunk)
        E.append(energy(m, q, v)[0])
    return np.array(E), q


__all__ = ["OracleBackend", "GpuBackend", "slope", "stiction", "backlash_stop", "settle",
           "resting_weight_from_depths", "flight_energy", "impedance", "external_force", "com_velocity",
           "energy", "_qmat"]
