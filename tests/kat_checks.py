"""Assertions of the known-answer experiments (tests/kat.py), shared by the oracle tests
(tests/test_oracle_kat.py) and the HIP tests (tests/test_gpu_kat.py): the same bars for both."""

import os

import numpy as np

from open_duck_playground_amd import constants
from open_duck_playground_amd.mjcf import Model
from tests import kat

MODELS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "models")
F_LOSS = 0.068  # dof frictionloss of the sts3215 class (open_duck_mini_v2.xml:47)


def model_path(name: str) -> str:
    return os.path.join(MODELS, f"{name}.npz")


def _slope_geometry(m):
    g = np.asarray(m.opt_gravity)
    th = np.arctan2(abs(g[1]), -g[2])
    return th, float(m.pair_friction[1][0])


def check_slope_stick(backend):
    m = backend.m
    th, mu = _slope_geometry(m)
    assert np.tan(th) < mu
    r = kat.slope(backend)
    late = r[r[:, 0] >= 0.45]
    assert np.abs(late[:, 1]).max() < 0.01, late[:, 1]                       # at rest (creep < 1 cm/s)
    np.testing.assert_allclose(late[:, 2], np.tan(th), rtol=0.02)             # F_t / F_n = tan(theta)
    np.testing.assert_allclose(late[:, 3], np.cos(th), rtol=0.02)             # F_n = m g cos(theta)
    return r


def check_slope_slide(backend):
    m = backend.m
    th, mu = _slope_geometry(m)
    assert np.tan(th) > mu
    r = kat.slope(backend)
    a_pred = kat.G * (np.sin(th) - mu * np.cos(th))
    t, v = r[:, 0], r[:, 1]
    sel = t >= 0.3
    a_fit = np.polyfit(t[sel], v[sel], 1)[0]
    assert abs(a_fit - a_pred) < 0.1 * a_pred, (a_fit, a_pred)               # g (sin - mu cos)
    loaded = r[:, 3] > 0.3                                                   # feet carrying the robot
    assert loaded.sum() >= 5
    np.testing.assert_allclose(r[loaded, 2], mu, rtol=0.03)                  # F_t / F_n = mu while sliding
    return r, a_fit, a_pred


def check_stiction(backend):
    """Every preload ends at rest inside the stiction band |kp (ctrl - q)| <= frictionloss; a
    preload above frictionloss moves the joint at least (tau - F) / kp."""
    taus = np.array([0.5, 0.8, 1.5, 3.0, 6.0]) * F_LOSS
    for act in (3, 6, 11):   # left knee, neck pitch, right hip pitch
        dqkp, qd, kp = kat.stiction(backend, act, taus)
        resid = taus - dqkp                                                  # servo torque at rest
        assert np.all(np.abs(resid) <= 1.05 * F_LOSS), (act, resid / F_LOSS)
        assert np.all(np.abs(qd) < 0.01), qd
        above = taus > F_LOSS
        assert np.all(dqkp[above] >= 0.95 * (taus[above] - F_LOSS)), dqkp / F_LOSS


def check_backlash_stop(backend):
    """Standing on the floor, the loaded backlash hinges sit at their +-0.00873 rad stops, no further
    than the limit's solimp width (0.001 rad) beyond them."""
    m = backend.m
    q, v, qa, dist = kat.settle(backend)
    names = m.names["jnt"]
    bl = [j for j, nm in enumerate(names) if nm.endswith("_backlash")]
    qb = np.abs(q[[m.jnt_qposadr[j] for j in bl]])
    lim = m.jnt_range[bl][:, 1]
    width = m.jnt_solimp[bl][:, 2]
    assert np.all(qb <= lim + width), qb - lim
    assert (qb >= lim - 2e-4).sum() >= 8, qb - lim                           # loaded hinges at the stop
    return qb - lim


def check_resting_penetration(backend):
    """At rest the reported contact depths carry the robot's weight through the impedance law."""
    q, v, qa, dist = kat.settle(backend)
    assert np.abs(v).max() < 0.02
    assert (dist < 0).sum() >= 3
    w = kat.resting_weight_from_depths(backend.m, dist)
    assert abs(w - 1.0) < 0.02, w
    return w


def check_energy(backend):
    """Conservative robot in flight: E(t) - E(0) = -n m g^2 dt^2 / 2 (semi-implicit Euler's exact
    energy error for the centre of mass in uniform gravity) and nothing else, to 1e-2 J."""
    m = backend.m
    E, q = kat.flight_energy(backend)
    n = np.arange(len(E)) * 25
    euler = n * 0.5 * m.body_mass.sum() * kat.G ** 2 * m.opt_timestep ** 2
    drift = E - E[0]
    np.testing.assert_allclose(drift[-1], -euler[-1], rtol=0.05)
    assert np.abs(drift + euler).max() < 1e-2, np.abs(drift + euler).max()


def flat():
    return Model.load(constants.task_to_xml("flat_terrain"))
