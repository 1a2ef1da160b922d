"""The oracle's forward dynamics obey the robot's Newton-Euler laws (tests/physics_laws.py).

An independent pin of the physics restatement: momentum rates are computed from body positions
alone (finite differences along the accelerated path), so the mass matrix, bias forces,
actuation, passive forces and the solver's internal rows are all checked at once against
dP/dt = m g and dL_com/dt = 0 for robots in flight. The GPU counterpart at 4096 envs per
compiled scene is tests/test_gpu_physics.py::test_flight_obeys_newton_euler.
"""

import numpy as np
import pytest

from open_duck_playground_amd import constants
from open_duck_playground_amd.mjcf import Model
from tests.oracle_ffi import OracleModel
from tests.physics_laws import centroidal_residual, flight_states


def _oracle_qacc(m, qpos, qvel, ctrl, smooth_warm=True):
    """Forward qacc; with smooth_warm the warm start is qacc_smooth itself (see physics_laws)."""
    om = OracleModel(m)
    out = []
    for e in range(len(qpos)):
        d = om.new_data(qpos=qpos[e], qvel=qvel[e], ctrl=ctrl[e])
        om.forward(d)
        if smooth_warm:
            d = om.new_data(qpos=qpos[e], qvel=qvel[e], ctrl=ctrl[e], warm=d.arr("qacc_smooth", m.nv).copy())
            om.forward(d)
        out.append(d.arr("qacc", m.nv).copy())
    return np.array(out)


@pytest.mark.parametrize("task", ["flat_terrain", "flat_terrain_backlash"])
def test_oracle_flight_obeys_newton_euler(task):
    m = Model.load(constants.task_to_xml(task))
    qpos, qvel, ctrl = flight_states(m, 96, seed=0)
    qacc = _oracle_qacc(m, qpos, qvel, ctrl)
    assert np.abs(qacc[:, 6:]).max() > 10.0  # actuators, damping and limits are really acting
    f, mom = centroidal_residual(m, qpos, qvel, qacc)
    assert f.max() < 1e-6 and mom.max() < 1e-6, (f.max(), mom.max())


def test_oracle_foot_foot_contact_obeys_newton_euler():
    """Foot/foot contact forces are internal too: the states of flight_states(seed=7) whose
    feet touch (hull/hull SAT contact rows active) obey the laws like the rest."""
    m = Model.load(constants.task_to_xml("flat_terrain"))
    qpos, qvel, ctrl = flight_states(m, 4096, seed=7)
    om = OracleModel(m)
    touch = []
    for e in range(len(qpos)):
        d = om.new_data(qpos=qpos[e], qvel=qvel[e], ctrl=ctrl[e])
        om.forward(d)
        if (d.arr("con_dist", 4 * m.npair)[:4] < 0).any():  # pair 0 = left/right foot
            touch.append(e)
    assert len(touch) >= 10
    qacc = _oracle_qacc(m, qpos[touch], qvel[touch], ctrl[touch])
    f, mom = centroidal_residual(m, qpos[touch], qvel[touch], qacc)
    assert f.max() < 1e-6 and mom.max() < 1e-6, (f.max(), mom.max())


def test_newton_euler_check_has_teeth():
    """Perturbing a single joint acceleration by 1 % (or dropping the velocity-product terms
    by evaluating at zero velocity) is caught by orders of magnitude."""
    m = Model.load(constants.task_to_xml("flat_terrain"))
    qpos, qvel, ctrl = flight_states(m, 32, seed=1)
    qacc = _oracle_qacc(m, qpos, qvel, ctrl)
    for dof in (6, 9, 15):  # hip yaw, knee, neck pitch
        bad = qacc.copy()
        bad[:, dof] *= 1.01
        f, mom = centroidal_residual(m, qpos, qvel, bad)
        assert np.median(np.maximum(f, mom)) > 1e-5
    qacc0 = _oracle_qacc(m, qpos, np.zeros_like(qvel), ctrl)  # no Coriolis/centrifugal terms
    f, mom = centroidal_residual(m, qpos, qvel, qacc0)
    assert np.median(np.maximum(f, mom)) > 1e-4


def _exhaustive_sat(hull, p1, R1, p2, R2):
    """Best separation over every face axis and every edge-pair axis (no filter), vectorised."""
    V1, V2 = p1 + hull.vert @ R1.T, p2 + hull.vert @ R2.T
    hc = hull.vert.mean(axis=0)
    cc = (p2 + R2 @ hc) - (p1 + R1 @ hc)
    U = np.vstack([hull.face_normal @ R1.T, -(hull.face_normal @ R2.T)])
    face = ((U @ V2.T).min(1) - (U @ V1.T).max(1)).max()
    d = hull.vert[hull.edge[:, 1]] - hull.vert[hull.edge[:, 0]]
    ea, eb = d @ R1.T, d @ R2.T
    u = np.cross(ea[:, None, :], eb[None, :, :]).reshape(-1, 3)
    un = np.linalg.norm(u, axis=1)
    ok = un >= 1e-6 * np.repeat(np.linalg.norm(ea, axis=1), len(eb)) * np.tile(np.linalg.norm(eb, axis=1), len(ea))
    u = u[ok] / un[ok, None]
    u *= np.where(u @ cc < 0, -1.0, 1.0)[:, None]
    edge = ((u @ V2.T).min(1) - (u @ V1.T).max(1)).max()
    return face, edge


def test_oracle_hull_sat_minkowski_filter_keeps_the_deepest_axis():
    """The hull/hull SAT tests only edge pairs whose Gauss-map arcs cross (faces of the
    Minkowski difference) and breaks near-ties with DUCK_HULL_SAT_TIE. Against a brute-force
    SAT over all 60 face axes and all 2025 edge pairs, the contact depth it reports is the
    deepest axis's to within that tolerance, for every touching state of flight_states(7)."""
    m = Model.load(constants.task_to_xml("flat_terrain"))
    qpos, qvel, ctrl = flight_states(m, 4096, seed=7)
    om = OracleModel(m)
    g1, g2 = int(m.pair_geom1[0]), int(m.pair_geom2[0])
    hull = m.hulls[0]
    n = 0
    for e in range(len(qpos)):
        d = om.new_data(qpos=qpos[e], qvel=qvel[e], ctrl=ctrl[e])
        om.forward(d)
        dist = d.arr("con_dist", 4 * m.npair)[:4]
        if not (dist < 0).any():
            continue
        X, R = d.arr("geom_xpos", m.ngeom), d.arr("geom_xmat", m.ngeom)
        face, edge = _exhaustive_sat(hull, np.array(X[g1]), np.array(R[g1]).reshape(3, 3),
                                     np.array(X[g2]), np.array(R[g2]).reshape(3, 3))
        top = max(face, edge)
        depth = dist[dist < 0].min()  # edge axis: one point; face axis: the deepest incident vertex
        assert top - 1e-5 - 1e-12 <= depth <= top + 1e-12, (e, depth, face, edge)
        n += 1
    assert n >= 10
