"""Known-answer and property tests of the CPU oracle (physics is not pinned by any
reference test: mujoco/mjx are absent, see DESIGN.md "Parity"). These are build-authored
analytic checks: threefry KATs, exact semi-implicit-Euler free fall, standing at rest,
reset determinism, and the auto-reset wrapper semantics (BraxAutoResetWrapper)."""

import ctypes as C
import os

import numpy as np
import pytest

from open_duck_playground_amd import constants
from open_duck_playground_amd.config import default_config, env_config_struct
from open_duck_playground_amd.mjcf import Model
from tests.oracle_ffi import OracleBatch, OracleEnv, OracleModel, lib


@pytest.fixture(scope="module")
def m():
    return Model.load(constants.task_to_xml("flat_terrain"))


@pytest.fixture(scope="module")
def om(m):
    return OracleModel(m)


@pytest.mark.parametrize("ctr,key,out", [
    ((0, 0), (0, 0), (0x6B200159, 0x99BA4EFE)),
    ((0xFFFFFFFF, 0xFFFFFFFF), (0xFFFFFFFF, 0xFFFFFFFF), (0x1CB996FC, 0xBB002BE7)),
    ((0x243F6A88, 0x85A308D3), (0x13198A2E, 0x03707344), (0xC4923A9C, 0x483DF7A0)),
])
def test_threefry_kat(ctr, key, out):
    """Random123 kat_vectors, threefry2x32 with 20 rounds."""
    k = (C.c_uint32 * 2)(*key)
    c = (C.c_uint32 * 2)(*ctr)
    o = (C.c_uint32 * 2)()
    lib().oracle_threefry2x32(k, c, o)
    assert (o[0], o[1]) == out


def _home(m):
    key = m.names["key"].index("home")
    return m.key_qpos[key].copy(), m.key_ctrl[key].copy()


def test_free_fall_is_exact_euler(m, om):
    q, _ = _home(m)
    q[2] = 5.0  # far above the floor: no contacts
    ctrl = q[7:7 + m.nu].copy()  # position servo at its target: zero actuator force
    d = om.new_data(qpos=q, qvel=np.zeros(m.nv), ctrl=ctrl)
    om.forward(d)
    qacc = d.arr("qacc", m.nv)
    g = -m.opt_gravity[2]
    np.testing.assert_allclose(qacc[2], -g, atol=1e-9)
    np.testing.assert_allclose(np.delete(qacc, 2), 0, atol=1e-9)
    n, dt = 25, m.opt_timestep
    om.step(d, n)
    qpos, qvel = d.arr("qpos", m.nq), d.arr("qvel", m.nv)
    np.testing.assert_allclose(qvel[2], -g * dt * n, rtol=1e-12)
    np.testing.assert_allclose(qpos[2], 5.0 - g * dt * dt * n * (n + 1) / 2, rtol=1e-12)
    np.testing.assert_allclose(qpos[7:], q[7:], atol=1e-12)


def test_standing_at_rest(m, om):
    q, ctrl = _home(m)
    d = om.new_data(qpos=q, qvel=np.zeros(m.nv), ctrl=ctrl)
    om.step(d, 500)  # 1 s
    qpos, qvel = d.arr("qpos", m.nq), d.arr("qvel", m.nv)
    assert 0.10 < qpos[2] < 0.20
    w, x, y, z = qpos[3:7]
    up_z = 1 - 2 * (x * x + y * y)
    assert up_z > 0.95
    assert np.abs(qvel).max() < 0.2
    assert np.isfinite(qpos).all()
    assert (d.arr("con_dist", 12) < 0.005).sum() >= 4  # both feet carry contacts


def _env(m, om, imit=False, auto_reset=False, episode_length=1000):
    cfgd = default_config()
    cfgd.episode_length = episode_length
    return OracleEnv(om, env_config_struct(m, cfgd, imit, auto_reset))


def test_reset_is_deterministic_per_env_id(m, om):
    e = _env(m, om)
    o1, p1 = e.reset(seed=3, env_id=5)
    o2, p2 = e.reset(seed=3, env_id=5)
    o3, _ = e.reset(seed=3, env_id=6)
    np.testing.assert_array_equal(o1, o2)
    np.testing.assert_array_equal(p1, p2)
    assert not np.array_equal(o1[6:13], o3[6:13])  # commands differ across envs


def test_autoreset_restores_first_state(m, om):
    e = _env(m, om, auto_reset=True, episode_length=5)
    o0, p0 = e.reset(seed=1)
    for t in range(5):
        o, p, r, done = e.step(np.zeros(m.nu))
    assert done == 1.0
    np.testing.assert_array_equal(o, o0)
    o, p, r, done = e.step(np.zeros(m.nu))
    assert done == 0.0


def test_batch_equals_single_env(m, om):
    """The OpenMP batch (SoA, stride n) gives the single-env results column by column."""
    n = 6
    cfg = env_config_struct(m, default_config(), False)
    b = OracleBatch(om, cfg, n)
    b.reset(seed=2, threads=2)
    rng = np.random.default_rng(0)
    acts = rng.uniform(-1, 1, (3, n, m.nu))
    for a in acts:
        b.step(a, threads=2)
    for env_id in (0, 4):
        e = OracleEnv(om, cfg)
        e.reset(seed=2, env_id=env_id)
        for a in acts:
            o, p, r, done = e.step(a[env_id])
        np.testing.assert_array_equal(b.obs[env_id], o)
        np.testing.assert_array_equal(b.rew[env_id], r)


def test_flat_height_field_matches_plane(m, om):
    """An all-zero height field, decomposed into prisms, touches where the z = 0 plane does: with
    each foot's deepest hull vertex 0.1-2 mm below the floor, every foot reports a contact, none
    deeper than that vertex, and mostly the deepest prism contact is that vertex through the
    prism's top face (depth equal, normal +z); the others are triangles the foot only grazes,
    whose shallowest separation is a side face or a crossing edge pair."""
    import copy
    mr = copy.deepcopy(Model.load(constants.task_to_xml("rough_terrain")))
    mr.arrays["hfield_data"] = np.zeros_like(mr.arrays["hfield_data"])
    omr = OracleModel(mr)
    hv = mr.hulls[0].vert
    floor = mr.id("geom", "floor")
    pairs = [(p, int(mr.pair_geom2[p])) for p in range(mr.npair) if int(mr.pair_geom1[p]) == floor]
    assert len(pairs) == 2
    rng = np.random.default_rng(3)
    q0, ctrl = _home(m)

    def lowest(d, g):
        x = np.ctypeslib.as_array(d.geom_xpos)[g] + hv @ np.ctypeslib.as_array(d.geom_xmat)[g].reshape(3, 3).T
        return x[:, 2].min()

    equal = total = 0
    for trial in range(24):
        q = q0.copy()
        q[0:2] += rng.uniform(-0.5, 0.5, 2)
        q[7:] += rng.uniform(-0.2, 0.2, m.nu)
        d = omr.new_data(qpos=q, qvel=np.zeros(m.nv), ctrl=ctrl)
        omr.forward(d)
        q[2] -= max(lowest(d, g) for _, g in pairs) + rng.uniform(1e-4, 2e-3)  # both feet 0.1-2 mm down
        d = omr.new_data(qpos=q, qvel=np.zeros(m.nv), ctrl=ctrl)
        omr.forward(d)
        dist = d.arr("con_dist", 4 * mr.npair)
        fr = np.ctypeslib.as_array(d.con_frame)
        for p, g in pairs:
            deep = -lowest(d, g)
            sl = dist[4 * p:4 * p + 4]
            assert deep > 0 and sl.min() < 0, (trial, p, deep, sl)
            assert -sl.min() <= deep + 1e-12
            total += 1
            k = 4 * p + int(np.argmin(sl))
            equal += abs(-sl.min() - deep) < 1e-12 and fr[k][2] > 1 - 1e-12
    assert equal >= 0.6 * total, (equal, total)


def test_height_field_contacts_follow_terrain():
    """On the rough scene, feet at rest report contacts whose normals match the terrain slope."""
    mr = Model.load(constants.task_to_xml("rough_terrain"))
    omr = OracleModel(mr)
    q, ctrl = _home(mr)
    d = omr.new_data(qpos=q, qvel=np.zeros(mr.nv), ctrl=ctrl)
    omr.step(d, 300)
    dist = d.arr("con_dist", 12)
    frames = np.ctypeslib.as_array(d.con_frame)[:12]
    active = dist[4:] < 0.002
    assert active.sum() >= 2
    normals = frames[4:][active][:, :3]
    np.testing.assert_allclose(np.linalg.norm(normals, axis=1), 1.0, atol=1e-9)
    assert (normals[:, 2] > 0.99).all()  # 1 cm relief over 7.8 cm cells: gentle slopes
    assert np.isfinite(d.arr("qpos", mr.nq)).all()


def test_standing_task_surface(m, om):
    """Standing (standing.py) on the oracle: obs 85 / privileged 153, zero initial motor targets,
    no walking command, base velocity drawn from U(+-0.5), reward = clip(sum(terms) * dt)."""
    from open_duck_playground_amd.config import standing_default_config
    n = 8
    cfg = env_config_struct(m, standing_default_config(), False, task=1)
    assert cfg.use_imitation == 0 and cfg.use_motor_speed_limits == 0 and cfg.scale_head_pos == -2.0
    b = OracleBatch(om, cfg, n)
    L = b.L
    assert (L.obs_size, L.priv_size) == (85, 153)
    b.reset(seed=5)
    F = b.fs.reshape(L.nfloat, n)
    np.testing.assert_array_equal(F[L.off["motor_targets"]:L.off["motor_targets"] + m.nu], 0.0)
    np.testing.assert_array_equal(F[L.off["command"]:L.off["command"] + 3], 0.0)
    qv = F[L.off["qvel"]:L.off["qvel"] + 6]
    assert np.abs(qv).max() <= 0.5 and np.abs(qv).max() > 0.05  # wider than the Joystick's +-0.05
    np.testing.assert_array_equal(b.obs[:, 6:9], 0.0)  # command[:3] in the state
    np.testing.assert_array_equal(b.priv[:, :85], b.obs)
    b.step(np.zeros((n, m.nu)))
    met = F[L.off["metrics"]:L.off["metrics"] + 8]
    # reward = clip((orientation + torques + action_rate + alive + stand_still + head_pos) * dt, 0, 1e4)
    terms = np.array([-met[0], -met[1], -met[2], met[3], -met[4], -met[5]])
    np.testing.assert_allclose(b.rew, np.clip(terms.sum(0) * float(np.float32(0.02)), 0, 1e4), rtol=1e-12)
    np.testing.assert_array_equal(met[3], 20.0)  # alive
    np.testing.assert_array_equal(met[5], 0.0)   # head_pos gated off: no walking command


def test_push_interval_rounding_to_zero_never_pushes(m, om):
    """interval_range below ctrl_dt / 2 rounds to a 0-step interval: jp.mod(push_step + 1, 0) is the
    dividend under XLA (joystick.py:388-390), so no push ever fires -- and nothing divides by zero."""
    cfgd = default_config()
    cfgd.push_config.interval_range = [0.0, 0.009]
    n = 8
    b = OracleBatch(om, env_config_struct(m, cfgd, False), n)
    b.reset(seed=4)
    L = b.L
    I = b.is_.reshape(L.nint, n)
    assert (I[L.ioff["push_interval"]] == 0).all()
    for _ in range(3):
        b.step(np.zeros((n, m.nu)))
        F = b.fs.reshape(L.nfloat, n)
        np.testing.assert_array_equal(F[L.off["push"]:L.off["push"] + 2], 0.0)


def test_hfield_contacts_match_brute_force_prisms():
    """the oracle's height-field contacts (MuJoCo's prism decomposition, exact
    penetration over the Minkowski-face axes, 4 slots by _manifold_points from the deepest) against
    the brute-force reference over every separating axis of every prism (oracle_hfield_prisms), on
    rough-terrain + DR env-steps: contact flags agree everywhere, the deepest contact's depth and
    normal agree to fp64 rounding (tools/hfield_deviation.py), with the declared plain weighted
    centroid and with round 4's point band (oracle_set_hf_band_scale(1), now a test aid): the point
    rule moves no depth or normal."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tools"))
    from hfield_deviation import measure
    for blend in (False, True):
        r = measure("rough_terrain", 16, 20, blend=blend)
        assert r["contact_ours"] > 100
        assert r["flag_agreement"] == 1.0, r
        assert r["depth_abs_diff_m"]["max"] < 1e-9, r
        assert r["normal_angle_deg"]["max"] < 1e-3, r
    # TPhys::collide_hfield does not test the prism's bottom-edge pairs: they never win (nor the
    # bottom face), while every other class does
    w = r["axis_wins"]
    assert w["bottom_edge"] == 0 and w["bottom"] == 0, w
    assert all(w[k] > 0 for k in ("top", "side", "hull_face", "top_edge", "vertical_edge")), w


def test_oracle_hull_hull_clipped_manifold():
    """Foot/foot contacts (oracle collide_convex_convex, mjx's clipped face manifold) of robots in
    flight whose feet touch (physics_laws.flight_states seed 7, the states of the GPU foot/foot
    test): 1-4 distinct points per touching pair, each the midpoint between a point of the incident
    face (on one foot hull's surface) and its projection on the reference plane, no deeper than
    the SAT penetration, all on the plane of the contact normal's face."""
    from tests.physics_laws import flight_states
    m = Model.load(constants.task_to_xml("flat_terrain"))
    om = OracleModel(m)
    hull = m.hulls[0]
    feet = [m.id("geom", g) for g in constants.FEET_GEOMS]
    p = [k for k in range(m.npair) if {int(m.pair_geom1[k]), int(m.pair_geom2[k])} == set(feet)][0]
    qpos, qvel, ctrl = flight_states(m, 4096, seed=7)
    touching = 0
    for e in range(len(qpos)):
        d = om.new_data(qpos=qpos[e], qvel=qvel[e], ctrl=ctrl[e])
        om.forward(d)
        dist = d.arr("con_dist", 4 * m.npair)[4 * p:4 * p + 4]
        if not (dist < 0).any():
            continue
        touching += 1
        pos = np.ctypeslib.as_array(d.con_pos)[4 * p:4 * p + 4]
        fr = np.ctypeslib.as_array(d.con_frame)[4 * p:4 * p + 4]
        act = dist < 0
        assert 1 <= act.sum() <= 4
        pts = pos[act]
        assert len(np.unique(np.round(pts, 12), axis=0)) == act.sum()
        n = fr[act][0][:3]
        assert np.allclose(fr[act][:, :3], n)
        gx = np.ctypeslib.as_array(d.geom_xpos)
        gm = np.ctypeslib.as_array(d.geom_xmat)
        for k in np.nonzero(act)[0]:
            q = pos[k] + 0.5 * dist[k] * n  # the clipped point on the incident face
            on = []
            for g in feet:
                R = gm[g].reshape(3, 3)
                v = R.T @ (q - gx[g])  # mesh frame
                on.append(np.max(hull.face_normal @ v - hull.face_offset))
            assert min(abs(x) for x in on) < 1e-9, on  # on one foot's surface
        # no point deeper than the SAT penetration (the deepest incident vertex along n)
        assert -dist[act].min() <= -dist.min() + 1e-12
    assert touching >= 10
