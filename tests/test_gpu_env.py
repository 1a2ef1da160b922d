"""GPU env parity: Joystick.reset/step in libduck.so vs the oracle's restatement.

Same seeds -> same threefry streams, so obs noise, action delays, pushes and commands
match draw for draw. Obs/priv/reward are compared within fp32 tolerances; done flags and
integer bookkeeping exactly (for envs whose physics stayed within tolerance).
"""

import numpy as np
import pytest
import torch

from open_duck_playground_amd.config import default_config, env_config_struct
from open_duck_playground_amd.joystick import Joystick, domain_randomize, wrap_for_brax_training
from tests.oracle_ffi import OracleBatch, OracleModel

pytestmark = pytest.mark.gpu


def _compare(env, st, ob, L, tol_obs=2e-3, frac=0.95):
    obs = st.obs["state"].cpu().numpy().astype(np.float64)
    priv = st.obs["privileged_state"].cpu().numpy().astype(np.float64)
    err = np.abs(obs - ob.obs).max(axis=1) / (1 + np.abs(ob.obs).max(axis=1))
    errp = np.abs(priv - ob.priv).max(axis=1) / (1 + np.abs(ob.priv).max(axis=1))
    good = (err < tol_obs) & (errp < tol_obs * 10)
    assert good.mean() >= frac, (good.mean(), np.sort(err)[-5:], np.sort(errp)[-5:])
    rew = st.reward.cpu().numpy()
    assert np.allclose(rew[good], ob.rew[good], rtol=1e-3, atol=1e-3)
    assert np.array_equal(st.done.cpu().numpy()[good], ob.done[good])
    ist = st.istate.view(L.nint, -1).cpu().numpy()
    oist = ob.is_.reshape(L.nint, -1)
    for name in ("rng_key", "rng_ctr", "push_step", "push_interval"):
        k = L.ioff[name]
        assert np.array_equal(ist[k][good], oist[k][good]), name
    return good


@pytest.mark.parametrize("task,imit", [("flat_terrain", False), ("flat_terrain", True), ("flat_terrain_backlash", True)])
def test_reset_step_parity(task, imit, gpu):
    n = 100  # not a multiple of the 16-lane workgroup
    env = Joystick(task, num_envs=n, device=gpu, use_imitation=imit)
    st = env.reset(rng=7)
    om = OracleModel(env.mj_model)
    cfg = env_config_struct(env.mj_model, default_config(), imit)
    ob = OracleBatch(om, cfg, n)
    ob.reset(seed=7)
    L = env._layout
    good = _compare(env, st, ob, L)
    rng = np.random.default_rng(0)
    for t in range(5):
        a = rng.uniform(-1, 1, (n, env.action_size)).astype(np.float32)
        st = env.step(st, torch.tensor(a, device=gpu))
        ob.step(a.astype(np.float64))
        good &= _compare(env, st, ob, L)
    assert good.mean() > 0.9


@pytest.mark.parametrize("task", ["flat_terrain", "flat_terrain_backlash"])
def test_standing_reset_step_parity(task, gpu):
    """Standing (standing.py) through the same kernels, task switch on: obs 85 / priv 153."""
    from open_duck_playground_amd.config import standing_default_config
    from open_duck_playground_amd.standing import Standing
    n = 100
    env = Standing(task, num_envs=n, device=gpu)
    assert env.observation_size == {"state": (85,), "privileged_state": (153,)}
    st = env.reset(rng=11)
    cfg = env_config_struct(env.mj_model, standing_default_config(), False, task=1)
    ob = OracleBatch(OracleModel(env.mj_model), cfg, n)
    ob.reset(seed=11)
    L = env._layout
    good = _compare(env, st, ob, L)
    rng = np.random.default_rng(1)
    for t in range(5):
        a = rng.uniform(-1, 1, (n, env.action_size)).astype(np.float32)
        st = env.step(st, torch.tensor(a, device=gpu))
        ob.step(a.astype(np.float64))
        good &= _compare(env, st, ob, L)
    assert good.mean() > 0.9
    assert set(st.metrics) == {"cost/orientation", "cost/torques", "cost/action_rate", "reward/alive",
                               "cost/stand_still", "cost/head_pos", "swing_peak"}


def test_autoreset_and_episode(gpu):
    n = 64
    env = wrap_for_brax_training(Joystick("flat_terrain", num_envs=n, device=gpu, use_imitation=False),
                                 episode_length=5)
    st = env.reset(rng=3)
    first_obs = st.obs["state"].clone()
    for t in range(5):
        st = env.step(st, torch.zeros(n, env.action_size, device=gpu))
    torch.cuda.synchronize()
    # episode_length reached: every env is done and restored to its first state
    assert torch.all(st.done == 1)
    assert torch.allclose(st.obs["state"], first_obs)
    assert torch.all(st.info["steps"] == 5)
    st = env.step(st, torch.zeros(n, env.action_size, device=gpu))
    assert torch.all(st.info["steps"] == 1)


@pytest.mark.parametrize("task", ["flat_terrain", "rough_terrain", "rough_terrain_backlash"])
def test_domain_randomization_parity(task, gpu):
    """C4 (rough + DR) and C5's per-GPU shard (rough + DR + backlash) against the oracle."""
    n = 48
    env = Joystick(task, num_envs=n, device=gpu, use_imitation=False)
    dr = domain_randomize(env, rng=11)
    st = env.reset(rng=5)
    base = OracleModel(env.mj_model)
    models = [OracleModel(env.mj_model, dr=base.dr_sample(11, e)) for e in range(n)]
    # the GPU DR record must match the oracle's sampling of the same streams
    D = dr.view(-1, n).cpu().numpy().T
    ref = np.array([base.dr_sample(11, e) for e in range(n)])
    np.testing.assert_allclose(D, ref, rtol=1e-5, atol=1e-6)
    cfg = env_config_struct(env.mj_model, default_config(), False, domain_randomize=True)
    ob = OracleBatch(models, cfg, n)
    ob.reset(seed=5)
    L = env._layout
    good = _compare(env, st, ob, L)
    rng = np.random.default_rng(1)
    for t in range(3):
        a = rng.uniform(-1, 1, (n, env.action_size)).astype(np.float32)
        st = env.step(st, torch.tensor(a, device=gpu))
        ob.step(a.astype(np.float64))
        good &= _compare(env, st, ob, L)
    print(task, "free-running envs within tolerance after 3 steps:", good.mean())
    assert good.mean() > 0.9


def test_edge_sizes(gpu):
    for n in (1, 17):
        env = Joystick("flat_terrain", num_envs=n, device=gpu, use_imitation=False)
        st = env.reset(rng=1)
        st = env.step(st, torch.zeros(n, env.action_size, device=gpu))
        torch.cuda.synchronize()
        assert torch.isfinite(st.obs["state"]).all()


def test_host_action_is_moved(gpu):
    env = Joystick("flat_terrain", num_envs=4, device=gpu, use_imitation=False)
    st = env.reset(rng=1)
    out = env.step(st, torch.zeros(4, env.action_size), inplace=True)  # host tensor is moved to the device
    assert out is st


def test_env_offset_shards_are_bit_identical(gpu):
    """Two shards (env_offset 0 and 24) reproduce one 48-env batch exactly (global env ids)."""
    n, h = 48, 24
    rng = np.random.default_rng(3)
    acts = [torch.tensor(rng.uniform(-1, 1, (n, 14)).astype(np.float32), device=gpu) for _ in range(3)]
    full = Joystick("flat_terrain", num_envs=n, device=gpu, use_imitation=True)
    sf = full.reset(rng=9)
    parts = [Joystick("flat_terrain", num_envs=h, device=gpu, use_imitation=True, env_offset=k * h) for k in range(2)]
    sp = [p.reset(rng=9) for p in parts]
    for a in acts:
        sf = full.step(sf, a)
        for k in range(2):
            sp[k] = parts[k].step(sp[k], a[k * h:(k + 1) * h])
    for key in ("state", "privileged_state"):
        got = torch.cat([s.obs[key] for s in sp])
        assert torch.equal(got, sf.obs[key]), key
    assert torch.equal(torch.cat([s.reward for s in sp]), sf.reward)


@pytest.mark.parametrize("cfg", ["C2", "C3", "C4", "C5"])
def test_full_size_runs_are_deterministic(cfg, gpu):
    """At the bench's sizes (C2 4096 flat, C3 4096 flat + imitation, C4 8192 rough + DR, C5 4096
    rough + DR + backlash), two
    runs from the same seeds give bit-identical obs, privileged obs, rewards and dones: no races
    between the team's lanes or the workgroup's staging, no order-dependent reductions."""
    from bench import CONFIGS
    c = CONFIGS[cfg]
    n = c["envs"]
    g = torch.Generator(device=gpu)
    g.manual_seed(5)
    acts = [torch.rand(n, 14, device=gpu, generator=g) * 2 - 1 for _ in range(6)]
    out = []
    for run in range(2):
        env = wrap_for_brax_training(Joystick(c["task"], num_envs=n, device=gpu, use_imitation=c["imitation"]),
                                     episode_length=1000, randomization_fn=domain_randomize if c["dr"] else None)
        st = env.reset(rng=3)
        for a in acts:
            st = env.step(st, a)
        torch.cuda.synchronize()
        out.append([st.obs["state"].clone(), st.obs["privileged_state"].clone(), st.reward.clone(), st.done.clone()])
    for x, y in zip(*out):
        assert torch.equal(x, y)


@pytest.mark.parametrize("cfg,n,mode", [("C2", 512, "latency"), ("C3", 1021, "latency"), ("C4", 1024, "latency"),
                                        ("C5", 510, "latency"), ("C2", 2048, "paired"), ("C3", 1021, "paired"),
                                        ("C4", 2044, "paired"), ("C5", 2048, "paired"), ("C2", 2048, "latency_x2"),
                                        ("C3", 1021, "latency_x2")])
def test_latency_mode_matches_throughput_mode(cfg, n, mode, gpu):
    """The latency kernel (each substep's stages split over four waves per 4 envs, DUCK_STEP_LATENCY)
    and the paired latency kernel (the stages over a pair of waves per 4 envs, 8 envs per workgroup,
    DUCK_STEP_PAIRED) run the same stage code on the same data as the throughput kernel (one team per
    env). Every env-step is taken by both kernels from the same state (the throughput kernel's), over
    auto-resets (5-step episodes), DR, and a batch with a partial workgroup (n % 4 != 0): fstate, obs,
    privileged obs, reward, istate and done equal bit for bit in every scene (round 4 had the flat
    scenes at fp32 rounding: FMAs formed across contact_jx's statements differed between the fused and
    the split warm start; contact_jx now contracts within expressions only). No cross-wave wait gave up."""
    from bench import CONFIGS
    c = CONFIGS[cfg]
    g = torch.Generator(device=gpu)
    g.manual_seed(11)
    envs = {}
    for m in ("throughput", mode):
        env = wrap_for_brax_training(Joystick(c["task"], num_envs=n, device=gpu, use_imitation=c["imitation"]),
                                     episode_length=5, randomization_fn=domain_randomize if c["dr"] else None)
        env.set_step_mode(m)
        assert env.step_kernel == m
        env.lat_timeouts(reset=True)
        envs["latency" if m == mode else m] = env
    st = envs["throughput"].reset(rng=4)
    for t in range(8):
        a = torch.rand(n, 14, device=gpu, generator=g) * 2 - 1
        s_t = envs["throughput"].step(st, a)
        s_l = envs["latency"].step(st, a)
        torch.cuda.synchronize()
        assert torch.equal(s_t.istate, s_l.istate) and torch.equal(s_t.done, s_l.done), t
        for x, y in ((s_t.fstate, s_l.fstate), (s_t.obs["state"], s_l.obs["state"]),
                     (s_t.obs["privileged_state"], s_l.obs["privileged_state"]), (s_t.reward, s_l.reward)):
            assert torch.equal(x, y), (t, (x != y).sum().item())
        st = s_t
    assert envs["latency"].lat_timeouts() == 0


@pytest.mark.parametrize("mode,wg_envs", [("latency", 4), ("paired", 8), ("latency_x2", 4)])
def test_latency_timeout_surfaces(mode, wg_envs, gpu, monkeypatch):
    """A latency-kernel launch whose cross-wave wait gives up is not silent: the test build
    (native.debug_library "force_timeout", -DDUCK_LAT_FORCE_TIMEOUT: in workgroup 1 the waits for the
    M event never see it and give up after a few polls) sets the handle's sticky device error word,
    writes NaN qpos for workgroup 1's envs (4..7 in the latency kernel, 8..15 in the paired one) and
    only those, and the next step raises DuckError (DUCK_EDEVICE) until the word is cleared. The
    shipped library's word stays 0 over the same steps."""
    import os
    from open_duck_playground_amd import joystick as jmod
    from open_duck_playground_amd.native import BUILD, DuckError
    path = os.path.join(BUILD, "libduck_force_timeout.so")
    assert os.path.exists(path), "built by __graft_entry__.build()"
    n = 4 * wg_envs
    ok = Joystick("flat_terrain", num_envs=n, device=gpu, use_imitation=False)
    ok.set_step_mode(mode)
    st = ok.reset(rng=1)
    for _ in range(2):
        st = ok.step(st, torch.zeros(n, 14, device=gpu))
    torch.cuda.synchronize()
    assert ok.device_error() == 0
    monkeypatch.setattr(jmod, "model_library", lambda m: path)
    env = Joystick("flat_terrain", num_envs=n, device=gpu, use_imitation=False)
    env.set_step_mode(mode)
    st = env.reset(rng=1)
    st = env.step(st, torch.zeros(n, 14, device=gpu))
    torch.cuda.synchronize()
    assert env.device_error() == 1          # DUCK_DEVERR_LAT_TIMEOUT
    L = env._layout
    q = st.fstate.view(L.nfloat, n)[L.off["qpos"]:L.off["qpos"] + env.mj_model.nq]
    bad = torch.isnan(q).any(dim=0).cpu().numpy()
    w = wg_envs
    assert bad[w:2 * w].all() and not bad[:w].any() and not bad[2 * w:].any(), bad
    with pytest.raises(DuckError, match="device error word"):
        env.step(st, torch.zeros(n, 14, device=gpu))
    assert env.device_error(clear=True) == 1 and env.device_error() == 0
    env.reset(rng=2)                         # usable again once cleared


def test_step_mode_auto_selects_by_batch(gpu):
    """AUTO: the latency kernel while the batch leaves a CU per 4 envs, the paired latency kernel while
    it leaves a CU per 8, the throughput kernel above."""
    ncu = torch.cuda.get_device_properties(gpu).multi_processor_count
    for task, mid in (("flat_terrain", "latency_x2"), ("rough_terrain", "paired"), ("rough_terrain_backlash", "paired"),
                      ("flat_terrain_backlash", "paired")):
        for n, want in ((4 * ncu, "latency"), (4 * ncu + 1, mid), (8 * ncu, mid), (8 * ncu + 1, "throughput")):
            env = Joystick(task, num_envs=n, device=gpu, use_imitation=False)
            assert env.step_kernel == want, (task, n, ncu)
    # a mode the model is not compiled for is refused (LATENCY_X2 exists for the plane floor without backlash)
    from open_duck_playground_amd.native import DuckError
    with pytest.raises(DuckError, match="not compiled for this model"):
        Joystick("rough_terrain", num_envs=64, device=gpu, use_imitation=False).set_step_mode("latency_x2")


def test_full_size_long_rollout_with_auto_reset(gpu):
    """4096 envs x 300 env-steps of U(-1,1) actions with a 100-step episode limit: every row stays
    finite and the EpisodeWrapper/AutoReset bookkeeping holds for every env: an env is done at the
    latest on its 100th step since its last reset, truncation marks exactly those, falls are the
    other dones (BraxAutoResetWrapper semantics, common/runner.py:117)."""
    n = 4096
    env = wrap_for_brax_training(Joystick("flat_terrain", num_envs=n, device=gpu, use_imitation=False),
                                 episode_length=100)
    st = env.reset(rng=0)
    g = torch.Generator(device=gpu)
    g.manual_seed(1234)
    ep = torch.zeros(n, device=gpu)
    falls = truncs = 0
    for t in range(300):
        st = env.step(st, torch.rand(n, 14, device=gpu, generator=g) * 2 - 1)
        ep += 1
        done, trunc = st.done, st.info["truncation"]
        assert bool((trunc <= done).all())
        assert bool(((ep >= 100) <= (done == 1)).all())          # nobody runs past the limit
        assert bool(((trunc == 1) <= (ep == 100)).all())         # truncation only at the limit
        falls += int((done - trunc).sum().item())
        truncs += int(trunc.sum().item())
        ep = torch.where(done == 1, torch.zeros_like(ep), ep)
        if t % 50 == 49:
            assert torch.isfinite(st.obs["state"]).all() and torch.isfinite(st.obs["privileged_state"]).all()
    assert truncs > 0 and falls > 0


def test_c5_full_shape_equals_eight_shards(gpu):
    """C5's full shape on one GPU: 32,768 envs of rough terrain + DR + backlash with the training
    wrappers (EpisodeWrapper at 2 env-steps + AutoReset, so the restore path runs) against the same
    batch as 8 shards of 4,096 (env_offset = k * 4096, what each of the 8 ranks runs): per-env DR,
    reset, pushes and steps are keyed by the global env id (randomize.py:26-146), so obs,
    privileged obs, reward and done are bit-identical at each of 3 env-steps."""
    from open_duck_playground_amd.joystick import domain_randomize, wrap_for_brax_training
    n, k = 32768, 8
    h = n // k
    g = torch.Generator(device=gpu)
    g.manual_seed(11)
    acts = [torch.rand(n, 14, device=gpu, generator=g) * 2 - 1 for _ in range(3)]

    def make(num, off):
        env = Joystick("rough_terrain_backlash", num_envs=num, device=gpu, use_imitation=False, env_offset=off)
        return wrap_for_brax_training(env, episode_length=2, randomization_fn=domain_randomize, rng=4)

    keys = ("state", "privileged_state", "reward", "done")
    pick = lambda st: [st.obs["state"], st.obs["privileged_state"], st.reward, st.done]  # noqa: E731
    full = make(n, 0)
    sf = full.reset(rng=9)
    ref = []
    for a in acts:
        sf = full.step(sf, a)
        ref.append([x.clone() for x in pick(sf)])
    del full, sf
    got = [[[] for _ in keys] for _ in acts]
    for s in range(k):
        part = make(h, s * h)
        sp = part.reset(rng=9)
        for t, a in enumerate(acts):
            sp = part.step(sp, a[s * h:(s + 1) * h])
            for j, x in enumerate(pick(sp)):
                got[t][j].append(x.clone())
        del part, sp
    assert float(ref[1][3].sum()) > n // 2  # episode_length 2: the envs truncate at step 2, then restore
    for t in range(len(acts)):
        for j, key in enumerate(keys):
            assert torch.equal(torch.cat(got[t][j]), ref[t][j]), (t, key)


def test_step_is_functional(gpu):
    """Joystick.step returns a new State and leaves its input as it was (the reference's
    state.replace, joystick.py:480-481; brax's unroll keeps both state and nstate), and the new
    State equals the in-place step bit for bit."""
    n = 64
    env = wrap_for_brax_training(Joystick("rough_terrain", num_envs=n, device=gpu, use_imitation=False),
                                 episode_length=2, randomization_fn=domain_randomize, rng=3)
    s0 = env.reset(rng=5)
    a = torch.rand(n, env.action_size, device=gpu) * 2 - 1
    keep = {"obs": s0.obs["state"].clone(), "priv": s0.obs["privileged_state"].clone(),
            "qpos": s0.data.qpos.clone(), "fstate": s0.fstate.clone(), "istate": s0.istate.clone()}
    s1 = env.step(s0, a)
    s2 = env.step(s1, a)  # the auto-reset restore (episode_length 2)
    torch.cuda.synchronize()
    assert s1 is not s0 and s1.fstate.data_ptr() != s0.fstate.data_ptr()
    assert torch.equal(s0.obs["state"], keep["obs"]) and torch.equal(s0.obs["privileged_state"], keep["priv"])
    assert torch.equal(s0.data.qpos, keep["qpos"])
    assert torch.equal(s0.fstate, keep["fstate"]) and torch.equal(s0.istate, keep["istate"])
    # in place from a copy of s0: bit-identical to the functional chain
    t = env.step(s0, torch.zeros_like(a))  # any State in fresh buffers
    t.fstate.copy_(keep["fstate"])
    t.istate.copy_(keep["istate"])
    for _ in range(2):
        out = env.step(t, a, inplace=True)
        assert out is t
    for key in ("state", "privileged_state"):
        assert torch.equal(t.obs[key], s2.obs[key]), key
    assert torch.equal(t.fstate, s2.fstate) and torch.equal(t.istate, s2.istate)
    assert torch.equal(t.reward, s2.reward) and torch.equal(t.done, s2.done)
    assert torch.equal(s1.data.qpos, env.step(s0, a).data.qpos)  # s0 still steps to s1
