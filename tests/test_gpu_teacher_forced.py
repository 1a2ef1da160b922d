"""Strict env parity: every env-step of libduck.so from the oracle's own (fp32-rounded) state.

See tests/teacher_forcing.py. Each case steps 256 envs for 6 env-steps; before every step the
oracle's state is uploaded into the GPU state, so each comparison is one Joystick.step
(joystick.py:323-481: action delay, push, 10 substeps, obs, rewards, termination, info
bookkeeping, and the EpisodeWrapper/AutoReset wrappers of common/runner.py:117 where on).

Bar: qpos rel 1e-4, qvel 2e-3, qacc_warmstart 2e-2, every info field / obs / privileged obs / reward
2e-3 (|gpu - oracle| / (1 + |oracle|)), done and every integer field exact, for >= 99.5 % of
env-steps; and every env-step outside that bar is explained at substep resolution (the kernel's
substep from its own input matches the oracle's substep from the same input to 1e-4, or is a
branch the oracle also takes under a 1e-6/1e-5 input perturbation; and that substep chain
reproduces step_kernel's own result for the env-step). The reset before step 0 is compared
strictly: every fstate row (incl. the auto-reset snapshot), obs, privileged obs and istate word of
every env at the same bar (teacher_forcing.reset_stats), >= 99.5 % of envs, the rest explained as a
contact branch of the reset's forward (explain_reset). Every case prints how many outliers each
explanation rule accepted ("rules:"; teacher_forcing.rule_of), and test_explain_has_teeth shows the
classifier says "defect" when the oracle is handed a deliberately wrong model (teacher_forcing.DEFECTS).
Measured on MI355X (profiles/r04_gpu_tests.log): median errors 1e-7 (qpos) .. 9e-6 (obs), a handful of
outliers per 1536 env-steps, all explained.
"""
from collections import Counter

import numpy as np
import pytest

from tests.teacher_forcing import CASES, DEFECTS, explain, explain_reset, nominal_agrees, oracle_knob, rule_of, run_case

pytestmark = pytest.mark.gpu


def _check(case, rep):
    s = rep.summary()
    print(case, {k: v for k, v in s.items()})
    # the reset itself, strictly: every fstate row, obs, privileged obs and istate word of every env
    # at the same bar, >= 99.5 % of envs, and every env outside it explained (explain_reset)
    r = rep.reset
    bad = (r["norm"] > 1) | r["int_mismatch"]
    print(f"  reset: worst err/bar {r['norm'].max():.3f} ({r['worst_row'][r['norm'].argmax()]}), "
          f"outside the bar {int(bad.sum())}, int mismatches {int(r['int_mismatch'].sum())}")
    assert bad.mean() <= 0.005, [(int(e), r["worst_row"][e], float(r["norm"][e])) for e in bad.nonzero()[0][:8]]
    for e in bad.nonzero()[0]:
        x = explain_reset(rep, int(e))
        print(f"  reset outlier env {e} ({r['worst_row'][e]}, err/bar {r['norm'][e]:.1f}): {x}")
        assert x["kind"] == "sensitive", (int(e), x)
    assert s["good_frac"] >= 0.995, s
    unexplained = []
    rules = Counter()
    for t, st in enumerate(rep.steps):
        out = rep.outliers(st) | st.done_mismatch | st.int_mismatch
        for e in out.nonzero()[0]:
            x = explain(rep, t, int(e))
            print(f"  outlier step {t} env {e}: {x['kind']} max substep err {max(x['substep_err']):.2e} "
                  f"flips {x.get('flips')} gpu_flip {x.get('gpu_flip')} chain_vs_step {x.get('chain_vs_step', 0):.2e}")
            rules.update(rule_of(x))
            if x["kind"] != "sensitive":
                unexplained.append((t, int(e), x))
    print(f"  rules: {dict(sorted(rules.items()))}")
    assert not unexplained, unexplained


@pytest.mark.parametrize("case", list(CASES))
def test_teacher_forced_step_parity(case, gpu):
    _check(case, run_case(case, gpu, n=256, steps=6, keep_states=True))


@pytest.mark.parametrize("case", ["rough_dr", "rough_backlash_dr"])
def test_teacher_forced_rough_long(case, gpu):
    """The height-field scenes (C4, C5) at 1024 envs x 10 env-steps: 10,240 teacher-forced env-steps
    each, at the same bar and with every outlier explained."""
    _check(case, run_case(case, gpu, n=1024, steps=10, keep_states=True))


def test_teacher_forced_paths_are_exercised(gpu):
    """The forced cases really run the rare env paths: pushes, the step-500 command resample and
    the auto-reset restore (free-running parity never reached them)."""
    from tests.teacher_forcing import run
    rep = run("flat_terrain", False, n=64, steps=3, device=gpu, force_push=True, force_resample=True,
              keep_states=True)
    env = rep.env
    L = env._layout
    fs1 = rep.pre[1][0].reshape(L.nfloat, 64)
    is1 = rep.pre[1][1].reshape(L.nint, 64)
    push = fs1[L.off["push"]:L.off["push"] + 2]
    assert (np.abs(push).sum(axis=0) > 0).sum() >= 64 // 3 - 1       # pushed envs
    assert (is1[L.ioff["step"]] == 0).sum() >= 64 // 4               # resampled envs restart at step 0
    assert rep.summary()["good_frac"] >= 0.995
    rep = run("flat_terrain", False, n=64, steps=4, device=gpu, auto_reset=True, episode_length=3, keep_states=True)
    L = rep.env._layout
    is3 = rep.pre[3][1].reshape(L.nint, 64)
    fs3 = rep.pre[3][0].reshape(L.nfloat, 64)
    assert (fs3[L.off["done"]] == 1).all() and (is3[L.ioff["ep_steps"]] == 3).all()   # every env restored at 3
    assert rep.summary()["good_frac"] >= 0.995


@pytest.mark.parametrize("defect", list(DEFECTS))
def test_explain_has_teeth(defect, gpu):
    """The classifier can say "defect": the oracle runs a deliberately wrong model (floor friction
    x 1.02, one servo's kp x 1.005 and x 1.001, hinge damping x 1.01, contact solref x 1.02, the foot hull
    scaled by 1.0005 on the height field) or a wrong contact generation (teacher_forcing.DEFECTS' oracle
    knobs, which change only the height field's contacts: round 4's point band, the witness band x 1.5,
    the deepest-prism tie x 100, the manifold from the second-deepest prism) while the GPU runs the
    nominal one. A model defect makes every outlier a real model difference; a contact knob counts
    only the outliers it induced -- those where the oracle without the knob, from the same pre-state,
    lands inside the bars on the GPU (nominal_agrees). Such outliers must appear (>= 20 for round 4's
    model edits over 256 envs x 2 env-steps; >= 8 for the small edits (kp x 1.001, damping x 1.01) and
    the knobs over 1,024 envs x 3), and explain() must return "defect" for >= 90 % of them (up to 40
    checked; per-rule counts printed)."""
    case, edit, knob = DEFECTS[defect]
    big = defect in ("floor_friction_x1.02", "actuator_kp_x1.005", "contact_solref_x1.02", "foot_hull_x1.0005_hfield")
    n, steps, need = (256, 2, 20) if big else (1024, 3, 8)
    with oracle_knob(knob):
        rep = run_case(case, gpu, n=n, steps=steps, keep_states=True, oracle_edit=edit)
        outl = [(t, int(e)) for t, st in enumerate(rep.steps)
                for e in (rep.outliers(st) | st.done_mismatch | st.int_mismatch).nonzero()[0]]
        natural = 0
        if knob is not None:
            induced = [(t, e) for t, e in outl if nominal_agrees(rep, t, e, knob)]
            natural = len(outl) - len(induced)
            outl = induced
        assert len(outl) >= need, f"the injected defect induced only {len(outl)} outliers"
        pick = [outl[i] for i in np.linspace(0, len(outl) - 1, min(40, len(outl))).astype(int)]
        rules = Counter()
        for t, e in pick:
            rules.update(rule_of(explain(rep, t, e)))
    n_def = rules["defect"]
    print(f"{defect}: {len(outl)} induced outliers of {sum(len(s.done_mismatch) for s in rep.steps)} env-steps "
          f"({natural} others, also outliers without the defect), {len(pick)} explained: {dict(sorted(rules.items()))}")
    assert n_def >= 0.9 * len(pick), dict(rules)
