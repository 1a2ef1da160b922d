"""Known-answer physics on the fp64 oracle (tests/kat.py, tests/kat_checks.py). The HIP kernels
pass the same checks in tests/test_gpu_kat.py.

The friction-cone checks use scenes solved to convergence (30 Newton iterations): with the
reference's single Newton iteration (open_duck_mini_v2.xml:6) the implied contact force of a sliding
robot is not on the cone (measured in tests/test_oracle_kat.py::test_single_iteration_slide_is_off_cone)."""

import numpy as np

from open_duck_playground_amd import constants
from open_duck_playground_amd.mjcf import Model
from tests import kat
from tests.kat_checks import (check_backlash_stop, check_energy, check_resting_penetration, check_slope_slide,
                              check_slope_stick, check_stiction, flat, model_path)


def _oracle(name):
    return kat.OracleBackend(Model.load(model_path(name)))


def test_slope_sticks_below_friction_angle():
    check_slope_stick(_oracle("slope_stick_converged"))


def test_slope_slides_above_friction_angle():
    check_slope_slide(_oracle("slope_slide_converged"))


def test_stiction_band():
    check_stiction(kat.OracleBackend(flat()))


def test_backlash_hinges_rest_on_their_stops():
    check_backlash_stop(kat.OracleBackend(Model.load(constants.task_to_xml("flat_terrain_backlash"))))


def test_resting_penetration_carries_the_weight():
    check_resting_penetration(kat.OracleBackend(flat()))


def test_energy_of_a_conservative_robot():
    check_energy(_oracle("flat_terrain_conservative"))


def test_single_iteration_slide_is_off_cone():
    """The reference's solver settings (1 Newton iteration, 5 line-search steps) on the slide slope:
    the robot still slides, but the floor force implied by qacc leaves the friction cone while the
    feet bounce (F_t / F_n well above mu), which a converged solve never does."""
    m = Model.load(model_path("slope_slide_converged"))
    m.arrays["opt_iterations"], m.arrays["opt_ls_iterations"] = np.array(1), np.array(5)
    r = kat.slope(kat.OracleBackend(m))
    mu = float(m.pair_friction[1][0])
    loaded = r[:, 3] > 0.3
    assert r[-1, 1] > 0.2                                   # it slides
    assert r[loaded, 2].max() > 1.2 * mu                    # but not on the cone
