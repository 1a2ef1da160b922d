"""Known-answer physics on the HIP kernels: the same experiments and bars as the oracle's
(tests/test_oracle_kat.py, tests/kat_checks.py), through duck_physics_step. The slope and
conservative scenes are edited MJCF scenes compiled into their own kernels (native.model_library),
including the 30-iteration Newton solve of the slope scenes."""

import pytest

from open_duck_playground_amd import constants
from tests import kat
from tests.kat_checks import (check_backlash_stop, check_energy, check_resting_penetration, check_slope_slide,
                              check_slope_stick, check_stiction, model_path)

pytestmark = pytest.mark.gpu


def test_slope_sticks_below_friction_angle(gpu):
    check_slope_stick(kat.GpuBackend(model_path("slope_stick_converged"), gpu))


def test_slope_slides_above_friction_angle(gpu):
    r, a_fit, a_pred = check_slope_slide(kat.GpuBackend(model_path("slope_slide_converged"), gpu))
    print(f"slide acceleration {a_fit:.4f} m/s^2 (closed form {a_pred:.4f})")


def test_stiction_band(gpu):
    check_stiction(kat.GpuBackend(constants.task_to_xml("flat_terrain"), gpu))


def test_backlash_hinges_rest_on_their_stops(gpu):
    check_backlash_stop(kat.GpuBackend(constants.task_to_xml("flat_terrain_backlash"), gpu))


def test_resting_penetration_carries_the_weight(gpu):
    w = check_resting_penetration(kat.GpuBackend(constants.task_to_xml("flat_terrain"), gpu))
    print(f"weight carried by the reported depths: {w:.4f} m g")


def test_energy_of_a_conservative_robot(gpu):
    check_energy(kat.GpuBackend(model_path("flat_terrain_conservative"), gpu))
