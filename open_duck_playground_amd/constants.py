"""Constants for Open Duck Mini V2 (mirror of playground/open_duck_mini_v2/constants.py).

Scene selection returns compiled-model asset paths instead of XML paths: the MJCF is
compiled once in the build container (``tools/build_assets.py``) because the reference
tree is not present where the env runs.
"""

import os

ROOT_PATH = os.path.dirname(os.path.abspath(__file__))
ASSETS = os.path.join(ROOT_PATH, "assets")
FLAT_TERRAIN = os.path.join(ASSETS, "flat_terrain.npz")
ROUGH_TERRAIN = os.path.join(ASSETS, "rough_terrain.npz")
FLAT_TERRAIN_BACKLASH = os.path.join(ASSETS, "flat_terrain_backlash.npz")
ROUGH_TERRAIN_BACKLASH = os.path.join(ASSETS, "rough_terrain_backlash.npz")
POLY_COEFFICIENTS = os.path.join(ASSETS, "polynomial_coefficients.npz")


def task_to_xml(task_name: str) -> str:
    """Same keys as constants.task_to_xml (constants.py:28-34); returns the compiled model.

    A path to an MJCF scene (``.xml``) or a compiled model (``.npz``) is returned as is: the env
    compiles it and, if no shipped kernel matches it, the kernels for it (native.model_library)."""
    if task_name.endswith((".xml", ".npz")):
        return task_name
    return {
        "flat_terrain": FLAT_TERRAIN,
        "rough_terrain": ROUGH_TERRAIN,
        "flat_terrain_backlash": FLAT_TERRAIN_BACKLASH,
        "rough_terrain_backlash": ROUGH_TERRAIN_BACKLASH,
    }[task_name]


FEET_SITES = ["left_foot", "right_foot"]
LEFT_FEET_GEOMS = ["left_foot_bottom_tpu"]
RIGHT_FEET_GEOMS = ["right_foot_bottom_tpu"]
HIP_JOINT_NAMES = ["left_hip_yaw", "left_hip_roll", "left_hip_pitch", "right_hip_yaw", "right_hip_roll",
                   "right_hip_pitch"]
KNEE_JOINT_NAMES = ["left_knee", "right_knee"]
JOINTS_ORDER_NO_HEAD = ["left_hip_yaw", "left_hip_roll", "left_hip_pitch", "left_knee", "left_ankle",
                        "right_hip_yaw", "right_hip_roll", "right_hip_pitch", "right_knee", "right_ankle"]
FEET_GEOMS = LEFT_FEET_GEOMS + RIGHT_FEET_GEOMS
FEET_POS_SENSOR = [f"{site}_pos" for site in FEET_SITES]
ROOT_BODY = "trunk_assembly"
GRAVITY_SENSOR = "upvector"
GLOBAL_LINVEL_SENSOR = "global_linvel"
GLOBAL_ANGVEL_SENSOR = "global_angvel"
LOCAL_LINVEL_SENSOR = "local_linvel"
ACCELEROMETER_SENSOR = "accelerometer"
GYRO_SENSOR = "gyro"
