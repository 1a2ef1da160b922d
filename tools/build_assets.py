#!/usr/bin/env python3
"""Compile the reference's MJCF scenes and reference-motion table into committed assets.

Runs in the build container only (it reads /root/reference, which does not exist on the
GPU box). Outputs:
  open_duck_playground_amd/assets/<task>.npz        compiled model per task
  open_duck_playground_amd/assets/polynomial_coefficients.npz   baked imitation table

Tasks follow constants.task_to_xml (playground/open_duck_mini_v2/constants.py:28-34).
"rough_terrain" points at a file the reference does not ship (constants.py:23); it is
composed here from the rough-terrain scene's floor + the non-backlash robot (declared in
DESIGN.md).
"""

import os
import re
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import numpy as np  # noqa: E402

from open_duck_playground_amd.mjcf import compile_mjcf  # noqa: E402
from open_duck_playground_amd.refmotion import bake_table, read_poly_pkl  # noqa: E402

REF = "/root/reference/playground/open_duck_mini_v2"
OUT = os.path.join(os.path.dirname(__file__), "..", "open_duck_playground_amd", "assets")

TASKS = {
    "flat_terrain": "scene_flat_terrain.xml",
    "flat_terrain_backlash": "scene_flat_terrain_backlash.xml",
    "rough_terrain_backlash": "scene_rough_terrain_backlash.xml",
}


def composed_rough_scene(tmpdir: str) -> str:
    xmls = os.path.join(REF, "xmls")
    rough = open(os.path.join(xmls, "scene_rough_terrain_backlash.xml")).read()
    flat = open(os.path.join(xmls, "scene_flat_terrain.xml")).read()
    rough = rough.replace('file="open_duck_mini_v2_backlash.xml"', f'file="{xmls}/open_duck_mini_v2.xml"')
    rough = rough.replace('file="assets/hfield.png"', f'file="{xmls}/assets/hfield.png"')
    key_flat = re.search(r"<keyframe>.*?</keyframe>", flat, re.S).group(0)
    rough = re.sub(r"<keyframe>.*?</keyframe>", key_flat, rough, flags=re.S)
    path = os.path.join(tmpdir, "scene_rough_terrain_composed.xml")
    with open(path, "w") as f:
        f.write(rough)
    return path


# Edited scenes for tests (tests/golden/models/): what a user of the reference does when they change
# the MJCF. Each is (robot-XML substitutions, scene-XML substitutions); the model compiler and
# native.model_library turn them into kernels with no hand edits (codegen.py).
SLOPE_MU = 0.2                        # floor friction of the slope scenes
SLOPE_STICK, SLOPE_SLIDE = 0.15, 0.40  # tan(slope) below / above the friction angle atan(0.2)
CONVERGED = ('<option iterations="1" ls_iterations="5">', '<option iterations="30" ls_iterations="30">')


def _slope(tan_theta: float) -> str:
    """gravity tilted about x: the same as a floor sloping down towards +y by atan(tan_theta)"""
    th = np.arctan(tan_theta)
    return f'<option gravity="0 {9.81 * np.sin(th):.17g} {-9.81 * np.cos(th):.17g}"/>'


_INC = '<include file="open_duck_mini_v2.xml"/>'
EDITED = {
    # a stiffer servo, an 8 % larger collision foot and a grippier floor
    "flat_terrain_edited": ([('<position kp="13.37"', '<position kp="16.0"'),
                             ('<mesh file="foot_bottom_tpu.stl"/>', '<mesh file="foot_bottom_tpu.stl" scale="1.08 1.08 1.08"/>')],
                            [('friction="0.6"', 'friction="0.8"')]),
    # a slippery slope below / above the friction angle, solved to convergence (30 Newton iterations)
    "slope_stick_converged": ([CONVERGED], [('friction="0.6"', f'friction="{SLOPE_MU}"'), (_INC, _INC + _slope(SLOPE_STICK))]),
    "slope_slide_converged": ([CONVERGED], [('friction="0.6"', f'friction="{SLOPE_MU}"'), (_INC, _INC + _slope(SLOPE_SLIDE))]),
    # no joint damping, no dof friction, no servo: a conservative articulated body in flight
    "flat_terrain_conservative": ([('damping="0.56" frictionloss="0.068"', 'damping="0" frictionloss="0"'),
                                   ('<position kp="13.37"', '<position kp="0"')], []),
}


def edited_scene(tmpdir: str, robot_edits, scene_edits) -> str:
    xmls = os.path.join(REF, "xmls")
    robot = open(os.path.join(xmls, "open_duck_mini_v2.xml")).read()
    for a, b in robot_edits:
        assert a in robot, a
        robot = robot.replace(a, b)
    robot = robot.replace('meshdir="assets"', f'meshdir="{xmls}/assets"')
    scene = open(os.path.join(xmls, "scene_flat_terrain.xml")).read()
    for a, b in scene_edits:
        assert a in scene, a
        scene = scene.replace(a, b)
    with open(os.path.join(tmpdir, "open_duck_mini_v2.xml"), "w") as f:
        f.write(robot)
    path = os.path.join(tmpdir, "scene.xml")
    with open(path, "w") as f:
        f.write(scene)
    return path


def build_edited(out_dir: str):
    os.makedirs(out_dir, exist_ok=True)
    for name, (re_, se) in EDITED.items():
        with tempfile.TemporaryDirectory() as td:
            m = compile_mjcf(edited_scene(td, re_, se), timestep=0.002)
        m.save(os.path.join(out_dir, f"{name}.npz"))
        print(name, m.nq, m.nv, m.nu, list(m.opt_gravity))


def main():
    os.makedirs(OUT, exist_ok=True)
    models = {}
    for task, fname in TASKS.items():
        models[task] = compile_mjcf(os.path.join(REF, "xmls", fname), timestep=0.002)
    with tempfile.TemporaryDirectory() as td:
        # the composed scene includes robot files by absolute path; meshdir resolves from them
        path = composed_rough_scene(td)
        models["rough_terrain"] = compile_mjcf(path, timestep=0.002, asset_dir=os.path.join(REF, "xmls"))
    for task, m in models.items():
        m.save(os.path.join(OUT, f"{task}.npz"))
        print(task, m.nq, m.nv, m.nu, m.ngeom, m.nsensordata)
    table = bake_table(read_poly_pkl(os.path.join(REF, "data", "polynomial_coefficients.pkl")))
    np.savez_compressed(os.path.join(OUT, "polynomial_coefficients.npz"), **table)
    print("refmotion", table["coeffs"].shape)
    build_edited(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "models"))


if __name__ == "__main__":
    main()
