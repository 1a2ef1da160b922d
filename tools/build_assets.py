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


if __name__ == "__main__":
    main()
