#!/usr/bin/env python3
"""Per-stage cost of the step kernel by doubling (tools/gpu_stage_pmc.sh).

--build: compile build/libduck_d<k>[_<variant>].so (DUCK_DOUBLE = k, one scene variant) and the same
variant without a doubled stage (build/libduck_stage_base[_<variant>].so), on the CPU.
--report DIR: for each doubled build, the difference to the base build of the launch time (bench.py's
HIP events) and of the SQ counters per launch (rocprofv3, quad-cycles for *_CYCLES / WAIT / ACTIVE):
that is the stage's own cost, including the waits its instructions carry.
"""

import argparse
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STAGES = {1: "crb", 2: "collision", 3: "make_rows", 4: "smooth_acc (qacc_smooth factor + solves)",
          5: "solve (warm start + Newton + line search)", 6: "kinematics", 7: "com_pos", 8: "rne + smooth",
          11: "hf SAT pass 2", 12: "hf SAT pass 1", 13: "hf contact point", 14: "hf screen",
          15: "hf vertical-edge pairs", 16: "hf setup (frames, hull vertices, box, sub-grid, side minima)",
          17: "hf silhouette lists", 18: "hf survivor descriptors", 19: "hf manifold slots + contact stores", 20: "hf hull-face axes", 21: "warm start", 22: "Newton direction (gradient, J'DJ, factor + solves)"}


def build(variant, stages):
    sys.path.insert(0, ROOT)
    from open_duck_playground_amd import native
    sfx = "" if variant == "flat" else "_" + variant  # (tools/gpu_stage_pmc.sh SUFFIX)
    print(native.debug_library("stage_base" + sfx, ["DUCK_STAGE_BASE"], variants=(variant,)))
    for k in stages:
        print(native.debug_library(f"d{k}{sfx}", [f"DUCK_DOUBLE={k}"], variants=(variant,)))


def counters(d):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "step_kernel" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def report(out):
    rows = {}
    for f in sorted(glob.glob(f"{out}/bench_*.json")):
        v = os.path.basename(f)[6:-5]
        b = json.load(open(f))
        c = counters(f"{out}/pmc_{v}")
        rows[v] = dict(ms=b["roofline"]["kernel_ms"], **c)
    base = rows["base"]
    waves = base["SQ_WAVES"]
    # per wave and launch: quad-cycles -> cycles (x4), instructions per wave
    def per_wave(r, k, scale=1.0):
        return r[k] * scale / r["SQ_WAVES"]
    lines = [f"per-stage cost by doubling ({out}); per wave and launch: wave cycles, VALU-active cycles, "
             "waiting cycles (any counter / LDS instructions), VALU and LDS instructions",
             f"base: kernel {base['ms']:.4f} ms, {waves:.0f} waves, wave cycles {per_wave(base, 'SQ_WAVE_CYCLES', 4):.0f}, "
             f"VALU-active {per_wave(base, 'SQ_ACTIVE_INST_VALU', 4):.0f}, wait any {per_wave(base, 'SQ_WAIT_ANY', 4):.0f}, "
             f"wait LDS {per_wave(base, 'SQ_WAIT_INST_LDS', 4):.0f}, VALU insts {per_wave(base, 'SQ_INSTS_VALU'):.0f}, "
             f"LDS insts {per_wave(base, 'SQ_INSTS_LDS'):.0f}",
             f"{'stage':44s} {'ms':>8s} {'share':>6s} {'cycles':>8s} {'valu_cyc':>8s} {'wait':>8s} {'waitLDS':>8s} "
             f"{'valu':>7s} {'lds':>6s} {'wait/cyc':>8s}"]
    res = {"base": base, "stages": {}}
    for v, r in rows.items():
        if v == "base":
            continue
        d = {k: per_wave(r, k, 4) - per_wave(base, k, 4) for k in
             ("SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_LDS")}
        d.update({k: per_wave(r, k) - per_wave(base, k) for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS")})
        dms = r["ms"] - base["ms"]
        name = STAGES.get(int(v), v)
        res["stages"][name] = dict(d_ms=dms, share=dms / base["ms"], **d)
        lines.append(f"{name:44s} {dms:8.4f} {dms / base['ms']:6.1%} {d['SQ_WAVE_CYCLES']:8.0f} "
                     f"{d['SQ_ACTIVE_INST_VALU']:8.0f} {d['SQ_WAIT_ANY']:8.0f} {d['SQ_WAIT_INST_LDS']:8.0f} "
                     f"{d['SQ_INSTS_VALU']:7.0f} {d['SQ_INSTS_LDS']:6.0f} "
                     f"{d['SQ_WAIT_ANY'] / max(d['SQ_WAVE_CYCLES'], 1.0):8.2f}")
    txt = "\n".join(lines)
    print(txt)
    open(f"{out}/summary.txt", "w").write(txt + "\n")
    json.dump(res, open(f"{out}/summary.json", "w"), indent=1)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--variant", default="flat")
    ap.add_argument("--stages", type=int, nargs="*", default=[1, 2, 3, 4, 5, 6, 7, 8])
    ap.add_argument("--report")
    a = ap.parse_args()
    if a.build:
        build(a.variant, a.stages)
    if a.report:
        report(a.report)
