#!/usr/bin/env python3
"""Summarise a tools/gpu_pmc.sh run: step_kernel's average duration (kernel trace), FETCH_SIZE /
WRITE_SIZE and SQ counters per dispatch, and the library they were measured on (duck_build_id).

usage: pmc_summary.py OUT_DIR TAG CONFIG   -> OUT_DIR/<TAG>_pmc_<config>.json, _stats.csv
"""

import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(d):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "step_kernel" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    out, tag, cfg = sys.argv[1], sys.argv[2], sys.argv[3]
    stats = glob.glob(f"{out}/trace/**/*kernel_stats.csv", recursive=True)[0]
    avg_ns = None
    for r in csv.DictReader(open(stats)):
        if "step_kernel" in r["Name"]:
            avg_ns = float(r["AverageNs"])
    c = {}
    for d in ("fetch", "write", "sq1", "sq2"):
        c.update(counters(f"{out}/{d}"))
    sys.path.insert(0, ROOT)
    from open_duck_playground_amd.native import lib
    res = {
        "config": cfg, "kernel": "step_kernel", "build_id": lib().duck_build_id().decode(),
        "kernel_avg_ns": avg_ns,
        "fetch_kb": c["FETCH_SIZE"], "write_kb": c["WRITE_SIZE"],
        "hbm_bytes_per_launch": (c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0,
        "hbm_note": "raw FETCH_SIZE + WRITE_SIZE; the guide's x2 FETCH_SIZE correction is calibrated for 16 B/lane "
                    "streaming reads, not these 4 B/lane SoA rows",
        "SQ_INSTS_VALU": c["SQ_INSTS_VALU"],
        "valu_busy_frac": c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"],
        "waitcnt_frac": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
        "lds_busy_frac": c["SQ_ACTIVE_INST_LDS"] / c["SQ_WAVE_CYCLES"],
        "salu_frac": c["SQ_INST_CYCLES_SALU"] / c["SQ_WAVE_CYCLES"],
        "lds_bank_conflict_frac": c["SQ_LDS_BANK_CONFLICT"] / c["SQ_WAVE_CYCLES"],
        "valu_insts_per_wave": c["SQ_INSTS_VALU"] / c["SQ_WAVES"],
        "raw": c,
    }
    base = os.path.join(out, f"{tag}_pmc_{cfg.lower()}")  # copied into profiles/ from gpurun_out
    json.dump(res, open(base + ".json", "w"), indent=1)
    shutil.copy(stats, base + "_stats.csv")
    print(json.dumps({k: v for k, v in res.items() if k != "raw"}, indent=1))


if __name__ == "__main__":
    main()
