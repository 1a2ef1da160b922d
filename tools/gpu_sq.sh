#!/bin/bash
# SQ issue/wait counters of step_kernel (two PMC passes, each its own run).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1)); rm -rf $OUT/sq$i
  timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/sq$i -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-budget 0 > /dev/null 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob("gpurun_out/sq*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "step_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
