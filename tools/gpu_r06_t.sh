#!/bin/bash
# Learner GEMM counters, pass 2: where the grouped GEMM waves spend their cycles (parked at waitcnt or barrier, issue-stalled, issuing).
set -o pipefail
OUT=gpurun_out/r06t; rm -rf $OUT; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA -d $GRAFT_REPO_ROOT/$OUT/pmc -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ppo_throughput.py --updates 1 > $GRAFT_REPO_ROOT/$OUT/pmc.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$OUT/pmc.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $OUT/pmc -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
agg = defaultdict(lambda: defaultdict(float)); cnt = defaultdict(set)
for r in rows:
    k = r["Kernel_Name"]
    if "mlp_group" not in k and "step_kernel" not in k: continue
    kk = "mlp_group" if "mlp_group" in k else "step_kernel"
    agg[kk][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[kk].add(r["Dispatch_Id"])
for k, d in agg.items():
    n = len(cnt[k])
    print(k, "dispatches", n, {c: f"{v / n:.4g}" for c, v in sorted(d.items())})
PY
rm -f $f
