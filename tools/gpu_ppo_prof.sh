#!/bin/bash
# Kernel-level profile of the PPO outer loop (tools/ppo_throughput.py), for the learner's cost split.
set -o pipefail
OUT=gpurun_out/ppo_prof; rm -rf $OUT; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/ppo_throughput.py --updates 3 > $OUT/plain.json 2>&1 || { tail $OUT/plain.json; exit 1; }
cat $OUT/plain.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/ppo_throughput.py --updates 2 > $OUT/prof.json 2>&1 || { tail $OUT/prof.json; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/ppo_prof/trace/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total kernel ms", tot / 1e6, "kernels", sum(int(r["Calls"]) for r in rows))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print("%8.2f ms %6d calls %7.1f us  %s" % (float(r["TotalDurationNs"]) / 1e6, int(r["Calls"]), float(r["AverageNs"]) / 1e3, r["Name"][:110]))
PY
