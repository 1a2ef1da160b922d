#!/bin/bash
# rocprofv3 kernel trace of PPO training updates (tools/ppo_throughput.py): per-kernel time of the
# rollout and the learner. usage: bash tools/gpu_ppo_prof.sh [tag]
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T=${1:-ppo}
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_$T -o prof -- python3 $GRAFT_REPO_ROOT/tools/ppo_throughput.py --updates 2 > $GRAFT_REPO_ROOT/$OUT/prof_$T.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$OUT/prof_$T.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $OUT/prof_$T -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms")
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:8.2f} ms {int(r["Calls"]):7d} calls {float(r["AverageNs"])/1e3:8.2f} us  {r["Name"][:90]}')
PY
