#!/bin/bash
# Learner: per-launch durations with 64-wide output tiles everywhere (DUCK_MLP_BN=64) against the default
# per-launch tiles, one kernel trace each (tools/ppo_trace_summary.py).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
for v in base bn64; do
  BN=32; [ $v = bn64 ] && BN=64
  cd /tmp && DUCK_MLP_BN=$BN $T 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/r06v_$v -o tr -- python3 $GRAFT_REPO_ROOT/tools/ppo_throughput.py --updates 1 > $GRAFT_REPO_ROOT/$OUT/r06v_$v.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$OUT/r06v_$v.log; exit 1; }
  cd $GRAFT_REPO_ROOT
  f=$(find $OUT/r06v_$v -name "*kernel_trace.csv" | head -1)
  python3 tools/ppo_trace_summary.py $f > $OUT/r06v_${v}_summary.txt && head -16 $OUT/r06v_${v}_summary.txt | cut -c1-60
  rm -f $f
done
