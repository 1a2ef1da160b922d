#!/bin/bash
# Learner: per-launch durations of the grouped GEMMs with 32-row tiles (build/libduck_bm32.so) against the
# shipped 64-row tiles: one kernel trace each (tools/ppo_trace_summary.py).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
for v in base bm32; do
  L=""; [ $v = bm32 ] && L=$GRAFT_REPO_ROOT/open_duck_playground_amd/build/libduck_bm32.so
  cd /tmp && DUCK_LIB=$L $T 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/r06u_$v -o tr -- python3 $GRAFT_REPO_ROOT/tools/ppo_throughput.py --updates 1 > $GRAFT_REPO_ROOT/$OUT/r06u_$v.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$OUT/r06u_$v.log; exit 1; }
  cd $GRAFT_REPO_ROOT
  f=$(find $OUT/r06u_$v -name "*kernel_trace.csv" | head -1)
  python3 tools/ppo_trace_summary.py $f > $OUT/r06u_${v}_summary.txt && head -17 $OUT/r06u_${v}_summary.txt | cut -c1-60
  rm -f $f
done
