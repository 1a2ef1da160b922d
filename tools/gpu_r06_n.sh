#!/bin/bash
# Where the learner's time between minibatches and epochs goes: a kernel trace of one PPO update
# (tools/ppo_throughput.py --updates 1) summarised by tools/ppo_trace_summary.py (idle stretches included).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
cd /tmp && $T 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/r06n_trace -o tr -- python3 $GRAFT_REPO_ROOT/tools/ppo_throughput.py --updates 1 > $GRAFT_REPO_ROOT/$OUT/r06n_trace.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$OUT/r06n_trace.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $OUT/r06n_trace -name "*kernel_trace.csv" | head -1)
python3 tools/ppo_trace_summary.py $f > $OUT/r06n_trace_summary.txt && cat $OUT/r06n_trace_summary.txt
tail -1 $OUT/r06n_trace.log | cut -c1-600
rm -f $f
