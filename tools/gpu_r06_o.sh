#!/bin/bash
# The normaliser update on duck_column_stats: the GPU PPO tests, then training throughput and the
# per-kernel trace of one update (tools/ppo_trace_summary.py).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_ppo.py -x -q --timeout 300 --timeout-method thread > $OUT/r06o_tests.log 2>&1 || { tail -40 $OUT/r06o_tests.log; exit 1; }
tail -1 $OUT/r06o_tests.log
for run in 1 2; do
  $T 300 python tools/ppo_throughput.py --updates 6 > $OUT/r06o_tp.json 2> $OUT/r06o.err || { tail -20 $OUT/r06o.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/r06o_tp.json'));print('$run', '%.3fM training env-steps/s' % (d['value']/1e6), 'learn %.1f ms/update, rollout %.1f ms/update' % (d['timing']['learn_s']/6e-3, d['timing']['rollout_s']/6e-3))"
done
cd /tmp && $T 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/r06o_trace -o tr -- python3 $GRAFT_REPO_ROOT/tools/ppo_throughput.py --updates 1 > $GRAFT_REPO_ROOT/$OUT/r06o_trace.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$OUT/r06o_trace.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $OUT/r06o_trace -name "*kernel_trace.csv" | head -1)
python3 tools/ppo_trace_summary.py $f > $OUT/r06o_trace_summary.txt && tail -32 $OUT/r06o_trace_summary.txt
rm -f $f
