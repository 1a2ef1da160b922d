#!/bin/bash
# Round 6 learner work: the PPO GPU tests, training throughput (tools/ppo_throughput.py) and the
# per-launch learner trace (tools/ppo_trace_summary.py). usage: bash tools/gpu_r06_d.sh <tag>
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
TAG=${1:-d}
$T 600 python -u -m pytest tests/test_gpu_ppo.py -x -v --timeout 300 --timeout-method thread > $OUT/r06${TAG}_ppo_tests.log 2>&1 || { tail -60 $OUT/r06${TAG}_ppo_tests.log; exit 1; }
grep -E "passed|failed" $OUT/r06${TAG}_ppo_tests.log | tail -2
for BNM in ${BN_MODES:-auto}; do
  DUCK_MLP_BN=$BNM $T 300 python tools/ppo_throughput.py --updates 6 > $OUT/r06${TAG}_ppo_throughput_$BNM.json 2> $OUT/r06${TAG}_ppo_throughput.err || { tail -20 $OUT/r06${TAG}_ppo_throughput.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/r06${TAG}_ppo_throughput_$BNM.json'));print('DUCK_MLP_BN=$BNM', '%.3fM training env-steps/s' % (d['value']/1e6), d['timing'])"
done
cd /tmp && $T 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/r06${TAG}_ppo_trace -o tr -- python3 $GRAFT_REPO_ROOT/tools/ppo_throughput.py --updates 1 > $GRAFT_REPO_ROOT/$OUT/r06${TAG}_ppo_trace.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$OUT/r06${TAG}_ppo_trace.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $OUT/r06${TAG}_ppo_trace -name "*kernel_trace.csv" | head -1)
python3 tools/ppo_trace_summary.py $f > $OUT/r06${TAG}_ppo_trace_summary.txt && cat $OUT/r06${TAG}_ppo_trace_summary.txt
rm -f $f
