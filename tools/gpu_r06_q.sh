#!/bin/bash
# The rollout's transition stores as one gather launch per env-step: the GPU PPO tests, training throughput,
# the per-kernel trace of one update and the 60 M-step run (compared value for value with the committed one).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_ppo.py -x -q --timeout 300 --timeout-method thread > $OUT/r06q_tests.log 2>&1 || { tail -40 $OUT/r06q_tests.log; exit 1; }
tail -1 $OUT/r06q_tests.log
for run in 1 2; do
  $T 300 python tools/ppo_throughput.py --updates 6 > $OUT/r06q_tp_$run.json 2> $OUT/r06q.err || { tail -20 $OUT/r06q.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/r06q_tp_$run.json'));print('$run', '%.3fM training env-steps/s' % (d['value']/1e6), 'learn %.1f ms/update, rollout %.1f ms/update' % (d['timing']['learn_s']/6e-3, d['timing']['rollout_s']/6e-3))"
done
cd /tmp && $T 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/r06q_trace -o tr -- python3 $GRAFT_REPO_ROOT/tools/ppo_throughput.py --updates 1 > $GRAFT_REPO_ROOT/$OUT/r06q_trace.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$OUT/r06q_trace.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $OUT/r06q_trace -name "*kernel_trace.csv" | head -1)
python3 tools/ppo_trace_summary.py $f > $OUT/r06q_trace_summary.txt && grep -A8 busiest $OUT/r06q_trace_summary.txt
rm -f $f
rm -rf $OUT/ppo60M_q
$T 600 python -u -m open_duck_playground_amd.runner --num_timesteps 60000000 --output_dir $OUT/ppo60M_q > $OUT/r06q_ppo60M.log 2>&1 || { tail -20 $OUT/r06q_ppo60M.log; exit 1; }
rm -f $OUT/ppo60M_q/*.onnx $OUT/ppo60M_q/*.pt
python3 - <<'PY'
import json, statistics
a = [json.loads(l) for l in open("gpurun_out/ppo60M_q/metrics.jsonl")]
b = [json.loads(l) for l in open("profiles/r06_ppo_c2_60M_metrics.jsonl")]
same = sum(all(x.get(k) == y.get(k) for k in x if k.startswith(("train/", "eval/"))) for x, y in zip(a, b))
print("60M run: records", len(a), "identical to the committed run:", same, "median sps", statistics.median(r["sps"] for r in a if "sps" in r))
PY
