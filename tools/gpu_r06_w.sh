#!/bin/bash
# The reference runner's full budget (open_duck_mini_v2/runner.py:44: 150 M env-steps) on one MI355X with the
# final learner: the runner CLI with its evaluations, checkpoints and ONNX exports.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
rm -rf $OUT/ppo150M
timeout -k 10 900 python -u -m open_duck_playground_amd.runner --num_timesteps 150000000 --output_dir $OUT/ppo150M > $OUT/r06w_ppo150M.log 2>&1 || { tail -20 $OUT/r06w_ppo150M.log; exit 1; }
rm -f $OUT/ppo150M/*.onnx $OUT/ppo150M/*.pt
grep -v amdgpu.ids $OUT/r06w_ppo150M.log | tail -2 | cut -c1-300
python3 - <<'PY'
import json, statistics
r = [json.loads(l) for l in open("gpurun_out/ppo150M/metrics.jsonl")]
ev = [(x["step"], round(x["eval/episode_reward"], 1), round(x["eval/avg_episode_length"], 1)) for x in r if "eval/episode_reward" in x]
print("evals", ev)
print("median sps", statistics.median(x["sps"] for x in r if "sps" in x))
PY
