#!/bin/bash
# Learner: the entropy draw on a side stream beside the single-workgroup GAE launch (DUCK_PPO_SIDE_EPS=1, the
# default) against the draw in line (=0), same box; the GPU PPO tests and the 60 M-step run's identity first.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_ppo.py -x -q --timeout 300 --timeout-method thread > $OUT/r06y_tests.log 2>&1 || { tail -40 $OUT/r06y_tests.log; exit 1; }
tail -1 $OUT/r06y_tests.log
for run in 1 2 3; do
  for W in 0 1; do
    DUCK_PPO_SIDE_EPS=$W $T 300 python tools/ppo_throughput.py --updates 6 > $OUT/r06y_$W.json 2> $OUT/r06y.err || { tail -20 $OUT/r06y.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/r06y_$W.json'));print('$run side_eps=$W', '%.3fM training env-steps/s' % (d['value']/1e6), 'learn %.2f ms/update' % (d['timing']['learn_s']/6e-3))"
  done
done
rm -rf $OUT/ppo60M_y
$T 600 python -u -m open_duck_playground_amd.runner --num_timesteps 60000000 --output_dir $OUT/ppo60M_y > $OUT/r06y_ppo60M.log 2>&1 || { tail -20 $OUT/r06y_ppo60M.log; exit 1; }
rm -f $OUT/ppo60M_y/*.onnx $OUT/ppo60M_y/*.pt
python3 - <<'PY'
import json
a = [json.loads(l) for l in open("gpurun_out/ppo60M_y/metrics.jsonl")]
b = [json.loads(l) for l in open("profiles/r06_ppo_c2_60M_metrics.jsonl")]
same = sum(all(x.get(k) == y.get(k) for k in x if k.startswith(("train/", "eval/"))) for x, y in zip(a, b))
print("60M run: records", len(a), "identical to the committed run:", same)
PY
