#!/bin/bash
# Round 6 final evidence, second pass (the learner kernels changed libduck.so after the first): the GPU suite,
# smoke(), the C2 / C5 / C4 rocprofv3 evidence (tools/gpu_pmc.sh, one directory per config), the bench lines
# (C2 steady and in the driver's 20-after-5 form, C3, C4, C5, --gpus 2 direct weak and --strong), PPO training
# throughput and the 60 M-step learning run.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/r06b_gpu_tests.log 2>&1 || { tail -60 $OUT/r06b_gpu_tests.log; exit 1; }
grep -E "passed|failed" $OUT/r06b_gpu_tests.log | tail -1
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/r06b_smoke.log 2>&1 || { tail -20 $OUT/r06b_smoke.log; exit 1; }
grep smoke $OUT/r06b_smoke.log
for C in C2 C5 C4; do
  $T 400 bash tools/gpu_pmc.sh r06 $C > $OUT/r06b_pmc_$C.log 2>&1 || { tail -20 $OUT/r06b_pmc_$C.log; exit 1; }
done
ls $OUT/pmc_r06_C2 $OUT/pmc_r06_C5 $OUT/pmc_r06_C4 | grep json
$T 300 python bench.py > $OUT/r06b_bench_C2.json 2> $OUT/r06b_bench.err || { tail -20 $OUT/r06b_bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/r06b_bench_C2.json'));print('C2 steady %.4gM %.4f ms' % (d['value']/1e6, d['ms_per_step']))"
rm -f $OUT/r06b_bench_C2_driver_style.jsonl
for i in 1 2 3; do
  $T 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-budget 0 >> $OUT/r06b_bench_C2_driver_style.jsonl 2> $OUT/r06b_bench.err || { tail -20 $OUT/r06b_bench.err; exit 1; }
done
python -c "import json; print('driver form', [round(json.loads(l)['value']/1e6, 3) for l in open('$OUT/r06b_bench_C2_driver_style.jsonl')])"
for C in C3 C4 C5; do
  $T 300 python bench.py --config $C --cpu-budget 0 > $OUT/r06b_bench_$C.json 2> $OUT/r06b_bench.err || { tail -20 $OUT/r06b_bench.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/r06b_bench_$C.json'));print('$C', '%.4gM env-steps/s %.4f ms' % (d['value']/1e6, d['ms_per_step']))"
done
DUCK_DIST_BACKEND=gloo $T 300 python bench.py --gpus 2 --steps 100 --warmup 10 --cpu-budget 0 > $OUT/r06b_bench_direct2.jsonl 2> $OUT/r06b_bench.err || { tail -20 $OUT/r06b_bench.err; exit 1; }
DUCK_DIST_BACKEND=gloo $T 300 python bench.py --gpus 2 --strong --steps 100 --warmup 10 --cpu-budget 0 >> $OUT/r06b_bench_direct2.jsonl 2> $OUT/r06b_bench.err || { tail -20 $OUT/r06b_bench.err; exit 1; }
cut -c1-300 $OUT/r06b_bench_direct2.jsonl
for run in 1 2; do
  $T 300 python tools/ppo_throughput.py --updates 6 > $OUT/r06b_ppo_tp_$run.json 2> $OUT/r06b.err || { tail -20 $OUT/r06b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/r06b_ppo_tp_$run.json'));print('ppo $run', '%.3fM training env-steps/s' % (d['value']/1e6), 'learn %.1f ms/update, rollout %.1f ms/update' % (d['timing']['learn_s']/6e-3, d['timing']['rollout_s']/6e-3))"
done
rm -rf $OUT/ppo60M_b
$T 600 python -u -m open_duck_playground_amd.runner --num_timesteps 60000000 --output_dir $OUT/ppo60M_b > $OUT/r06b_ppo60M.log 2>&1 || { tail -20 $OUT/r06b_ppo60M.log; exit 1; }
grep -v amdgpu.ids $OUT/r06b_ppo60M.log | tail -2 | cut -c1-400
rm -f $OUT/ppo60M_b/*.onnx $OUT/ppo60M_b/*.pt
