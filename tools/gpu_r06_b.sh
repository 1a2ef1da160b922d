#!/bin/bash
# Round 6 call B: the two-waves-per-SIMD latency kernel (lat2w / lat2wb debug builds) bit for bit against
# the throughput kernel in every scene, and against the paired kernel at 2,048 envs in the rough scenes;
# then a per-dispatch kernel trace of the PPO learner (tools/ppo_trace_summary.py).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
DUCK_LIB=open_duck_playground_amd/build/libduck_lat2w.so $T 300 python tools/lat_bitcmp.py C2 C3 C4 > $OUT/r06b_bitcmp.txt 2>&1 || { tail -20 $OUT/r06b_bitcmp.txt; exit 1; }
DUCK_LIB=open_duck_playground_amd/build/libduck_lat2wb.so $T 300 python tools/lat_bitcmp.py C5 >> $OUT/r06b_bitcmp.txt 2>&1 || { tail -20 $OUT/r06b_bitcmp.txt; exit 1; }
grep "@" $OUT/r06b_bitcmp.txt
for C in C4 C5; do
  LIB=open_duck_playground_amd/build/libduck_lat2w.so; [ $C = C5 ] && LIB=open_duck_playground_amd/build/libduck_lat2wb.so
  for N in 1024 2048; do
    for M in paired latency; do
      f=$OUT/r06b_w_${C}_${M}_$N
      $T 240 python bench.py --config $C --envs $N --steps 100 --warmup 10 --cpu-budget 0 --step-mode $M > $f.json 2> $f.err || { tail $f.err; exit 1; }
      python -c "import json;d=json.load(open('$f.json'));print('shipped', '$C', '$M', $N, '%.4gM env-steps/s %.4f ms kernel %.4f' % (d['value']/1e6, d['ms_per_step'], d['roofline']['kernel_ms']))"
    done
    f=$OUT/r06b_w_${C}_lat2w_$N
    DUCK_LIB=$LIB $T 240 python bench.py --config $C --envs $N --steps 100 --warmup 10 --cpu-budget 0 --step-mode latency > $f.json 2> $f.err || { tail $f.err; exit 1; }
    python -c "import json;d=json.load(open('$f.json'));print('lat2w  ', '$C', 'latency', $N, '%.4gM env-steps/s %.4f ms kernel %.4f' % (d['value']/1e6, d['ms_per_step'], d['roofline']['kernel_ms']))"
  done
done
cd /tmp && $T 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/r06b_ppo_trace -o tr -- python3 $GRAFT_REPO_ROOT/tools/ppo_throughput.py --updates 1 > $GRAFT_REPO_ROOT/$OUT/r06b_ppo_trace.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$OUT/r06b_ppo_trace.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $OUT/r06b_ppo_trace -name "*kernel_trace.csv" | head -1)
python3 tools/ppo_trace_summary.py $f > $OUT/r06b_ppo_trace_summary.txt && cat $OUT/r06b_ppo_trace_summary.txt
rm -f $f
