#!/bin/bash
# Round 6 learner: the swizzled / natural LDS tile layouts (shipped libduck.so, 6 waves per SIMD) against the
# previous layouts (build/libduck_base.so) and the new layouts uncapped (build/libduck_wpe1.so, 5 waves).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_ppo.py -x -q --timeout 300 --timeout-method thread > $OUT/r06k_tests.log 2>&1 || { tail -40 $OUT/r06k_tests.log; exit 1; }
tail -1 $OUT/r06k_tests.log
for run in 1 2; do
  for LIBV in base new wpe1; do
    L=""; [ $LIBV = base ] && L=open_duck_playground_amd/build/libduck_base.so; [ $LIBV = wpe1 ] && L=open_duck_playground_amd/build/libduck_wpe1.so
    DUCK_LIB=$L $T 300 python tools/ppo_throughput.py --updates 6 > $OUT/r06k_${LIBV}.json 2> $OUT/r06k.err || { tail -20 $OUT/r06k.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/r06k_${LIBV}.json'));print('$run $LIBV', '%.3fM training env-steps/s' % (d['value']/1e6), 'learn %.1f ms/update' % (d['timing']['learn_s']/6e-3))"
  done
done
cd /tmp && $T 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/r06k_trace -o tr -- python3 $GRAFT_REPO_ROOT/tools/ppo_throughput.py --updates 1 > $GRAFT_REPO_ROOT/$OUT/r06k_trace.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$OUT/r06k_trace.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $OUT/r06k_trace -name "*kernel_trace.csv" | head -1)
python3 tools/ppo_trace_summary.py $f > $OUT/r06k_trace_summary.txt && cat $OUT/r06k_trace_summary.txt
rm -f $f
