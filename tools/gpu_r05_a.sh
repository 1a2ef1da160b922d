#!/bin/bash
# Round 5, first evidence pass: the point band removed (kernel) / a test aid (oracle), the tightened
# classifier (backward_error with contacts, the replica-based selection rules, contact-generation
# defects), the surfaced latency timeout; flat latency/throughput bit-compare with the plane collision
# uncontracted; the height-field contact points against the oracle; the rough_dr seed sweep.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_env.py::test_latency_timeout_surfaces \
  "tests/test_gpu_physics.py::test_hfield_kernel_matches_brute_force_prisms" \
  tests/test_gpu_teacher_forced.py -s > $OUT/r05a_tests.log 2>&1 || { tail -30 $OUT/r05a_tests.log; exit 1; }
grep -E "passed|failed" $OUT/r05a_tests.log | tail -3
for lib in libduck libduck_nocontract; do
  DUCK_LIB=$PWD/open_duck_playground_amd/$lib.so $T 300 python -u tools/lat_bitcmp.py C2 C3 C4 > $OUT/r05a_bitcmp_$lib.txt 2>&1 || { tail -5 $OUT/r05a_bitcmp_$lib.txt; exit 1; }
  echo "== $lib"; cat $OUT/r05a_bitcmp_$lib.txt
done
$T 600 python -u tools/hfield_deviation.py 64 30 --gpu > $OUT/r05_hfield_deviation_gpu.jsonl 2>&1 || { tail -5 $OUT/r05_hfield_deviation_gpu.jsonl; exit 1; }
cut -c1-900 $OUT/r05_hfield_deviation_gpu.jsonl
$T 700 python -u tools/tf_seed_sweep.py rough_dr 7 11 13 17 > $OUT/r05a_sweep.txt 2>&1 || { tail -5 $OUT/r05a_sweep.txt; exit 1; }
grep seed $OUT/r05a_sweep.txt | cut -c1-700
