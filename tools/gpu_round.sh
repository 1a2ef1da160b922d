#!/bin/bash
# One GPU call: GPU parity suite, C2 bench, rocprofv3 kernel trace + separate PMC passes, summary.
# usage (from the repo root, on the box): bash tools/gpu_round.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > $OUT/gpu_tests_$TAG.log 2>&1 || { tail -30 $OUT/gpu_tests_$TAG.log; exit 1; }
  tail -3 $OUT/gpu_tests_$TAG.log
fi
timeout -k 10 300 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { cat $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
rm -rf $OUT/prof_$TAG $OUT/pmcf_$TAG $OUT/pmcw_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv rocpd -- \
  python3 bench.py --steps 100 --cpu-budget 0 > $OUT/bench_prof_$TAG.json 2>&1 || { tail $OUT/bench_prof_$TAG.json; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmcf_$TAG -o run --output-format rocpd -- \
  python3 bench.py --steps 20 --warmup 5 --cpu-budget 0 > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmcw_$TAG -o run --output-format rocpd -- \
  python3 bench.py --steps 20 --warmup 5 --cpu-budget 0 > /dev/null 2>&1 || exit 1
ls -R $OUT/prof_$TAG | head -20
