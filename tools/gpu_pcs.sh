#!/bin/bash
# PC sampling of the C2 step kernel (rocprofv3 beta, stochastic or host_trap): which instructions the
# waves stall at. usage: bash tools/gpu_pcs.sh [METHOD] [INTERVAL]
set -o pipefail
OUT=gpurun_out/pcs; rm -rf $OUT; mkdir -p $OUT; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/list.txt 2>&1; grep -i -A12 "pc.sampl" $OUT/list.txt | head -40
timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${1:-stochastic} --pc-sampling-unit cycles \
  --pc-sampling-interval ${2:-262144} -d $OUT/run -o run --output-format csv -- python3 bench.py --steps 50 --warmup 10 --cpu-budget 0 \
  > $OUT/bench.json 2> $OUT/err.txt || { tail -20 $OUT/err.txt; exit 1; }
find $OUT/run -type f | head; du -sh $OUT/run
