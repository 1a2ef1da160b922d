#!/bin/bash
# rocprofv3 evidence for the bench line of one configuration, each pass its own run:
#   kernel trace + stats, FETCH_SIZE, WRITE_SIZE, two SQ counter passes
# then tools/pmc_summary.py -> profiles/<TAG>_pmc_<cfg>.json (+ stats csv, text summary).
# usage (repo root, on the box): bash tools/gpu_pmc.sh TAG [CONFIG]
set -o pipefail
TAG=${1:-r02}
CFG=${2:-C2}
OUT=gpurun_out/pmc_${TAG}_$CFG
export TMPDIR=/tmp
rm -rf $OUT; mkdir -p $OUT
B="python3 bench.py --config $CFG --cpu-budget 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B --steps 100 \
  > $OUT/bench_trace.json 2>&1 || { tail $OUT/bench_trace.json; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B --steps 20 --warmup 5 \
  > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B --steps 20 --warmup 5 \
  > /dev/null 2>&1 || exit 1
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32"
timeout -s KILL 120 rocprofv3 --pmc $P1 -d $OUT/sq1 -o run --output-format csv -- $B --steps 10 --warmup 2 \
  > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $P2 -d $OUT/sq2 -o run --output-format csv -- $B --steps 10 --warmup 2 \
  > /dev/null 2>&1 || exit 1
python3 tools/pmc_summary.py $OUT $TAG $CFG
