#!/bin/bash
# Per-stage attribution of the step kernel's cycles, VALU instructions and waits by doubling: for
# each build/libduck_d<k>.so (one idempotent stage run twice per substep, DUCK_DOUBLE = k, see
# duck_team.h step()) the launch time from bench.py and one rocprofv3 pass of 8 SQ counters; the
# difference to the normal build is that stage's share, unperturbed by markers
# (tools/stage_pmc_summary.py). Build the libraries on the CPU first:
#   python tools/stage_pmc_summary.py --build [--variant flat] [--stages 1 2 3 4 5 6 7 8]
# usage (repo root, on the box): CFG=C2 STAGES="1 2 3 4 5 6 7 8" bash tools/gpu_stage_pmc.sh
#   (rough scenes: CFG=C4 SUFFIX=_rough_terrain STAGES="2 11 12 ..."; libraries built with --variant rough_terrain)
set -o pipefail
CFG=${CFG:-C2}
SUFFIX=${SUFFIX:-}
OUT=gpurun_out/stage_pmc_$CFG
export TMPDIR=/tmp
rm -rf $OUT; mkdir -p $OUT
P="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS"
for v in base ${STAGES:-1 2 3 4 5 6 7 8}; do
  if [ $v = base ]; then export DUCK_LIB=$PWD/open_duck_playground_amd/build/libduck_stage_base$SUFFIX.so; else export DUCK_LIB=$PWD/open_duck_playground_amd/build/libduck_d$v$SUFFIX.so; fi
  timeout -k 10 200 python3 bench.py --cpu-budget 0 --steps 100 --warmup 10 --config $CFG > $OUT/bench_$v.json 2> $OUT/bench_$v.err \
    || { tail -3 $OUT/bench_$v.err; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/pmc_$v -o run --output-format csv -- python3 bench.py --cpu-budget 0 \
    --config $CFG --steps 10 --warmup 2 > /dev/null 2>&1 || { echo "pmc pass $v failed"; exit 1; }
  echo "$v done"
done
python3 tools/stage_pmc_summary.py --report $OUT
