#!/bin/bash
# Real per-stage cost by doubling: libduck_d<k>.so runs one idempotent stage twice per substep
# (DUCK_DOUBLE = 1 crb, 2 collision, 3 make_rows, 4 the qacc_smooth factor + solves); the time
# difference to libduck.so is that stage's cost in the unperturbed kernel. Build the libraries first:
#   for d in 1 2 3 4; do python -c "from open_duck_playground_amd import native; native.build(defines=['DUCK_DOUBLE=$d'], out='open_duck_playground_amd/libduck_d$d.so')"; done
# usage: bash tools/gpu_stage_double.sh
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for C in ${CFGS:-C2 C4 C5}; do
  for v in base d1 d2 d3 d4; do
    if [ $v = base ]; then unset DUCK_LIB; else export DUCK_LIB=$PWD/open_duck_playground_amd/libduck_$v.so; fi
    timeout -k 10 200 python bench.py --cpu-budget 0 --steps 100 --warmup 10 --config $C > $OUT/sd_$C$v.json 2> $OUT/sd_$C$v.err || { tail -3 $OUT/sd_$C$v.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/sd_$C$v.json'));print('$C $v kernel_ms %.4f' % d['roofline']['kernel_ms'])"
  done
done
