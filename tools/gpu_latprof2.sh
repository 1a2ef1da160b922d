#!/bin/bash
# timelines of both latency kernels (DUCK_LAT_PROF build libduck_latprof.so: native.build(defines=["DUCK_LAT_PROF"],
# isa_check=False); its throughput kernels are not used) for the configs in CFGS at ENVS envs
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for C in ${CFGS:-C2 C5}; do
  for M in ${MODES:-paired latency}; do
    DUCK_LIB=$PWD/open_duck_playground_amd/libduck_latprof.so timeout -k 10 120 python tools/lat_prof.py --config $C --mode $M --envs ${ENVS:-1024} > $OUT/r05_latprof_${C}_$M.txt 2>&1 || { tail $OUT/r05_latprof_${C}_$M.txt; exit 1; }
    echo "== $C $M"; grep -v amdgpu.ids $OUT/r05_latprof_${C}_$M.txt | head -${LINES_:-45}
  done
done
