#!/bin/bash
# latency-kernel timeline + per-stage cycles (DUCK_LAT_PROF build; its throughput kernels are not used and
# not ISA-gated) for the configs in CFGS
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for C in ${CFGS:-C2 C5}; do
  DUCK_LIB=$PWD/open_duck_playground_amd/libduck_latprof.so timeout -k 10 120 python tools/lat_prof.py --config $C > $OUT/r04_latprof_$C.txt 2>&1 || { tail $OUT/r04_latprof_$C.txt; exit 1; }
  echo "== $C"; grep -v amdgpu.ids $OUT/r04_latprof_$C.txt
done
