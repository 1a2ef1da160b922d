#!/bin/bash
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
L=$PWD/open_duck_playground_amd
DUCK_LIB=$L/libduck_A.so timeout -k 10 300 python tools/tf_defect_probe.py rough_dr 17 3:933 > $OUT/probe_A17.txt 2>&1 || { tail $OUT/probe_A17.txt; exit 1; }
timeout -k 10 300 python tools/tf_defect_probe.py rough_dr 7 6:619 9:388 > $OUT/probe_c7.txt 2>&1 || { tail $OUT/probe_c7.txt; exit 1; }
grep -v amdgpu.ids $OUT/probe_A17.txt | head -60
