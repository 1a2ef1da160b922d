#!/bin/bash
# three-lane height-field SAT (hf_exec3): bit-identity against libduck_A.so (-DDUCK_HF_NO_SPLIT) and the C4/C5 A/B;
# the survivors-per-wave histogram of the stage build; latency/throughput bit-compare with DR toggles
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
$T 900 bash tools/gpu_ab_bitcmp.sh r05e || exit 1
$T 400 bash tools/gpu_stage_rough.sh > /dev/null || exit 1
grep -iE "surviv|queue|pass|collision|hfield" gpurun_out/stage_rough_terrain.txt gpurun_out/stage_rough_terrain_backlash.txt
$T 500 python -u tools/lat_bitcmp.py C2 C2+dr C4-dr C4 C2@paired C4@paired > $OUT/r05d_bitcmp.txt 2>&1 || { tail -5 $OUT/r05d_bitcmp.txt; exit 1; }
grep -v amdgpu.ids $OUT/r05d_bitcmp.txt
