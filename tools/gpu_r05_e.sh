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
DUCK_LIB=$PWD/open_duck_playground_amd/libduck_contracton.so $T 300 python -u tools/lat_bitcmp.py C2 C3 > $OUT/r05e_bitcmp_on.txt 2>&1 || { tail -5 $OUT/r05e_bitcmp_on.txt; exit 1; }
echo "== -ffp-contract=on"; grep -v amdgpu.ids $OUT/r05e_bitcmp_on.txt
for i in 1 2; do for v in libduck libduck_contracton; do
  DUCK_LIB=$PWD/open_duck_playground_amd/$v.so $T 200 python bench.py --steps 400 --warmup 50 --cpu-budget 0 > $OUT/r05e_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/r05e_$v.json'));print('C2 $v', '%.4gM' % (d['value']/1e6), 'kernel_ms %.4f' % d['roofline']['kernel_ms'])"
done; done
