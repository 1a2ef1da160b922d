#!/bin/bash
# Round 5: is the height-field point band (HF_POINT_BAND) what took rough_dr long from 10 to ~36
# outliers? Same seeds through the banded kernel + banded oracle and through a -DDUCK_HF_POINT_BAND=0
# kernel + oracle_set_hf_band_scale(0) (round 3's plain weighted centroid).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
L=$PWD/open_duck_playground_amd
SEEDS=${SEEDS:-7 11 13 17}
for v in ${VARIANTS:-band noband}; do
  if [ $v = band ]; then f=$L/libduck.so; s=1; else f=$L/libduck_$v.so; s=0; fi
  DUCK_LIB=$f ORACLE_HF_BAND_SCALE=$s timeout -k 10 ${TMO:-560} python -u tools/tf_seed_sweep.py ${CASE:-rough_dr} $SEEDS \
    > $OUT/r05_band_$v.txt 2>&1 || { tail -5 $OUT/r05_band_$v.txt; exit 1; }
  echo "== $v"; grep seed $OUT/r05_band_$v.txt | cut -c1-600
done
