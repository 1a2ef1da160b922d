#!/bin/bash
# The three unexplained outliers of the final-build seed sweep (profiles/r06_tf_seed_sweep_final.txt) in detail.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
rm -f $OUT/r06_tf_defects.txt
$T 400 python -u tools/tf_defect_detail.py rough_dr 29 5 100 >> $OUT/r06_tf_defects.txt 2> $OUT/r06aa.err || { tail -20 $OUT/r06aa.err; exit 1; }
$T 400 python -u tools/tf_defect_detail.py rough_backlash_dr 19 0 52 >> $OUT/r06_tf_defects.txt 2> $OUT/r06aa.err || { tail -20 $OUT/r06aa.err; exit 1; }
$T 400 python -u tools/tf_defect_detail.py flat_backlash_imitation 23 6 133 >> $OUT/r06_tf_defects.txt 2> $OUT/r06aa.err || { tail -20 $OUT/r06aa.err; exit 1; }
cut -c1-400 $OUT/r06_tf_defects.txt
