#!/bin/bash
# Parity on the final round-6 build: the teacher-forced sweep (tools/tf_seed_sweep.py, 1,024 envs x 10 env-steps
# per seed, every outlier classified by explain()) over seeds the suite does not use, flat and rough cases.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
rm -f $OUT/r06_tf_seed_sweep_final.txt
for c in flat rough_dr rough_backlash_dr flat_backlash_imitation; do
  $T 500 python -u tools/tf_seed_sweep.py $c 19 23 29 31 >> $OUT/r06_tf_seed_sweep_final.txt 2> $OUT/r06z.err || { tail -20 $OUT/r06z.err; exit 1; }
done
cut -c1-260 $OUT/r06_tf_seed_sweep_final.txt
