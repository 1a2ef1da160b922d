#!/bin/bash
# Round 5, last GPU call: bit-identity of the final build against the build of the first evidence
# pass (libduck_A.so = e244d24) on C4 / C5 with their A/B lines, then the round-end evidence
# (tools/gpu_round_end.sh) and the height-field evidence (tools/gpu_r05_hf_final.sh).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
REPS=1 bash tools/gpu_ab_bitcmp.sh fin > $OUT/fin_ab.txt 2>&1 || { tail -20 $OUT/fin_ab.txt; exit 1; }
cat $OUT/fin_ab.txt
PMC_EXTRA=C5 bash tools/gpu_round_end.sh r05 || exit 1
bash tools/gpu_r05_hf_final.sh || exit 1
