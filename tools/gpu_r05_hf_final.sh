#!/bin/bash
# Round 5, final build: the height-field contact points against the oracle (hfield_deviation --gpu)
# and the rough + DR teacher-forced seed sweep (seeds 7, 11, 13, 17).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u tools/hfield_deviation.py 64 30 --gpu > $OUT/r05_hfield_deviation_gpu.jsonl 2>&1 || { tail -5 $OUT/r05_hfield_deviation_gpu.jsonl; exit 1; }
cut -c1-900 $OUT/r05_hfield_deviation_gpu.jsonl
$T 700 python -u tools/tf_seed_sweep.py rough_dr 7 11 13 17 > $OUT/r05_sweep_final.txt 2>&1 || { tail -5 $OUT/r05_sweep_final.txt; exit 1; }
grep seed $OUT/r05_sweep_final.txt | cut -c1-700
