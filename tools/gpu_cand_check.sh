#!/bin/bash
# A kernel candidate on the box: per-env-step comparison with libduck_A.so (C4 shape, 4096 envs, the
# first 5 env-steps), then the whole -m gpu suite on the candidate (libduck.so).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-cc}
L=$PWD/open_duck_playground_amd
for v in A cand; do
  if [ $v = cand ]; then f=$L/libduck.so; else f=$L/libduck_$v.so; fi
  DUCK_LIB=$f timeout -k 10 200 python tools/lib_bitcmp.py --config ${BCFG:-C4} --envs 4096 --steps 5 --every 1 --out $OUT/${TAG}_$v.npz > $OUT/${TAG}_$v.log 2>&1 || { tail -5 $OUT/${TAG}_$v.log; exit 1; }
done
python tools/lib_bitcmp.py --cmp $OUT/${TAG}_A.npz $OUT/${TAG}_cand.npz
rm -f $OUT/${TAG}_A.npz $OUT/${TAG}_cand.npz
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/${TAG}_suite.log 2>&1
rc=$?; grep -E "rules:|passed|failed|good" $OUT/${TAG}_suite.log | cut -c1-220 | tail -40; exit $rc
