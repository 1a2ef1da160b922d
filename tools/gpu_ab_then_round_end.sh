#!/bin/bash
# Same-box A/B of libduck.so (candidate) against libduck_base.so, then the round-end evidence
# (tools/gpu_round_end.sh) on whichever is faster: a losing candidate is replaced by the base build
# before the profile, bench lines and GPU suite run. usage (repo root, on the box): bash tools/gpu_ab_then_round_end.sh TAG
set -o pipefail
TAG=${1:-r02}
OUT=gpurun_out; mkdir -p $OUT
A=base bash tools/gpu_ab_lib.sh > $OUT/ab_final.log 2>&1 || { tail -20 $OUT/ab_final.log; exit 1; }
grep -E "passed|value" $OUT/ab_final.log
WIN=$(python3 -c "
import json
v = lambda t: sum(json.load(open(f'$OUT/ab_{t}{i}.json'))['value'] for i in (1, 2, 3)) / 3
print('cand' if v('cand') > v('base') else 'base')")
echo "faster: $WIN"
if [ "$WIN" = base ]; then cp open_duck_playground_amd/libduck_base.so open_duck_playground_amd/libduck.so; fi
bash tools/gpu_round_end.sh $TAG
