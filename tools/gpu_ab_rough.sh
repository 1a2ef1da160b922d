#!/bin/bash
# Same-box A/B of libduck.so against libduck_b.so on C4 / C5 (3 alternating runs each).
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for L in libduck libduck_b; do
    for C in C4 C5; do
      DUCK_LIB=$PWD/open_duck_playground_amd/$L.so timeout -k 10 200 python bench.py --config $C --cpu-budget 0 --steps 50 --warmup 10 > gpurun_out/ab_${L}_${C}_$r.json 2>/dev/null || exit 1
    done
  done
done
python3 - <<'PY'
import json
for L in ("libduck", "libduck_b"):
    for C in ("C4", "C5"):
        v = [json.load(open(f"gpurun_out/ab_{L}_{C}_{r}.json"))["value"] / 1e6 for r in (1, 2, 3)]
        print(L, C, " ".join(f"{x:.3f}" for x in v), "mean %.3f" % (sum(v) / 3))
PY
