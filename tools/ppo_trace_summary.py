#!/usr/bin/env python3
"""Per-launch costs of one PPO learner minibatch from a rocprofv3 --kernel-trace CSV (tools/gpu_ppo_trace.sh):
the dispatches between two consecutive gather_kernel launches are one minibatch; for each position in that
sequence it prints the kernel, its mean duration and the mean idle gap in front of it (launch overhead inside
the replayed graph), then the minibatch's wall span. usage: python tools/ppo_trace_summary.py kernel_trace.csv"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    starts = [i for i, e in enumerate(ev) if "gather_kernel" in e[2]]
    seqs = [ev[a:b] for a, b in zip(starts[:-1], starts[1:])]
    # the learner's minibatches: the most common sequence length (rollout segments differ)
    lens = defaultdict(int)
    for s in seqs:
        lens[len(s)] += 1
    L = max(lens, key=lens.get)
    seqs = [s for s in seqs if len(s) == L]
    print(f"{len(seqs)} minibatches of {L} launches (sequence lengths seen: {dict(lens)})")
    dur, gap = [0.0] * L, [0.0] * L
    for s in seqs:
        for k, (a, b, _) in enumerate(s):
            dur[k] += (b - a) / 1e3
            if k:
                gap[k] += (a - s[k - 1][1]) / 1e3
    n = len(seqs)
    span = sum((s[-1][1] - s[0][0]) / 1e3 for s in seqs) / n
    for k in range(L):
        print(f"{k:3d} {dur[k] / n:8.2f} us  gap {gap[k] / n:6.2f} us  {seqs[0][k][2][:100]}")
    print(f"busy {sum(dur) / n:.1f} us, gaps {sum(gap) / n:.1f} us, span gather..last end {span:.1f} us per minibatch")
    # idle time in front of every minibatch (inside an epoch graph, at epoch boundaries) and the
    # longest idle stretches of the whole trace with the kernels around them
    pre = sorted(((ev[i][0] - ev[i - 1][1]) / 1e3, i) for i in starts if i > 0)
    if pre:
        g = [x for x, _ in pre]
        print(f"idle before a minibatch's gather: median {g[len(g) // 2]:.2f} us, max {g[-1]:.1f} us, "
              f"sum {sum(g):.1f} us over {len(g)}")
    idle = sorted((((ev[i][0] - ev[i - 1][1]) / 1e3, i) for i in range(1, len(ev))), reverse=True)[:12]
    for x, i in idle:
        print(f"  idle {x:9.1f} us  after {ev[i - 1][2][:60]}  before {ev[i][2][:60]}")
    agg = defaultdict(lambda: [0, 0.0])
    for a, b, k in ev:
        agg[k[:70]][0] += 1
        agg[k[:70]][1] += (b - a) / 1e3
    print("busiest kernels of the trace (count, total us):")
    for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
        print(f"  {c:6d} {t:10.1f}  {k}")
    print(f"trace: {len(ev)} dispatches over {(ev[-1][1] - ev[0][0]) / 1e6:.2f} ms, busy "
          f"{sum(b - a for a, b, _ in ev) / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
