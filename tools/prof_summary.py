#!/usr/bin/env python3
"""Summarise rocprofv3 run_results.db files (kernel trace stats and PMC counters) as text.

usage: prof_summary.py OUT.txt trace_dir [pmc_dir ...]
"""

import sqlite3
import sys


def short(name: str, n: int = 90) -> str:
    return name if len(name) <= n else name[:n] + "..."


def main():
    out = open(sys.argv[1], "w")
    trace = sys.argv[2]
    con = sqlite3.connect(f"{trace}/run_results.db")
    out.write(f"# rocprofv3 --kernel-trace --stats  ({trace})\n")
    out.write(f"{'kernel':92s} {'calls':>6s} {'total_ms':>12s} {'avg_ms':>10s} {'pct':>7s}\n")
    for name, calls, tot, avg, pct in con.execute("select name,total_calls,total_duration,average,percentage "
                                                  "from top_kernels order by total_duration desc"):
        out.write(f"{short(name):92s} {calls:6d} {tot / 1e3:12.1f} {avg / 1e3:10.2f} {pct:7.2f}\n")
    # launch geometry / resources of our kernels
    out.write("\n# kernel resources (first dispatch)\n")
    seen = set()
    for r in con.execute("select name, grid_x, workgroup_x, lds_size, scratch_size, vgpr_count, "
                         "accum_vgpr_count, sgpr_count from kernels"):
        if r[0] in seen or r[0].startswith("void at::"):
            continue
        seen.add(r[0])
        out.write(f"{short(r[0], 60):62s} grid {r[1]} wg {r[2]} lds {r[3]} scratch {r[4]} vgpr {r[5]} "
                  f"agpr {r[6]} sgpr {r[7]}\n")
    for pmc in sys.argv[3:]:
        c = sqlite3.connect(f"{pmc}/run_results.db")
        out.write(f"\n# rocprofv3 --pmc  ({pmc}); values per dispatch, FETCH_SIZE/WRITE_SIZE in KB\n")
        for k, cn, avg, cnt in c.execute("select kernel_name, counter_name, avg(value), count(*) from "
                                         "counters_collection group by kernel_name, counter_name"):
            if k.startswith("void at::") or k.startswith("__amd"):
                continue
            out.write(f"{short(k, 60):62s} {cn:12s} avg {avg:14.2f} over {cnt} dispatches\n")
    out.close()


if __name__ == "__main__":
    main()
