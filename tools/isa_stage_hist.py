#!/usr/bin/env python3
"""Static instruction mix of the step kernel per stage (CPU only).

Compiles one scene unit to assembly with -DDUCK_ASM_MARKS (each STAGE_MARK(k) becomes the comment
"; STAGE_MARK k", no code) and the library's own flags, then counts the instructions of
step_kernel<...> between consecutive marks: the region that ends at mark k is named after k
(duck_team.h: 0 kinematics, 1 com_pos, 2 rne, 3 crb, 28 smooth, 5 collision, 6 make_rows, 20 load_cols,
4 smooth_acc, 25/9 warm start, 16-18 Newton direction, 12 search products, 13 line search, 7/8
sensors + Euler). Static counts of straight-line code are its per-substep dynamic counts; loops
(the line search, the height field's queue) run more often.

usage: python tools/isa_stage_hist.py [--variant flat] [--kernel step_kernel] [--lat 0]
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = {0: "kinematics", 1: "com_pos", 2: "rne", 3: "crb", 28: "smooth", 5: "collision", 6: "make_rows",
         20: "load_cols", 4: "smooth_acc", 25: "warm start (products)", 9: "warm start (rows, choice)",
         16: "newton: gradient + M columns", 17: "newton: J'DJ blocks", 18: "newton: factor + solves",
         10: "newton: store", 11: "newton: -", 12: "search products + rows", 13: "line search + update",
         7: "solve tail", 8: "sensors + euler", 24: "kinematics (poses)", 21: "rne: velocities",
         22: "rne: forces", 35: "rne: subtree a", 36: "rne: subtree b", 19: "crb: inertias", 26: "collision: planes"}


def classify(op):
    if op.startswith("v_pk_"):
        return "valu_pk"
    if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
        return "lane_rw"
    if op.startswith(("v_accvgpr")):
        return "agpr_mov"
    if "_dpp" in op:
        return "valu_dpp"
    if op.startswith(("v_add_u32", "v_sub_u32", "v_lshl", "v_mad_u", "v_mul_u", "v_add3_u32", "v_and_b32",
                      "v_or_b32", "v_xor_b32", "v_lshr", "v_ashr", "v_mul_lo", "v_mad_i", "v_add_co", "v_addc")):
        return "valu_int"
    if op.startswith(("v_cndmask", "v_cmp")):
        return "valu_sel"
    if op.startswith(("v_mov_b32", "v_mov_b64")):
        return "valu_mov"
    if op.startswith(("v_rcp", "v_sqrt", "v_rsq", "v_sin", "v_cos", "v_exp", "v_log")):
        return "valu_trans"
    if op.startswith("v_"):
        return "valu_fp"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op == "s_waitcnt":
        return "waitcnt"
    if op == "s_nop":
        return "s_nop"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="flat")
    ap.add_argument("--kernel", default="_Z11step_kernel")
    ap.add_argument("--defines", nargs="*", default=[])
    a = ap.parse_args()
    sys.path.insert(0, ROOT)
    from open_duck_playground_amd import native
    csrc = os.path.join(ROOT, "open_duck_playground_amd", "csrc")
    src = os.path.join(csrc, f"variant_{a.variant}.hip")
    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, "k.s")
        cmd = (["hipcc"] + native._base_flags(os.path.join(csrc, "generated")) + native.ILP_FLAGS +
               ["-DDUCK_ASM_MARKS"] + [f"-D{d}" for d in a.defines] +
               ["--cuda-device-only", "-S", "-o", out, src])
        subprocess.check_call(cmd, cwd=csrc)
        text = open(out).read()
    m = re.search(rf"^({re.escape(a.kernel)}\w*):[^\n]*$(.*?)^\s*s_endpgm", text, re.M | re.S)
    if not m:
        raise SystemExit(f"kernel {a.kernel} not found")
    body = m.group(2)
    regions, cur, order = collections.OrderedDict(), collections.Counter(), []
    for line in body.splitlines():
        mk = re.match(r"\s*;\s*STAGE_MARK (\d+)", line)
        if mk:
            k = int(mk.group(1))
            key = f"{k:>2} {NAMES.get(k, '?')}"
            regions.setdefault(key, collections.Counter()).update(cur)
            cur = collections.Counter()
            continue
        mi = re.match(r"\s+([a-z][a-z0-9_]*)\b", line)
        if mi and not line.strip().startswith(";"):
            cur[classify(mi.group(1))] += 1
    regions.setdefault("(after last mark)", collections.Counter()).update(cur)
    cols = ["valu_fp", "valu_pk", "valu_dpp", "valu_int", "valu_sel", "valu_mov", "valu_trans", "lane_rw",
            "agpr_mov", "lds", "vmem", "waitcnt", "s_nop", "salu"]
    print(f"{m.group(1)[:60]} ({a.variant}): static instructions per region (ending at STAGE_MARK k)")
    print(f"{'region':34s} {'total':>6s} " + " ".join(f"{c:>9s}" for c in cols))
    tot = collections.Counter()
    for k, c in regions.items():
        tot.update(c)
        print(f"{k[:34]:34s} {sum(c.values()):6d} " + " ".join(f"{c[x]:9d}" for x in cols))
    print(f"{'total':34s} {sum(tot.values()):6d} " + " ".join(f"{tot[x]:9d}" for x in cols))


if __name__ == "__main__":
    main()
