#!/usr/bin/env python3
"""Scan an AMDGPU asm file for DPP reads of a VGPR written by a VALU fewer than 2 wait states
earlier (the GFX9 "VALU write VGPR -> DPP read" hazard), following fall-through and branch
predecessors. Also lists DPP instructions placed under a non-trivial exec mask context.

usage: isa_dpp_hazards.py file.s [kernel-substring]"""
import re
import sys

path = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else None
lines = open(path).read().split("\n")

# function bodies: from "name:" to s_endpgm / s_setpc (return)
funcs, cur, name = [], None, None
for i, l in enumerate(lines):
    m = re.match(r"^(_Z\S+):", l)
    if m:
        name, cur = m.group(1), []
        funcs.append((name, cur))
        continue
    if cur is not None:
        cur.append((i + 1, l))
        if "s_endpgm" in l or l.strip().startswith(".Lfunc_end"):
            cur = None


def regs_of(op):
    out = set()
    for m in re.finditer(r"v\[(\d+):(\d+)\]", op):
        out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r"\bv(\d+)\b", op):
        out.add(int(m.group(1)))
    return out


def parse(l):
    s = l.split(";")[0].strip()
    if not s or s.startswith("."):
        return None
    if s.endswith(":"):
        return ("label", s[:-1])
    parts = s.split(None, 1)
    return ("ins", parts[0], parts[1] if len(parts) > 1 else "")


for fname, body in funcs:
    if want and want not in fname:
        continue
    seq = []  # (lineno, kind, ...)
    labels = {}
    for ln, l in body:
        p = parse(l)
        if p is None:
            continue
        if p[0] == "label":
            labels[p[1]] = len(seq)
        seq.append((ln,) + p)
    # predecessors of each label index
    preds = {}
    for k, it in enumerate(seq):
        if it[1] == "ins" and it[2].startswith("s_branch") or (it[1] == "ins" and it[2].startswith("s_cbranch")):
            tgt = it[3].split()[0]
            if tgt in labels:
                preds.setdefault(labels[tgt], []).append(k)

    def back(k, need, depth=0, seen=None):
        """walk back from index k-1 collecting up to `need` wait-state-carrying instructions,
        yielding (writes, lineno, waits_before) along every path"""
        seen = seen or set()
        waits = 0
        j = k - 1
        out = []
        while j >= 0 and waits < need:
            it = seq[j]
            if it[1] == "label":
                # fall-through into this label plus branches to it
                for pk in preds.get(j, []):
                    if (pk, waits) not in seen and depth < 8:
                        seen.add((pk, waits))
                        for w in back(pk + 1, need - waits, depth + 1, seen):
                            out.append((w[0], w[1], w[2] + waits))
                j -= 1
                continue
            op = it[2]
            if op.startswith("s_nop"):
                waits += int(it[3].strip() or 0) + 1
            else:
                if op.startswith("v_"):
                    dst = it[3].split(",")[0]
                    out.append((regs_of(dst), it[0], waits))
                waits += 1
                if op.startswith("s_branch") or op.startswith("s_setpc"):
                    break
            j -= 1
        return out

    nd = nh = 0
    for k, it in enumerate(seq):
        if it[1] != "ins":
            continue
        ops = it[3]
        if not ("_dpp" in it[2] or "quad_perm" in ops or "row_" in ops):
            continue
        nd += 1
        srcs = ops.split(",")[1:]
        src0 = regs_of(srcs[0]) if srcs else set()
        for wr, wl, w in back(k, 2):
            if wr & src0:
                nh += 1
                print(f"{fname[:60]} line {it[0]}: DPP reads v{sorted(wr & src0)} written at line {wl} with {w} wait states")
    print(f"{fname[:80]}: {nd} DPP instructions, {nh} hazards")
