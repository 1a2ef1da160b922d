#!/usr/bin/env python3
"""Static check for the register-allocation fault behind the max-ILP physics_kernel miscompute.

At the join block of a lane-divergent ``if`` the compiler restores the wave's exec mask with
``s_or_b64 exec, exec, s[..]`` (the lowered end-of-region). When register pressure makes the
allocator split a live range at such a join, it can place the split copies (``v_accvgpr_write``
/ ``v_mov_b32`` / scratch spill stores) at the top of the block, BEFORE the exec restore: they then
run with the region's narrower mask, and the lanes outside the region are never copied. A later
full-mask copy back hands those lanes stale values (lanes 14-15 of every team lost
their LDS row address, so the line search's |s|^2 / s.Ma / s.f / s.Ms sums were wrong).

Usage: isa_exec_check.py <file.s | lib.so> ...   (a .so is disassembled with llvm-objdump)
Prints every block whose prologue moves a register to/from an AGPR or scratch before its exec
restore; exit status 1 if any is found."""
import os
import re
import subprocess
import sys
import tempfile

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
BUNDLER = "/opt/rocm/lib/llvm/bin/clang-offload-bundler"

EXEC_RESTORE = re.compile(r"^s_or_b(64|32)\s+exec\s*,\s*exec\s*,|^s_or_saveexec_b(64|32)\s+s\[\d+:\d+\]\s*,\s*s\[")
LABEL = re.compile(r"^(\.LBB\d+_\d+|[A-Za-z_.$][\w.$]*):")
WRITES_VREG = re.compile(r"^(v_\w+)\s+(v\d+|a\d+|v\[\d+:\d+\]|a\[\d+:\d+\])")
# register-allocator moves: live-range splits and spills to/from AGPRs or scratch. A v_mov there can
# be a legitimate phi copy of the region (only the region's lanes take the new value), an AGPR or
# scratch move cannot: it exists to carry a value every lane needs
RA_MOVE = re.compile(r"^(v_accvgpr_write_b32|v_accvgpr_read_b32|v_accvgpr_mov_b32|scratch_store|scratch_load|buffer_store|buffer_load)")


def code_objects(path):
    """gfx950 code objects of a HIP fat binary (.so) as disassembly text."""
    out = []
    with tempfile.TemporaryDirectory() as tmp:
        blob = subprocess.run([OBJDUMP, "-h", path], capture_output=True, text=True).stdout
        if ".hip_fatbin" not in blob:
            return out
        fat = os.path.join(tmp, "fat.bin")
        subprocess.check_call(["/opt/rocm/lib/llvm/bin/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", path])
        data = open(fat, "rb").read()
        # one clang-offload-bundle per translation unit; unbundle each
        starts = [m.start() for m in re.finditer(rb"__CLANG_OFFLOAD_BUNDLE__", data)]
        for k, s in enumerate(starts):
            e = starts[k + 1] if k + 1 < len(starts) else len(data)
            b = os.path.join(tmp, f"b{k}.bin")
            open(b, "wb").write(data[s:e])
            co = os.path.join(tmp, f"co{k}.o")
            r = subprocess.run([BUNDLER, "--unbundle", "--type=o", f"--input={b}", f"--output={co}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], capture_output=True)
            if r.returncode != 0 or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            dis = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", "--mcpu=gfx950", co], capture_output=True,
                                 text=True).stdout
            out.append(with_block_labels(dis))
    return out


def with_block_labels(dis):
    """llvm-objdump prints branch targets as <func+0xoff>; put a '.LBBaddr:' line before every target
    instruction so that the scanner sees the block starts the assembler output would show."""
    funcs = {m.group(2): int(m.group(1), 16) for m in re.finditer(r"^([0-9a-f]+) <(\S+)>:$", dis, re.M)}
    targets = set()
    for m in re.finditer(r"s_c?branch\w*\s+\S+\s+//.*<(\S+)\+0x([0-9a-f]+)>", dis):
        if m.group(1) in funcs:
            targets.add(funcs[m.group(1)] + int(m.group(2), 16))
    out = []
    for line in dis.split("\n"):
        m = re.search(r"// ([0-9A-F]{12}):", line)
        if m and int(m.group(1), 16) in targets:
            out.append(f".LBB{int(m.group(1), 16):x}:")
        out.append(line.split("//")[0])
    return "\n".join(out)


def scan(text, name):
    bad = []
    lines = text.split("\n")
    func = "?"
    i = 0
    while i < len(lines):
        raw = lines[i].strip()
        m = re.match(r"^([0-9a-f]+ )?<(_Z\S+)>:$", raw) or re.match(r"^(_Z\S+):", raw)
        if m:
            func = m.group(2) if m.lastindex and m.lastindex >= 2 else m.group(1)
        if LABEL.match(raw) or re.match(r"^[0-9a-f]+ <\S+>:$", raw):
            # block prologue: instructions up to the first exec restore (or a non-copy)
            pre = []
            j = i + 1
            while j < len(lines) and j < i + 40:
                ins = lines[j].split(";")[0].split("//")[0].strip()
                ins = re.sub(r"^[0-9a-f]+:\s*", "", ins)
                j += 1
                if not ins or ins.startswith(".") or ins.startswith(";"):
                    continue
                if LABEL.match(ins):
                    break
                if EXEC_RESTORE.match(ins):
                    moves = [x for x in pre if RA_MOVE.match(x)]
                    if moves:
                        bad.append((name, func, i + 1, moves, ins))
                    break
                if WRITES_VREG.match(ins) or RA_MOVE.match(ins):
                    pre.append(ins)
                    continue
                break  # anything else ends the prologue: the restore (if any) is not at the block top
        i += 1
    return bad


def main():
    found = []
    for p in sys.argv[1:]:
        texts = code_objects(p) if p.endswith(".so") else [open(p).read()]
        for t in texts:
            found += scan(t, os.path.basename(p))
    for name, func, line, pre, ins in found:
        print(f"{name}: {func[:70]} line {line}: {len(pre)} register write(s) before '{ins}': {pre[:3]}")
    print(f"{len(found)} block(s) with register writes ahead of the exec restore")
    return 1 if found else 0


if __name__ == "__main__":
    sys.exit(main())
