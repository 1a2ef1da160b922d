#!/usr/bin/env python3
"""Which stages' cross-statement FMA contractions make the flat latency / paired kernels differ from the
throughput kernel (CPU build step; tools/lat_bitcmp.py compares on the GPU). -ffp-contract=on everywhere
makes them bit-identical (profiles/r05_lat_bitcmp.txt) at a C2 cost; this builds flat-only libraries
build/libduck_fpc_<name>.so in which `#pragma clang fp contract(on)` opens every function body of the
named line groups of duck_team.h (a temporary copy of csrc/; the shipped sources are not touched).
usage: python tools/fpc_bisect.py NAME:G1,G4 NAME2:G2 ..."""
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from open_duck_playground_amd import codegen, native  # noqa: E402

# function-definition line groups of duck_team.h, by the first and last definition name
GROUPS = {"G1": ("body_pose", "root_motion"), "G2": ("rne", "crb"), "G3": ("smooth", "smooth"),
          "G4": ("bc", "smooth_solve"), "G5": ("mul_acc", "newton_fused"), "G6": ("cgeom_frame", "collision"),
          "G7": ("make_rows", "quad2"), "G8": ("solve", "warm_start"), "G9": ("newton", "newton"),
          "G10": ("sensors", "euler")}


def mark(src: str, groups) -> str:
    lines = src.split("\n")
    defs = [(i, m.group(1)) for i, l in enumerate(lines)
            for m in [re.match(r"^  static DK [\w:<>, ]+?\b(\w+)\(", l)] if m]
    on = set()
    for g in groups:
        if g.startswith("f="):  # single functions: f=name1+name2
            on |= {i for i, n in defs if n in g[2:].split("+")}
            continue
        a, b = GROUPS[g]
        ia = next(i for i, n in defs if n == a)
        ib = max(i for i, n in defs if n == b)
        on |= {i for i, n in defs if ia <= i <= ib}
    out = list(lines)
    for i in sorted(on, reverse=True):
        j = i
        while not out[j].rstrip().endswith("{"):
            j += 1
        out.insert(j + 1, "#pragma clang fp contract(on)")
    return "\n".join(out)


def build(name: str, groups) -> str:
    tmp = tempfile.mkdtemp()
    cs = os.path.join(tmp, "pkg", "csrc")
    shutil.copytree(native.CSRC, cs)
    inc_root = os.path.join(tmp, "include")
    shutil.copytree(os.path.join(ROOT, "include"), inc_root)
    p = os.path.join(cs, "duck_team.h")
    marked = mark(open(p).read(), groups)
    open(p, "w").write(marked)
    gen = os.path.join(tmp, "gen")
    os.makedirs(gen)
    open(os.path.join(gen, "duck_variants.inc"), "w").write(codegen.variant_registry(["flat"]))
    shutil.copy(os.path.join(cs, "generated", "duck_model_flat.h"), gen)
    open(os.path.join(gen, "variant_flat.hip"), "w").write(codegen.variant_unit("flat", "duck_model_flat.h"))
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-fno-hip-fp32-correctly-rounded-divide-sqrt",
             "-fgpu-flush-denormals-to-zero", "-fno-slp-vectorize", "-fno-signed-zeros", "-fno-trapping-math",
             "-fno-math-errno", "-freciprocal-math", "-I" + cs, "-I" + gen] + native.ILP_FLAGS + \
        [f'-DDUCK_BUILD_ID="fpc_{name}"']
    objs = []
    for src in (os.path.join(cs, "duck_capi.hip"), os.path.join(gen, "variant_flat.hip")):
        o = src + ".o"
        subprocess.check_call(["hipcc"] + flags + ["-c", "-o", o, src], cwd=cs)
        objs.append(o)
    out = os.path.join(native.BUILD, f"libduck_fpc_{name}.so")
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-shared", "-o", out] + objs)
    shutil.rmtree(tmp)
    return out


if __name__ == "__main__":
    from concurrent.futures import ThreadPoolExecutor
    jobs = [(a.split(":")[0], [g for g in a.split(":")[1].split(",") if g]) for a in sys.argv[1:]]
    with ThreadPoolExecutor(max_workers=4) as ex:
        for out in ex.map(lambda j: build(*j), jobs):
            print("built", out)
