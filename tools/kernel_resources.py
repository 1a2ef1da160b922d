#!/usr/bin/env python3
"""Register / LDS / scratch use of every step kernel in a HIP fat binary (CPU only): the code objects'
AMDGPU metadata notes (.vgpr_count, .agpr_count, .sgpr_spill_count, .vgpr_spill_count,
.private_segment_fixed_size, .group_segment_fixed_size). usage: python tools/kernel_resources.py [lib.so] [name substring, default step_kernel]"""
import os
import re
import subprocess
import sys
import tempfile

BUNDLER = "/opt/rocm/lib/llvm/bin/clang-offload-bundler"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def main():
    match = sys.argv[2] if len(sys.argv) > 2 else "step_kernel"
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "open_duck_playground_amd", "libduck.so")
    with tempfile.TemporaryDirectory() as tmp:
        fat = os.path.join(tmp, "fat.bin")
        subprocess.check_call(["/opt/rocm/lib/llvm/bin/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", path])
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(rb"__CLANG_OFFLOAD_BUNDLE__", data)]
        for k, s in enumerate(starts):
            e = starts[k + 1] if k + 1 < len(starts) else len(data)
            b, co = os.path.join(tmp, f"b{k}.bin"), os.path.join(tmp, f"co{k}.o")
            open(b, "wb").write(data[s:e])
            r = subprocess.run([BUNDLER, "--unbundle", "--type=o", f"--input={b}", f"--output={co}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], capture_output=True)
            if r.returncode or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            notes = subprocess.run([READELF, "--notes", co], capture_output=True, text=True).stdout
            for blk in re.split(r"\n\s+- \.agpr_count", notes)[1:]:
                blk = ".agpr_count" + blk
                name = re.search(r"\.name:\s+(\S+)", blk)
                if not name or match not in name.group(1):
                    continue
                f = {k: re.search(rf"\.{k}:\s+(\S+)", blk) for k in
                     ("agpr_count", "vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                      "private_segment_fixed_size", "group_segment_fixed_size")}
                print(name.group(1)[:60], {k: (v.group(1) if v else None) for k, v in f.items()})


if __name__ == "__main__":
    main()
