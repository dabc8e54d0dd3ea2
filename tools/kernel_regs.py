"""VGPR / AGPR / spill / LDS of the library's kernels whose name contains a
pattern (the gfx950 code object's metadata notes).

    python tools/kernel_regs.py k_transform
"""
import os
import re
import subprocess
import sys
import tempfile

from korali_amd import _build

LLVM = "/opt/rocm/lib/llvm/bin"


def main():
    pat = sys.argv[1] if len(sys.argv) > 1 else ""
    d = tempfile.mkdtemp()
    fat, co = os.path.join(d, "f"), os.path.join(d, "c")
    subprocess.check_call(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", _build.LIB, fat])
    subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
    out = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    for blk in out.split(".name:")[1:]:
        name = blk.split("\n")[0].strip()
        if pat in name:
            get = lambda k: (re.search(rf"\.{k}:\s+(\d+)", blk) or [None, "?"])[1]
            print(f"{name[:70]:70s} vgpr {get('vgpr_count'):>4} agpr {get('agpr_count'):>4} "
                  f"spill {get('vgpr_spill_count')} lds {get('group_segment_fixed_size')}")


if __name__ == "__main__":
    main()
