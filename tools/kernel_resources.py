"""Registers / spills / scratch of the render kernels in a HIP object (code-object metadata):
    python tools/kernel_resources.py cuda-raytracing_amd/build/rt_fast_prod.hip.o [filter]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM_BIN = "/opt/rocm/lib/llvm/bin"


def resources(obj):
    with tempfile.TemporaryDirectory() as td:
        fat, co = os.path.join(td, "fat.bin"), os.path.join(td, "dev.co")
        subprocess.run([f"{LLVM_BIN}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(td, "x.o")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM_BIN}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--input={fat}", f"--output={co}", "--unbundle"], check=True, capture_output=True)
        notes = subprocess.run([f"{LLVM_BIN}/llvm-readelf", "--notes", co], check=True, capture_output=True, text=True).stdout
    out = []
    for blk in re.split(r"\n\s+- \.agpr_count", notes)[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        g = lambda k: int(re.search(r"\." + k + r":\s+(\d+)", blk).group(1))
        out.append((name, g("vgpr_count"), g("vgpr_spill_count"), g("sgpr_spill_count"), g("private_segment_fixed_size")))
    return out


if __name__ == "__main__":
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, v, vs, ss, priv in resources(sys.argv[1]):
        if flt in name:
            print(f"{name[:64]:64s} vgpr {v:3d} vgpr_spill {vs:4d} sgpr_spill {ss:4d} scratch {priv:4d} B")
