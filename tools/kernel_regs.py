"""Per-kernel register / LDS use of the gfx950 code object in libsacx.so (diagnostic):
VGPRs bound the waves per SIMD (512 / vgpr_count), hence how many workgroups of a launch
run at once.

usage: python tools/kernel_regs.py [path/to/libsacx.so] [substring of the mangled name]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_resources(so_path):
    with tempfile.TemporaryDirectory() as d:
        fat, dev = os.path.join(d, "fat.bin"), os.path.join(d, "dev.o")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", so_path,
                               os.path.join(d, "copy.so")])
        subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}", f"--output={dev}"])
        notes = subprocess.check_output([f"{LLVM}/llvm-readelf", "--notes", dev], text=True)
    # one YAML list item per kernel ("  - .agpr_count: ..."); keys before and after .name belong to it
    out, cur = {}, None
    for line in notes.splitlines():
        if re.match(r"\s{2}- \.", line):
            cur = {}
        if cur is None:
            continue
        m = re.match(r"\s*-?\s*\.name:\s+(\S+)", line)
        if m:
            out[m.group(1)] = cur
        for key in ("vgpr_count", "agpr_count", "sgpr_count", "group_segment_fixed_size"):
            m = re.match(r"\s*-?\s*\.%s:\s+(\d+)" % key, line)
            if m:
                cur[key] = int(m.group(1))
    return out


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "sac-expert_amd", "lib", "libsacx.so")
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    for n, v in sorted(kernel_resources(so).items()):
        if pat in n:
            vg = v.get("vgpr_count", 0)
            print(f"{n:70s} vgpr {vg:4d} agpr {v.get('agpr_count', 0):3d} lds {v.get('group_segment_fixed_size', 0):6d}"
                  f"  waves/SIMD {min(8, 512 // max(vg, 1))}")


if __name__ == "__main__":
    main()
