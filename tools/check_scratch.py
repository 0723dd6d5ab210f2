"""Build guard: no gfx950 kernel in libsacx.so may use more than a few bytes of scratch.

A kernel whose private segment grows to kilobytes has spilled or copied a large aggregate
(e.g. the kernel-argument block) into scratch memory; on the update chain that is a silent
2-3x slowdown (round 2: a chain of selects over the Adam learning rates made the 32x32 dW
variants copy all of GemmArgs, 3,280 B per lane, and halved the packed Humanoid rate).
The check unbundles the gfx950 code object from the .hip_fatbin section and reads each
kernel's .private_segment_fixed_size from its metadata notes.

It also bounds the VGPRs a kernel spills (.vgpr_spill_count): round 3 found the bf16 32x32
forward / dX tiles spilling 12-80 registers at 6 workgroups per CU (36-136 B per lane, under the
byte limit) and running 17 % slower for it.  The default bound, 20, admits the fp32 32x32 dX
tiles with the Q-head rows (17-18 spilled at 6 workgroups per CU; 5 per CU, without the spill,
measured neutral).

usage: python tools/check_scratch.py [path/to/libsacx.so] [max_bytes] [max_spilled_vgprs]
       (exit 1 on a violation)
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_scratch(so_path):
    """{kernel symbol: private segment bytes per lane} of the gfx950 code object in so_path."""
    with tempfile.TemporaryDirectory() as d:
        fat, dev = os.path.join(d, "fat.bin"), os.path.join(d, "dev.o")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", so_path,
                               os.path.join(d, "copy.so")])
        subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}", f"--output={dev}"])
        notes = subprocess.check_output([f"{LLVM}/llvm-readelf", "--notes", dev], text=True)
    out, spills, name = {}, {}, None
    for line in notes.splitlines():
        m = re.match(r"\s*\.name:\s+(\S+)", line)
        if m:
            name = m.group(1)
        m = re.match(r"\s*\.private_segment_fixed_size:\s+(\d+)", line)
        if m and name:
            out[name] = int(m.group(1))
        m = re.match(r"\s*\.vgpr_spill_count:\s+(\d+)", line)
        if m and name:
            spills[name] = int(m.group(1))
    kernel_scratch.spills = spills
    return out


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "sac-expert_amd", "lib", "libsacx.so")
    limit = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    max_spill = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    sizes = kernel_scratch(so)
    bad = {k: v for k, v in sizes.items() if v > limit}
    for k, v in sorted(bad.items()):
        print(f"scratch {v} B/lane > {limit}: {k}")
    spilled = {k: v for k, v in kernel_scratch.spills.items() if v > max_spill}
    for k, v in sorted(spilled.items()):
        print(f"{v} VGPRs spilled > {max_spill}: {k}")
    print(f"check_scratch: {len(sizes)} kernels, {len(bad)} over {limit} B/lane, {len(spilled)} spilling > {max_spill} VGPRs")
    return 1 if bad or spilled or not sizes else 0


if __name__ == "__main__":
    sys.exit(main())
