"""CPU-side checks of the drop-in boundary: libsacx.so loads and exports every
symbol include/sacx.h declares; the ctypes structs match the C layout.  No
compute calls (no GPU needed)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "sacx.h")).read()
    return sorted(set(re.findall(r"\b(sacx_[a-z_]+)\s*\(", txt)))


def test_library_exports_header_symbols():
    from sac_eo import _native as N
    L = N.lib()
    syms = _header_symbols()
    assert len(syms) >= 16
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(N.EXPORTS) == syms


def test_struct_layouts():
    from sac_eo import _native as N
    # offsets fixed by include/sacx.h (natural alignment)
    assert N.Config.buffer_capacity.offset == 32
    assert ctypes.sizeof(N.Config) == 392          # gcc: sizeof(sacx_config) (ABI 8)
    assert N.Config.gaussian_model.offset == 208 and N.Config.reward_hidden.offset == 220
    assert N.Config.reward_act_layers.offset == 228 and N.Config.critic_hidden.offset == 236
    assert N.Config.act_per_layer.offset == 172 and N.Config.act_layers.offset == 176
    assert N.Config.delta_clip_pred.offset == 200 and N.Config.single_seed_plan.offset == 204
    assert N.Config.reward_loss_coef.offset == 128
    assert N.Config.gemm_bf16.offset == 132
    assert N.Config.seeds.offset == 136
    assert N.Config.actor_gaussian.offset == 140 and N.Config.num_models.offset == 156
    assert N.Config.reward_clip_loss.offset == 168
    assert ctypes.sizeof(N.Segment) == 48 + 8 + 8 + 8 + 4 + 4
    assert ctypes.sizeof(N.LaunchInfo) == 32 + 32 + 4 + 4 + 8 + 8


def test_create_validates_without_gpu():
    """sacx_create / layout are host-only; bad configs fail with a message."""
    from sac_eo import _native as N
    from sac_eo.engine import EngineConfig
    L = N.lib()
    h = ctypes.c_void_p()
    c = EngineConfig(s_dim=17, a_dim=6).to_c()
    assert L.sacx_create(ctypes.byref(c), ctypes.byref(h)) == 0
    n = ctypes.c_int32()
    L.sacx_layout(h, None, 0, ctypes.byref(n))
    segs = (N.Segment * n.value)()
    L.sacx_layout(h, segs, n.value, ctypes.byref(n))
    names = {s.name.decode(): s for s in segs}
    for k in ("actor.l0", "q0.l2", "t1.l1", "alpha", "adam_m", "adam_v", "replay", "rng", "ctl"):
        assert k in names
    assert names["actor.l0"].rows == 18 and names["actor.l0"].cols == 256     # [W;b] Keras layout
    assert names["replay"].rows == 1_000_000 and names["replay"].cols == 44
    assert L.sacx_arena_bytes(h) > 176_000_000
    L.sacx_destroy(h)
    bad = EngineConfig(s_dim=17, a_dim=6, use_expert=True, expert_batch=7).to_c()
    assert L.sacx_create(ctypes.byref(bad), ctypes.byref(h)) != 0
    assert b"even" in L.sacx_last_error(None)


def test_packed_seed_layout_without_gpu():
    """cfg.seeds = K: K arena blocks of one seed's layout, 64 KiB-aligned stride."""
    from sac_eo import _native as N
    from sac_eo.engine import EngineConfig
    L = N.lib()
    h1, h3 = ctypes.c_void_p(), ctypes.c_void_p()
    c1 = EngineConfig(s_dim=17, a_dim=6, buffer_capacity=10_000).to_c()
    c3 = EngineConfig(s_dim=17, a_dim=6, buffer_capacity=10_000, seeds=3).to_c()
    assert L.sacx_create(ctypes.byref(c1), ctypes.byref(h1)) == 0
    assert L.sacx_create(ctypes.byref(c3), ctypes.byref(h3)) == 0
    one = L.sacx_arena_bytes(h1)
    assert L.sacx_seed_stride(h1) == one
    st = L.sacx_seed_stride(h3)
    assert st % 65536 == 0 and one <= st < one + 65536
    assert L.sacx_arena_bytes(h3) == 3 * st
    # seed selection needs a bound arena
    assert L.sacx_seed_select(h3, 1) != 0
    L.sacx_destroy(h1)
    L.sacx_destroy(h3)
    bad = EngineConfig(s_dim=17, a_dim=6, seeds=65).to_c()
    assert L.sacx_create(ctypes.byref(bad), ctypes.byref(h1)) != 0
    assert b"seeds" in L.sacx_last_error(None)


def test_no_kernel_uses_kilobytes_of_scratch():
    """Build guard (tools/check_scratch.py): every gfx950 kernel in libsacx.so keeps its
    private segment small -- kilobytes there mean a spilled / copied kernel-argument block."""
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = os.path.join(root, "sac-expert_amd", "lib", "libsacx.so")
    if not os.path.exists("/opt/rocm/lib/llvm/bin/clang-offload-bundler") or not os.path.exists(so):
        pytest.skip("ROCm LLVM tools or libsacx.so absent")
    sys.path.insert(0, os.path.join(root, "tools"))
    from check_scratch import kernel_scratch
    sizes = kernel_scratch(so)
    assert len(sizes) > 50
    bad = {k: v for k, v in sizes.items() if v > 256}
    assert not bad, bad


def test_config_layout_matches_gcc(tmp_path):
    """Every sacx_config field offset of the ctypes mirror equals gcc's offsetof on include/sacx.h."""
    import os
    import shutil
    import subprocess
    from sac_eo import _native as N
    if shutil.which("gcc") is None:
        pytest.skip("gcc not on PATH")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    names = [f[0] for f in N.Config._fields_]
    src = tmp_path / "lay.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "sacx.h"\nint main(void) {\n'
                   + "".join(f'  printf("%zu\\n", offsetof(sacx_config, {n}));\n' for n in names)
                   + '  printf("%zu\\n", sizeof(sacx_config));\n  return 0;\n}\n')
    exe = tmp_path / "lay"
    subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(root, "include"), str(src), "-o", str(exe)])
    got = [int(x) for x in subprocess.check_output([str(exe)], text=True).split()]
    want = [getattr(N.Config, n).offset for n in names] + [ctypes.sizeof(N.Config)]
    assert got == want, list(zip(names + ["sizeof"], got, want))


def test_launch_header_round_trip(tmp_path):
    """The k_gemm / k_dwl launch header (sacx_internal.h KHdr: the workgroup-role scalars packed
    into 4 preloaded dwords) decodes to the GemmArgs values it was built from, and is marked
    invalid when a value does not fit (the kernels then read GemmArgs)."""
    import os
    import shutil
    import subprocess
    if shutil.which("g++") is None:
        pytest.skip("g++ not on PATH")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = tmp_path / "khdr"
    subprocess.check_call(["g++", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                           "-I", os.path.join(root, "include"), "-I", os.path.join(root, "sac-expert_amd", "csrc"),
                           os.path.join(root, "tests", "khdr_check.cpp"), "-o", str(exe)])
    out = subprocess.check_output([str(exe)], text=True)
    assert "0 mismatches" in out, out


def test_mt_jump_windows(tmp_path):
    """The segmented sampler's jump-ahead (csrc/mt_jump.cpp: MT19937's characteristic polynomial
    by Berlekamp-Massey, x^(kL) mod phi): the 624-word windows k L + 1 .. k L + 624 rebuilt as
    XORs of the words after a key block equal the directly generated stream (3 segment lengths,
    k = 1 .. 4)."""
    import os
    import shutil
    import subprocess
    if shutil.which("g++") is None:
        pytest.skip("g++ not on PATH")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    csrc = os.path.join(root, "sac-expert_amd", "csrc")
    exe = tmp_path / "mtj"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", csrc, os.path.join(root, "tests", "mtjump_check.cpp"),
                           os.path.join(csrc, "mt_jump.cpp"), "-o", str(exe)])
    out = subprocess.check_output([str(exe)], text=True)
    assert " 0 mismatches" in out, out
