"""CPU-side checks of the C-ABI boundary: the library loads (no GPU needed) and
exports exactly the entry points include/vitmi.h declares; host validation
rejects bad shapes before any launch."""
import os
import re

import pytest

from vitmi import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "vitmi.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vitmi_[a-z0-9_]+)\s*\(", src)))


def test_header_matches_loader_table():
    assert header_functions() == sorted(_lib.exported_symbols())


def test_library_exports_every_symbol():
    lib = _lib.lib()
    for name in header_functions():
        assert hasattr(lib, name), name
    assert lib.vitmi_version() >= 100


def test_host_validation_rejects_bad_shapes():
    lib = _lib.lib()
    # k-major operand with K % 64 != 0 (bf16) must fail before any launch
    rc = lib.vitmi_gemm(1, 1, 1, 128, 128, 100, 16, 128, 16, 128, 16, 128, 1, 0, None, None, 0, None, 0,
                        None, 0, None)
    assert rc == 1
    assert b"K %" in lib.vitmi_last_error() or b"K " in lib.vitmi_last_error()
    # attention head dim must be 64
    rc = lib.vitmi_attention_fwd(1, 1, 10, 2, 32, 1.0, 16, 16, 16, None)
    assert rc == 1 and b"64" in lib.vitmi_last_error()
    # layernorm D must be a multiple of 4
    rc = lib.vitmi_layernorm_fwd(4, 30, 16, 30, 16, 16, 1e-6, 16, 0, 30, 16, 16, None)
    assert rc == 1


def test_precision_knob_entry_points_validate_on_the_host():
    """The split-operand paths of the bf16x3 knob reject bad arguments before any launch."""
    lib = _lib.lib()
    # VITMI_BF16X3 LayerNorm output needs ldy >= 3D
    rc = lib.vitmi_layernorm_fwd(4, 64, 16, 64, 16, 16, 1e-6, 16, 3, 64, 16, 16, None)
    assert rc == 1 and b"3D" in lib.vitmi_last_error()
    # an unknown LayerNorm output dtype
    rc = lib.vitmi_layernorm_fwd(4, 64, 16, 64, 16, 16, 1e-6, 16, 7, 64, 16, 16, None)
    assert rc == 1 and b"dtype" in lib.vitmi_last_error()
    # the x3 attention forward serves the whole-sequence kernels only (N <= 256)
    rc = lib.vitmi_attention_fwd_x3(1, 300, 2, 64, 0.125, 16, 16, 16, 16, None)
    assert rc == 1 and b"256" in lib.vitmi_last_error()
    # VITMI_EPI_SPLIT_X3 only with the bias+GELU epilogue, and the 3N-wide output row of linear_fwd
    rc = lib.vitmi_gemm(1, 1, 1, 128, 128, 128, 16, 128, 16, 128, 16, 128, 1, 0x200, None, None, 0, None, 0,
                        None, 0, None)
    assert rc == 1 and b"SPLIT_X3" in lib.vitmi_last_error()
    rc = lib.vitmi_gemm(1, 1, 1, 128, 128, 128, 16, 128, 16, 128, 16, 128, 1, 0x201, None, 16, 128, None, 0,
                        None, 0, None)
    assert rc == 1 and b"3N" in lib.vitmi_last_error()
    # split_bf16x3: K % 4 and the pattern
    assert lib.vitmi_split_bf16x3(4, 6, 16, 6, 16, 18, 0, None, 0, None) == 1
    assert lib.vitmi_split_bf16x3(4, 8, 16, 8, 16, 24, 2, None, 0, None) == 1


def test_bf16f8_knob_entry_points_validate_on_the_host():
    """The VITMI_BF16F8 paths (the knob's e4m3-correction form) reject bad arguments before any launch."""
    lib = _lib.lib()
    # LayerNorm VITMI_BF16F8 output rows are 2D bf16 units
    rc = lib.vitmi_layernorm_fwd(4, 64, 16, 64, 16, 16, 1e-6, 16, 4, 64, 16, 16, None)
    assert rc == 1 and b"2D" in lib.vitmi_last_error()
    # linear_fwd on VITMI_BF16F8 operands: K % 64 and N % 16
    rc = lib.vitmi_linear_fwd(4, 128, 128, 96, 16, 16, None, 16, 0, 0, None, None, None, 0, None)
    assert rc == 1 and b"K % 64" in lib.vitmi_last_error()
    rc = lib.vitmi_linear_fwd(4, 128, 120, 128, 16, 16, None, 16, 0, 0, None, None, None, 0, None)
    assert rc == 1 and b"N % 16" in lib.vitmi_last_error()
    # VITMI_EPI_SPLIT_F8 needs VITMI_BF16F8 operands
    rc = lib.vitmi_linear_fwd(1, 128, 128, 128, 16, 16, None, 16, 1, 0x401, 16, None, None, 0, None)
    assert rc == 1 and b"SPLIT_F8" in lib.vitmi_last_error()
    # the generic GEMM entry (wgrad-style split) does not take them
    rc = lib.vitmi_gemm(4, 1, 1, 128, 128, 128, 16, 256, 16, 256, 16, 128, 0, 4, None, None, 0, None, 0,
                        None, 0, None)
    assert rc == 1 and b"BF16F8" in lib.vitmi_last_error()
    # split_bf16f8: K % 64, ld_dst >= 2K and the pattern
    assert lib.vitmi_split_bf16f8(4, 8, 16, 8, 16, 16, 0, None, 0, None) == 1
    assert lib.vitmi_split_bf16f8(4, 64, 16, 64, 16, 96, 0, None, 0, None) == 1
    assert lib.vitmi_split_bf16f8(4, 64, 16, 64, 16, 128, 2, None, 0, None) == 1
    # LayerNorm VITMI_BF16F8 output needs D % 64
    rc = lib.vitmi_layernorm_fwd(4, 96, 16, 96, 16, 16, 1e-6, 16, 4, 192, 16, 16, None)
    assert rc == 1 and b"64" in lib.vitmi_last_error()
    import ctypes
    one = (ctypes.c_int64 * 1)(96)
    ptr = (ctypes.c_void_p * 1)(16)
    assert lib.vitmi_split_bf16f8_weights(0, ptr, ptr, one, one, None) == 1            # n in 1..8
    assert lib.vitmi_split_bf16f8_weights(1, ptr, ptr, one, one, None) == 1            # K % 64
    rc = lib.vitmi_attention_fwd_f8(1, 300, 2, 64, 0.125, 16, 16, 16, 16, None)
    assert rc == 1 and b"256" in lib.vitmi_last_error()


def test_workspace_queries_are_pure_host():
    lib = _lib.lib()
    assert lib.vitmi_attention_bwd_workspace_size(2, 197, 12) == 2 * 197 * 12 * 4
    assert lib.vitmi_linear_wgrad_workspace_size(1, 50432, 768, 768) > 0
    assert lib.vitmi_bias_grad_workspace_size(50432, 768) > 0
    # the grouped weight gradients of a ViT-B block: 108 tiles -> 7 slabs each (756 units on 3
    # rounds of 256 CUs), 7 x (4 x 768 x 3072 / 2 + 768 x 768 + 2304 x 768) fp32 partials
    import ctypes
    Ns = (ctypes.c_int64 * 4)(768, 3072, 768, 2304)
    Ks = (ctypes.c_int64 * 4)(3072, 768, 768, 768)
    need = lib.vitmi_linear_wgrad_group_workspace_size(1, 4, 50432, Ns, Ks)
    assert need == 7 * (2 * 768 * 3072 + 768 * 768 + 2304 * 768) * 4
    assert lib.vitmi_linear_wgrad_group_workspace_size(1, 5, 50432, Ns, Ks) == 0     # n > 4
    assert lib.vitmi_linear_wgrad_group(1, 5, 50432, Ns, Ks, None, None, None, None, None, None, 0, None) == 1


def test_wgrad_group_rejects_bad_arguments():
    import ctypes
    lib = _lib.lib()
    Ns = (ctypes.c_int64 * 2)(768, 768)
    Ks = (ctypes.c_int64 * 2)(768, 768)
    # null operand arrays
    assert lib.vitmi_linear_wgrad_group(1, 2, 1000, Ns, Ks, None, None, None, None, None, None, 0, None) == 1
    assert b"null" in lib.vitmi_last_error()
    # nothing to do
    assert lib.vitmi_linear_wgrad_group(1, 0, 1000, None, None, None, None, None, None, None, None, 0, None) == 0


@pytest.mark.parametrize("name", ["vitmi_gemm", "vitmi_attention_fwd", "vitmi_layernorm_bwd"])
def test_argtypes_declared(name):
    fn = getattr(_lib.lib(), name)
    assert fn.argtypes is not None and len(fn.argtypes) > 5


def test_build_id_matches_sources_and_flags():
    """the .so was built from the csrc/ + include/ in this tree (a stale library is caught), and
    its id carries the hash of the compiler command line it reports (a -D variant differs)"""
    want = _lib.source_build_id()
    assert want is not None
    src, flags = _lib.build_id_parts(_lib.lib().vitmi_build_id().decode())
    assert src == want
    cmd = _lib.lib().vitmi_build_flags().decode()
    assert "--offload-arch=gfx950" in cmd and flags == _lib.flags_id(cmd)


def test_section8b_entry_points_exported():
    """the boundary exports vitmi_{patch_embed,layernorm,linear,attention,xent,
    mse}_{fwd,bwd} (+ workspace queries), the comm leg, vitmi_last_error and vitmi_version."""
    names = set(header_functions())
    for op in ("patch_embed", "layernorm", "linear", "attention", "xent", "mse"):
        for d in ("fwd", "bwd"):
            assert f"vitmi_{op}_{d}" in names, (op, d)
    for n in ("vitmi_patch_embed_fwd_workspace_size", "vitmi_patch_embed_bwd_workspace_size",
              "vitmi_linear_bwd_workspace_size", "vitmi_layernorm_bwd_workspace_size",
              "vitmi_attention_bwd_workspace_size", "vitmi_comm_init", "vitmi_comm_allreduce_async",
              "vitmi_comm_destroy", "vitmi_last_error", "vitmi_version"):
        assert n in names, n


def test_section8b_host_validation():
    lib = _lib.lib()
    # workspace queries are pure host arithmetic
    n = lib.vitmi_patch_embed_fwd_workspace_size(1, 256, 3, 224, 16, 768)
    assert n >= 256 * 196 * 768 * 4
    assert lib.vitmi_patch_embed_bwd_workspace_size(1, 256, 3, 224, 16, 768) >= 256 * 196 * 768 * 2
    assert lib.vitmi_linear_bwd_workspace_size(1, 50432, 768, 768) >= lib.vitmi_linear_wgrad_workspace_size(
        1, 50432, 768, 768)
    # too-small workspaces and bad shapes fail before any launch
    rc = lib.vitmi_patch_embed_fwd(1, 2, 3, 32, 8, 64, 16, 16, None, None, None, 16, 16, 16, 8, None)
    assert rc == 1 and b"workspace" in lib.vitmi_last_error()
    rc = lib.vitmi_patch_embed_fwd(1, 2, 3, 30, 8, 64, 16, 16, None, None, None, 16, 16, 16, 1 << 30, None)
    assert rc == 1 and b"shape" in lib.vitmi_last_error()
    rc = lib.vitmi_linear_bwd(1, 64, 64, 64, 16, 16, 16, 16, 1, 16, 16, 16, 8, None)
    assert rc == 1 and b"workspace" in lib.vitmi_last_error()
    assert lib.vitmi_xent_fwd(2, 2, 16, 16, None, None) == 1
    assert lib.vitmi_mse_bwd(2, 1, 16, 16, None, None) == 1
    # the bf16 GELU epilogue writes bf16: an fp32 C is rejected
    rc = lib.vitmi_gemm(1, 1, 1, 128, 128, 64, 16, 64, 16, 64, 16, 128, 0, 1, None, 16, 128, None, 0,
                        None, 0, None)
    assert rc == 1 and b"GELU" in lib.vitmi_last_error()


def test_comm_entry_points_validate_without_a_communicator():
    lib = _lib.lib()
    assert lib.vitmi_comm_destroy(0) == 0                      # nothing to destroy
    assert lib.vitmi_comm_check() == 0
    rc = lib.vitmi_comm_allreduce_async(16, 4, 0, 1, None, None)
    assert rc == 1 and b"no communicator" in lib.vitmi_last_error()
    rc = lib.vitmi_comm_init(2, 2, b"\0" * 128)                # rank out of range: host check
    assert rc == 1 and b"rank" in lib.vitmi_last_error()
    assert lib.vitmi_comm_get_unique_id(None) == 1


def test_policy_knobs_round_trip():
    lib = _lib.lib()
    prev = lib.vitmi_attention_set_policy(1)
    assert lib.vitmi_attention_set_policy(prev) == 1
    assert lib.vitmi_attention_set_policy(7) == 1              # out of range: rejected
    assert lib.vitmi_attention_set_policy(2) == prev           # the 32-query whole-sequence forms
    assert lib.vitmi_attention_set_policy(prev) == 2
    prev = lib.vitmi_gemm_set_reserved_cus(8)
    assert lib.vitmi_gemm_set_reserved_cus(prev) == 8
