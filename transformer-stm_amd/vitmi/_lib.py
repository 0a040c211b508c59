"""ctypes loader for libvitmi.so (the C ABI declared in include/vitmi.h).

torch is imported first on purpose: it loads its bundled ``libamdhip64.so``
(SONAME ``libamdhip64.so.7``), so the library's own DT_NEEDED on that SONAME
resolves to the SAME HIP runtime instance and torch's streams / device pointers
are valid inside the kernels.  There is no fallback: if the library is missing
every op raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
# VITMI_LIB: load another build of the same ABI (A/B timing of kernel variants)
LIB_PATH = os.environ.get("VITMI_LIB") or os.path.join(_HERE, "libvitmi.so")

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_int64
F = ctypes.c_float
D = ctypes.c_double
S = ctypes.c_size_t
U = ctypes.c_uint32

# name -> (restype, argtypes); mirrors include/vitmi.h one to one
SIGNATURES = {
    "vitmi_version": (I, []),
    "vitmi_build_id": (ctypes.c_char_p, []),
    "vitmi_build_flags": (ctypes.c_char_p, []),
    "vitmi_last_error": (ctypes.c_char_p, []),
    "vitmi_device_cus": (I, []),
    "vitmi_gemm": (I, [I, I, I, L, L, L, P, L, P, L, P, L, I, I, P, P, L, P, L, P, S, P]),
    "vitmi_gemm_workspace_size": (S, [I, I, I, L, L, L, I]),
    "vitmi_gemm_set_policy": (I, [I]),
    "vitmi_linear_fwd": (I, [I, L, L, L, P, P, P, P, I, I, P, P, P, S, P]),
    "vitmi_linear_fwd_workspace_size": (S, [I, L, L, L]),
    "vitmi_aux_tiled_bytes": (S, [L, L]),
    "vitmi_linear_dgrad": (I, [I, L, L, L, P, P, P, I, I, P, P, S, P]),
    "vitmi_linear_dgrad_workspace_size": (S, [I, L, L, L]),
    "vitmi_linear_wgrad": (I, [I, L, L, L, P, P, P, P, S, P]),
    "vitmi_linear_wgrad_workspace_size": (S, [I, L, L, L]),
    "vitmi_linear_wgrad_group": (I, [I, I, L, P, P, P, P, P, P, P, P, S, P]),
    "vitmi_linear_wgrad_group_workspace_size": (S, [I, I, L, P, P]),
    "vitmi_bias_grad": (I, [I, L, L, P, L, P, P, S, P]),
    "vitmi_bias_grad_workspace_size": (S, [L, L]),
    "vitmi_layernorm_fwd": (I, [L, I, P, L, P, P, F, P, I, L, P, P, P]),
    "vitmi_layernorm_bwd": (I, [L, I, P, I, L, P, L, P, P, P, P, L, P, L, P, L, P, P, P, P, S, P]),
    "vitmi_layernorm_bwd_workspace_size": (S, [L, I]),
    "vitmi_attention_fwd": (I, [I, I, I, I, I, F, P, P, P, P]),
    "vitmi_attention_fwd_x3": (I, [I, I, I, I, F, P, P, P, P, P]),
    "vitmi_attention_fwd_f8": (I, [I, I, I, I, F, P, P, P, P, P]),
    "vitmi_attention_bwd": (I, [I, I, I, I, I, F, P, P, P, P, P, P, S, P]),
    "vitmi_attention_bwd_workspace_size": (S, [I, I, I]),
    "vitmi_patch_im2col": (I, [I, I, I, I, I, P, P, P]),
    "vitmi_tokens_assemble": (I, [I, I, I, P, P, P, P, P]),
    "vitmi_tokens_assemble_bwd": (I, [I, I, I, P, P, P, P, P, P]),
    "vitmi_head_fwd": (I, [I, I, I, P, L, P, P, P, P]),
    "vitmi_head_bwd": (I, [I, I, I, P, P, L, P, P, P, P, P]),
    "vitmi_loss_fwd_bwd": (I, [I, I, I, P, P, P, P, P]),
    "vitmi_cast_f32_bf16": (I, [L, P, P, P]),
    "vitmi_split_bf16x3": (I, [L, L, P, L, P, L, I, P, L, P]),
    "vitmi_split_bf16f8": (I, [L, L, P, L, P, L, I, P, L, P]),
    "vitmi_split_bf16f8_weights": (I, [I, P, P, P, P, P]),
    "vitmi_split_bf16f8_weights_mixed": (I, [I, P, P, P, P, P, P]),
    "vitmi_fold_begin": (I, []),
    "vitmi_fold_end": (I, [P]),
    "vitmi_dropout_hash": (U, [U, U, U, U]),
    "vitmi_linear_fwd_dropout": (I, [I, L, L, L, P, P, P, P, I, I, P, P, P, S, U, U, U, F, P]),
    "vitmi_dropout_apply": (I, [L, L, P, L, P, I, L, U, U, U, F, P]),
    "vitmi_conv_same_geometry": (I, [I, I, I, I, I, P, P, P, P]),
    "vitmi_conv_im2col": (I, [I, I, I, I, I, I, I, I, I, I, I, I, P, L, L, L, P, I, P]),
    "vitmi_conv_col2im": (I, [I, I, I, I, I, I, I, I, I, I, I, I, P, I, P, L, L, L, I, P]),
    "vitmi_dwconv_bn_workspace_size": (S, [I, I, I, I]),
    "vitmi_dwconv_bn_fwd": (I, [I, I, I, I, P, L, L, L, P, P, P, F, F, I, P, P, P, P, P, P, I, L, L, L, P, S, P]),
    "vitmi_dwconv_bn_bwd": (I, [I, I, I, I, P, I, L, L, L, P, L, L, L, P, P, P, P, P, P, P, P, P, P, S, P]),
    "vitmi_sls_resize_table": (I, [I, I, P, P]),
    "vitmi_sls_preprocess": (I, [I, I, I, P, L, L, I, I, I, P, P, P, P, P, P]),
    "vitmi_gather_rows": (I, [L, L, P, L, P, P, P]),
    "vitmi_linear_dgrad_bias_workspace_size": (S, [I, L, L, L]),
    "vitmi_linear_dgrad_bias": (I, [I, L, L, L, P, P, P, I, I, P, P, P, S, P]),
    "vitmi_attention_bwd_bias_workspace_size": (S, [I, I, I]),
    "vitmi_attention_bwd_bias": (I, [I, I, I, I, I, F, P, P, P, P, P, P, P, S, P]),
    "vitmi_adam_step": (I, [L, P, P, P, P, P, F, D, D, F, F, P]),
    "vitmi_dense_f32_fwd": (I, [I, I, I, P, L, P, P, P, L, I, P]),
    "vitmi_dense_f32_bwd": (I, [I, I, I, P, L, P, L, P, L, P, P, L, P, P, I, P]),
    "vitmi_avgpool3_fwd": (I, [I, I, I, I, P, L, L, L, P, I, L, L, L, I, P]),
    "vitmi_avgpool3_bwd": (I, [I, I, I, I, P, I, L, L, L, P, L, L, L, I, P]),
    "vitmi_cast_bf16_f32": (I, [L, P, P, P]),
    "vitmi_stats_enable": (I, [I]),
    "vitmi_stats_count": (I, []),
    "vitmi_stats_get": (I, [I, P, I, P, P, P]),
    "vitmi_trace_enable": (I, [I]),
    "vitmi_trace_push": (I, [ctypes.c_char_p]),
    "vitmi_trace_pop": (I, []),
    "vitmi_attention_set_policy": (I, [I]),
    "vitmi_gemm_set_reserved_cus": (I, [I]),
    "vitmi_comm_get_unique_id": (I, [P]),
    "vitmi_comm_init": (I, [I, I, P]),
    "vitmi_comm_info": (I, [P, P]),
    "vitmi_comm_library": (I, [P, I]),
    "vitmi_comm_allreduce_async": (I, [P, L, I, I, P, P]),
    "vitmi_comm_broadcast": (I, [P, L, I, I, P]),
    "vitmi_comm_check": (I, []),
    "vitmi_comm_destroy": (I, [I]),
    "vitmi_patch_embed_fwd_workspace_size": (S, [I, I, I, I, I, I]),
    "vitmi_patch_embed_fwd": (I, [I, I, I, I, I, I, P, P, P, P, P, P, P, P, S, P]),
    "vitmi_patch_embed_bwd_workspace_size": (S, [I, I, I, I, I, I]),
    "vitmi_patch_embed_bwd": (I, [I, I, I, I, I, I, P, P, P, P, P, P, P, S, P]),
    "vitmi_linear_bwd_workspace_size": (S, [I, L, L, L]),
    "vitmi_linear_bwd": (I, [I, L, L, L, P, P, P, P, I, P, P, P, S, P]),
    "vitmi_xent_fwd": (I, [I, I, P, P, P, P]),
    "vitmi_xent_bwd": (I, [I, I, P, P, P, P]),
    "vitmi_mse_fwd": (I, [I, I, P, P, P, P]),
    "vitmi_mse_bwd": (I, [I, I, P, P, P, P]),
}

_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"vitmi: native library not built ({LIB_PATH}); run "
                "`make -C transformer-stm_amd` or __graft_entry__.build()")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().vitmi_last_error().decode(errors="replace")
        raise RuntimeError(f"vitmi {what} failed (code {rc}): {msg}")


def exported_symbols():
    return list(SIGNATURES)


def build_id_parts(build_id: str):
    """vitmi_build_id() = "<sources>-<flags>" -> (sources, flags) hashes."""
    src, _, flags = build_id.partition("-")
    return src, flags


def flags_id(flags: str) -> str:
    """The flags part of the build id: first 8 hex digits of sha256(vitmi_build_flags())."""
    import hashlib
    return hashlib.sha256(flags.encode()).hexdigest()[:8]


def source_build_id():
    """The sources part of the build id the Makefile stamps into the library (vitmi_build_id):
    sha256 over the bytes of csrc/*.{cpp,h,hip} (sorted by path) followed by include/vitmi.h,
    first 16 hex digits.  None when the sources are not present next to the package."""
    import glob
    import hashlib
    pkg = os.path.dirname(_HERE)
    hdr = os.path.join(os.path.dirname(pkg), "include", "vitmi.h")
    names = sorted(os.path.relpath(f, pkg) for ext in ("hip", "cpp", "h")
                   for f in glob.glob(os.path.join(pkg, "csrc", "*." + ext)))
    if not names or not os.path.exists(hdr):
        return None
    h = hashlib.sha256()
    for n in names:
        with open(os.path.join(pkg, n), "rb") as f:
            h.update(f.read())
    with open(hdr, "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:16]
