"""Tensor-level wrappers over the C ABI (include/vitmi.h).

Every function here launches hand-written gfx950 kernels from libvitmi.so on
torch's current HIP stream; torch only allocates the buffers (caching
allocator).  Inputs must be CUDA(HIP) tensors; there is no CPU or eager
fallback — a missing library or a bad shape raises.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional, Tuple

import torch

from ._lib import check, lib

Tensor = torch.Tensor

F32, BF16 = 0, 1
EPI_STORE, EPI_BIAS_GELU, EPI_RESIDUAL, EPI_DGELU, EPI_ACCUM = 0, 1, 2, 3, 4
EPI_AUX_TILED = 0x100   # gelu' in the library's tile-native layout (include/vitmi.h)
EPI_SPLIT_X3 = 0x200    # BIAS_GELU output as [hi | hi | lo] rows (the precision knob)
EPI_SPLIT_F8 = 0x400    # BIAS_GELU output as VITMI_BF16F8 A-operand rows (the knob's bf16f8 form)
BF16F8_DT = 4           # VITMI_BF16F8: rows of 2K bf16 units, [hi | e4m3 parts] (include/vitmi.h)
BF16F8W_DT = 5          # VITMI_BF16F8W: rows of 1.5K bf16 units, [hi | hi8 (A) or lo8 (weight)]
LOSS_CE, LOSS_MSE = 0, 1

_DT = {torch.float32: F32, torch.bfloat16: BF16}


def dt(t: torch.dtype) -> int:
    try:
        return _DT[t]
    except KeyError:
        raise TypeError(f"vitmi: unsupported dtype {t}") from None


def torch_dtype(name: str) -> torch.dtype:
    """The compute dtype of a ViTConfig.dtype ("bf16x3" / "bf16f8": bf16 MFMA with split forward
    operands; the backward is bf16)."""
    return {"bf16": torch.bfloat16, "bf16x3": torch.bfloat16, "bf16f8": torch.bfloat16, "fp32": torch.float32}[name]


def _s() -> int:
    return torch.cuda.current_stream().cuda_stream


# Optional live probe: HIP events around every linear_fwd launch of one (M, N, K)
# shape, recorded on the stream the kernel runs on (bench.py's roofline leg).
_PROBE = None


def set_probe(key):
    """key = (M, N, K) to time, or None to disable.  Returns the event-pair list."""
    global _PROBE
    _PROBE = None if key is None else {"key": tuple(key), "events": []}
    return None if _PROBE is None else _PROBE["events"]


def _p(t: Optional[Tensor]) -> Optional[int]:
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("vitmi: tensors must live on the GPU (no CPU fallback)")
    return t.data_ptr()


# per host thread (the library's fold queue is thread-local too): the workspaces of calls whose
# partial-sum folds are queued
_TLS = threading.local()


def _ws(nbytes: int, like: Tensor) -> Tensor:
    ws = torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=like.device)
    hold = getattr(_TLS, "hold", None)
    if hold is not None:
        hold.append(ws)
    return ws


class deferred_folds:
    """``with ops.deferred_folds(): ...`` -- the partial-sum folds of the parameter-gradient
    outputs inside (LayerNorm dgamma/dbeta/column sums, fused bias-gradient column sums) are
    queued and launched together at exit (vitmi_fold_begin / vitmi_fold_end); the workspaces
    they read are held until then.  The gradients are final in stream order after the exit."""

    def __enter__(self):
        self._nested = getattr(_TLS, "hold", None) is not None
        if not self._nested:
            _TLS.hold = []
            check(lib().vitmi_fold_begin(), "fold_begin")
        return self

    def __exit__(self, *exc):
        if self._nested:
            return False
        try:
            check(lib().vitmi_fold_end(_s()), "fold_end")
        finally:
            _TLS.hold = None
        return False


def _rows(t: Tensor) -> Tuple[int, int]:
    """(rows, row stride) of a tensor viewed as [rows, last-dim] with unit inner stride."""
    if t.stride(-1) != 1 and t.shape[-1] != 1:
        raise RuntimeError("vitmi: last dim must be contiguous")
    return t.numel() // t.shape[-1], t.stride(-2) if t.dim() > 1 else t.shape[-1]


# ---------------------------------------------------------------- GEMM
def dropout_params(p: float):
    """(thresh, scale) of rate p: keep iff vitmi_dropout_hash >= thresh (include/vitmi.h)."""
    return min(int(round(p * 2.0 ** 32)), 0xFFFFFFFF), 1.0 / (1.0 - p)


def linear_fwd(x: Tensor, w: Tensor, bias: Optional[Tensor], out_dtype: torch.dtype,
               epilogue: int = EPI_STORE, residual: Optional[Tensor] = None, dropout=None,
               aux_tiled: bool = False, split_x3: bool = False, f8=False, split_f8: bool = False):
    """y = x W^T + b (+GELU, +residual).  x [M,K], w [N,K] (same dtype).  Returns y
    (and gelu'(pre-activation), the saved GELU derivative, for EPI_BIAS_GELU).
    ``dropout`` = (seed, site, rate) fuses the dropout of the GELU output / of the branch
    before the residual add into the epilogue (vitmi_linear_fwd_dropout).
    ``aux_tiled`` (bf16): gelu' comes back as an opaque buffer in the tile-native layout, for a
    linear_dgrad(..., EPI_DGELU, aux_tiled=True) of the same [M, N].
    ``split_x3`` (EPI_BIAS_GELU, bf16): y is [M, 3N], each row [hi | hi | lo] of the fp32 GELU
    output (VITMI_EPI_SPLIT_X3, the precision knob's fc2 A operand).
    ``f8``: x [M, 2K] and w [N, 2K] are VITMI_BF16F8 rows (split_bf16f8 patterns 0 / 1; the bf16f8
    knob); ``split_f8`` (with f8, EPI_BIAS_GELU): y is [M, 2N] in the A-operand layout.
    ``f8="w"``: x [M, 1.5K] and w [N, 1.5K] are VITMI_BF16F8W rows (patterns 2 / 3: the weight-side
    correction alone, the knob's qkv GEMM)."""
    assert x.is_contiguous() and w.is_contiguous() and x.dtype == w.dtype
    M, K = x.numel() // x.shape[-1], x.shape[-1]
    N = w.shape[0]
    assert w.shape[1] == K
    assert not split_x3 or (epilogue == EPI_BIAS_GELU and dropout is None)
    assert not split_f8 or (f8 and epilogue == EPI_BIAS_GELU and dropout is None)
    f8w = f8 == "w"
    if f8w:
        assert x.dtype == torch.bfloat16 and K % 3 == 0 and dropout is None and not split_f8
        K = K * 2 // 3
    elif f8:
        assert x.dtype == torch.bfloat16 and K % 2 == 0 and dropout is None
        K //= 2
    y = torch.empty(*x.shape[:-1], 3 * N if split_x3 else 2 * N if split_f8 else N, dtype=out_dtype,
                    device=x.device)
    aux = None
    aux_tiled = aux_tiled and epilogue == EPI_BIAS_GELU
    if aux_tiled:
        aux = torch.empty(lib().vitmi_aux_tiled_bytes(M, N) // 2, dtype=x.dtype, device=x.device)
        epilogue |= EPI_AUX_TILED
    elif epilogue == EPI_BIAS_GELU:
        aux = torch.empty(*x.shape[:-1], N, dtype=x.dtype, device=x.device)
    if split_x3:
        epilogue |= EPI_SPLIT_X3
    if split_f8:
        epilogue |= EPI_SPLIT_F8
    if residual is not None:
        assert residual.is_contiguous() and residual.dtype == torch.float32
    probe = _PROBE is not None and _PROBE["key"] == (M, N, K)
    if probe:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    xdt = BF16F8W_DT if f8w else BF16F8_DT if f8 else dt(x.dtype)
    nws = lib().vitmi_linear_fwd_workspace_size(xdt, M, N, K)
    ws = _ws(nws, x) if nws else None
    if dropout is not None and dropout[2] > 0:
        seed, site, rate = dropout
        thresh, scale = dropout_params(rate)
        check(lib().vitmi_linear_fwd_dropout(dt(x.dtype), M, N, K, _p(x), _p(w), _p(bias), _p(y),
                                             dt(out_dtype), epilogue, _p(aux), _p(residual), _p(ws), nws,
                                             seed & 0xFFFFFFFF, site, thresh, scale, _s()), "linear_fwd_dropout")
    else:
        check(lib().vitmi_linear_fwd(xdt, M, N, K, _p(x), _p(w), _p(bias), _p(y), dt(out_dtype),
                                     epilogue, _p(aux), _p(residual), _p(ws), nws, _s()), "linear_fwd")
    if probe:
        e1.record()
        _PROBE["events"].append((e0, e1))
    return (y, aux) if epilogue & ~(EPI_AUX_TILED | EPI_SPLIT_X3 | EPI_SPLIT_F8) == EPI_BIAS_GELU else y


def dropout_apply(x: Tensor, seed: int, site: int, rate: float, out_dtype: torch.dtype) -> Tensor:
    """x (fp32, rows x C) * keep(seed, site, row, col) / (1 - rate), in out_dtype: the masked
    gradient of a dropped branch (the forward applied the same mask in a GEMM epilogue)."""
    M, ldx = _rows(x)
    N = x.shape[-1]
    y = torch.empty(M, N, dtype=out_dtype, device=x.device)
    thresh, scale = dropout_params(rate)
    check(lib().vitmi_dropout_apply(M, N, _p(x), ldx, _p(y), dt(out_dtype), N, seed & 0xFFFFFFFF, site,
                                    thresh, scale, _s()), "dropout_apply")
    return y


def linear_dgrad(dy: Tensor, w: Tensor, out_dtype: torch.dtype, epilogue: int = EPI_STORE,
                 aux: Optional[Tensor] = None, bias_grad: Optional[Tensor] = None,
                 aux_tiled: bool = False) -> Tensor:
    """dx[M,K] = dy[M,N] W[N,K] (optionally * aux, the gelu' saved by the forward; ``aux_tiled``:
    aux is the tile-native buffer of linear_fwd(..., aux_tiled=True)).
    ``bias_grad`` (fp32 [K]) += column sums of dx, fused into the GEMM epilogue where the
    kernel allows (vitmi_linear_dgrad_bias)."""
    assert dy.is_contiguous() and w.is_contiguous() and dy.dtype == w.dtype
    if aux_tiled and epilogue == EPI_DGELU:
        epilogue |= EPI_AUX_TILED
    M, N = dy.numel() // dy.shape[-1], dy.shape[-1]
    K = w.shape[1]
    dx = torch.empty(*dy.shape[:-1], K, dtype=out_dtype, device=dy.device)
    if bias_grad is not None:
        assert bias_grad.dtype == torch.float32 and bias_grad.is_contiguous() and bias_grad.numel() == K
        nws = lib().vitmi_linear_dgrad_bias_workspace_size(dt(dy.dtype), M, N, K)
        ws = _ws(nws, dy)
        check(lib().vitmi_linear_dgrad_bias(dt(dy.dtype), M, N, K, _p(dy), _p(w), _p(dx), dt(out_dtype), epilogue,
                                            _p(aux), _p(bias_grad), _p(ws), ws.numel(), _s()), "linear_dgrad_bias")
        return dx
    nws = lib().vitmi_linear_dgrad_workspace_size(dt(dy.dtype), M, N, K)
    ws = _ws(nws, dy) if nws else None
    check(lib().vitmi_linear_dgrad(dt(dy.dtype), M, N, K, _p(dy), _p(w), _p(dx), dt(out_dtype),
                                   epilogue, _p(aux), _p(ws), nws, _s()), "linear_dgrad")
    return dx




def bias_grad_(dy: Tensor, db: Tensor) -> None:
    bias_grad(dy, db)


def linear_wgrad(dy: Tensor, x: Tensor, dw: Tensor) -> None:
    """dw[N,K] (fp32) += dy[M,N]^T x[M,K].  x may be row-strided (the hi part of a split
    operand); then the generic GEMM entry point takes its row stride."""
    assert dy.is_contiguous() and dy.dtype == x.dtype
    assert dw.dtype == torch.float32 and dw.is_contiguous()
    if not x.is_contiguous():
        M, N, K = dy.numel() // dy.shape[-1], dy.shape[-1], x.shape[-1]
        gemm(dy.view(M, N), x, False, False, N, K, M, dw, EPI_ACCUM)
        return
    M, N, K = dy.numel() // dy.shape[-1], dy.shape[-1], x.shape[-1]
    ws_n = lib().vitmi_linear_wgrad_workspace_size(dt(dy.dtype), M, N, K)
    ws = _ws(ws_n, dy)
    check(lib().vitmi_linear_wgrad(dt(dy.dtype), M, N, K, _p(dy), _p(x), _p(dw), _p(ws), ws.numel(),
                                   _s()), "linear_wgrad")


# How a block's backward groups its weight gradients (vitmi/modules.py _BlockFn.backward): 0 = one
# launch per problem where each gradient's operands are ready, 1 = all four in one launch at the end,
# 2 = the MLP pair at fc1's point and the attention pair at qkv's, 3 = only the attention pair
# (out-projection + qkv) grouped, at qkv's point.  Measured (profiles/r06_wgg/): alone, one grouped
# launch of all four is 52 us (ViT-B) / 79 us (ViT-L) faster than four; in the step the MLP
# weight gradients run faster where the DGELU GEMM has just written du (their operands still in
# the caches), so 1 loses that and 3 keeps it: C3 kernel time per step 36.16 (0) / 36.35 (1) /
# 36.00 ms (3), the out-projection's 28 slabs of 28 K-steps become 7 of 113.
WGRAD_GROUP = int(os.environ.get("VITMI_WGRAD_GROUP", "3"))
_WGRAD_GROUP = WGRAD_GROUP != 0


def linear_wgrad_group(items) -> None:
    """For each (dy[M, N_p], x[M, K_p], dw[N_p, K_p]) of ``items`` (at most 4, one row count M):
    dw (fp32) += dy^T x, all in ONE split-K launch and one reduction (vitmi_linear_wgrad_group; the
    weight gradients of one transformer block).  x may be row-strided (the hi part of a split
    operand).  Mixed dtypes, other row counts or more than 4 items run one linear_wgrad each."""
    items = [t for t in items if t is not None]
    if not items:
        return
    if not _WGRAD_GROUP:   # (A/B switch: VITMI_WGRAD_GROUP=0 runs one launch per problem)
        for dy, x, dw in items:
            linear_wgrad(dy, x, dw)
        return
    M = items[0][0].numel() // items[0][0].shape[-1]
    dt0 = items[0][0].dtype
    if len(items) == 1 or len(items) > 4 or any(
            dy.dtype != dt0 or x.dtype != dt0 or dy.numel() // dy.shape[-1] != M or not dy.is_contiguous()
            or x.stride(-1) != 1 or dw.dtype != torch.float32 or not dw.is_contiguous() for dy, x, dw in items):
        for dy, x, dw in items:
            linear_wgrad(dy, x, dw)
        return
    n = len(items)
    arr = lambda t, v: (t * n)(*v)  # noqa: E731
    Ns = arr(ctypes.c_int64, [dy.shape[-1] for dy, _, _ in items])
    Ks = arr(ctypes.c_int64, [x.shape[-1] for _, x, _ in items])
    ws_n = lib().vitmi_linear_wgrad_group_workspace_size(dt(dt0), n, M, Ns, Ks)
    ws = _ws(ws_n, items[0][0])
    check(lib().vitmi_linear_wgrad_group(
        dt(dt0), n, M, Ns, Ks, arr(ctypes.c_void_p, [_p(dy) for dy, _, _ in items]),
        arr(ctypes.c_int64, [dy.shape[-1] for dy, _, _ in items]),
        arr(ctypes.c_void_p, [_p(x) for _, x, _ in items]),
        arr(ctypes.c_int64, [x.stride(0) if x.dim() == 2 else x.shape[-1] for _, x, _ in items]),
        arr(ctypes.c_void_p, [_p(dw) for _, _, dw in items]), _p(ws), ws.numel(), _s()), "linear_wgrad_group")


def bias_grad(dy: Tensor, db: Tensor) -> None:
    """db[N] (fp32) += sum over rows of dy[..., N]."""
    M, ld = _rows(dy)
    N = dy.shape[-1]
    ws = _ws(lib().vitmi_bias_grad_workspace_size(M, N), dy)
    check(lib().vitmi_bias_grad(dt(dy.dtype), M, N, _p(dy), ld, _p(db), _p(ws), ws.numel(), _s()),
          "bias_grad")


def gemm(a: Tensor, b: Tensor, a_kmajor: bool, b_kmajor: bool, M: int, N: int, K: int,
         out: Tensor, epilogue: int = EPI_STORE, bias=None, aux=None, residual=None) -> Tensor:
    """Generic C[M,N] = A(m,k) B(k,n) (see vitmi_gemm in include/vitmi.h)."""
    lda = a.stride(0)
    ldb = b.stride(0)
    ws_n = lib().vitmi_gemm_workspace_size(dt(a.dtype), int(a_kmajor), int(b_kmajor), M, N, K, epilogue)
    ws = _ws(ws_n, a)
    check(lib().vitmi_gemm(dt(a.dtype), int(a_kmajor), int(b_kmajor), M, N, K, _p(a), lda, _p(b), ldb,
                           _p(out), out.stride(0), dt(out.dtype), epilogue, _p(bias), _p(aux),
                           aux.stride(0) if aux is not None else 0, _p(residual),
                           residual.stride(0) if residual is not None else 0, _p(ws), ws.numel(), _s()),
          "gemm")
    return out


# ---------------------------------------------------------------- LayerNorm
BF16X3 = "bf16x3"   # layernorm_fwd out_dtype of the precision knob (VITMI_BF16X3)
BF16F8 = "bf16f8"   # ... of its bf16f8 form (VITMI_BF16F8 A-operand rows)
BF16F8W = "bf16f8w"  # ... and of the weight-side form (VITMI_BF16F8W A-operand rows [hi | hi8])
ATTN_SEQ_MAX = 256  # largest N of the whole-sequence attention kernels (csrc/attention.hip SEQ_MAX)


def layernorm_fwd(x: Tensor, w: Tensor, b: Tensor, eps: float, out_dtype):
    """x fp32 [..., D] (rows may be strided) -> (y [rows, D] contiguous, mean, rstd).
    out_dtype BF16X3: y is bf16 [rows, 3D], each row [hi | hi | lo] of the fp32 result;
    BF16F8: y is [rows, 2D] bf16 units, each row the VITMI_BF16F8 A-operand layout; BF16F8W: [rows,
    1.5D], the VITMI_BF16F8W A-operand rows [hi | hi8]."""
    assert x.dtype == torch.float32
    M, ldx = _rows(x)
    D = x.shape[-1]
    x3, f8, f8w = out_dtype == BF16X3, out_dtype == BF16F8, out_dtype == BF16F8W
    width = 3 * D if x3 else 2 * D if f8 else D + D // 2 if f8w else D
    y = torch.empty(M, width, dtype=torch.bfloat16 if x3 or f8 or f8w else out_dtype, device=x.device)
    mean = torch.empty(M, dtype=torch.float32, device=x.device)
    rstd = torch.empty(M, dtype=torch.float32, device=x.device)
    code = 3 if x3 else BF16F8_DT if f8 else BF16F8W_DT if f8w else dt(out_dtype)
    check(lib().vitmi_layernorm_fwd(M, D, _p(x), ldx, _p(w), _p(b), float(eps), _p(y), code,
                                    y.shape[1], _p(mean), _p(rstd), _s()), "layernorm_fwd")
    return y, mean, rstd


def layernorm_bwd(dy: Tensor, x: Tensor, mean: Tensor, rstd: Tensor, w: Tensor,
                  dgamma: Optional[Tensor], dbeta: Optional[Tensor], dres: Optional[Tensor] = None,
                  dx: Optional[Tensor] = None, lp_dtype: Optional[torch.dtype] = None,
                  dxsum: Optional[Tensor] = None, dx_lp: Optional[Tensor] = None):
    """dx = dres + LN'(dy); dgamma/dbeta (fp32) +=; dxsum += column sums of dx.
    Returns (dx fp32, dx_lp or None).

    ``dx`` and ``dx_lp`` (the low-precision copy, dtype lp_dtype) may be pre-allocated, possibly
    row-strided destinations."""
    M, ldy = _rows(dy)
    _, ldx = _rows(x)
    D = x.shape[-1]
    if dx is None:
        dx = torch.empty(M, D, dtype=torch.float32, device=x.device)
    _, lddx = _rows(dx)
    lp_ld = D
    if dx_lp is not None:
        assert lp_dtype is not None and dx_lp.dtype == lp_dtype
        lp_ld = _rows(dx_lp)[1]
    elif lp_dtype is not None and lp_dtype != torch.float32:
        dx_lp = torch.empty(M, D, dtype=lp_dtype, device=x.device)
    ldres = _rows(dres)[1] if dres is not None else 0
    ws = _ws(lib().vitmi_layernorm_bwd_workspace_size(M, D), x)
    check(lib().vitmi_layernorm_bwd(M, D, _p(dy), dt(dy.dtype), ldy, _p(x), ldx, _p(mean), _p(rstd), _p(w),
                                    _p(dres), ldres, _p(dx), lddx, _p(dx_lp), lp_ld, _p(dgamma), _p(dbeta),
                                    _p(dxsum), _p(ws), ws.numel(), _s()), "layernorm_bwd")
    return dx, dx_lp


# ---------------------------------------------------------------- attention
def attention_set_policy(policy: int) -> int:
    """0 = auto, 1 = always the streamed kernels, 2 = the whole-sequence 32-query forward / dQ
    forms (tests).  Returns the previous policy."""
    return lib().vitmi_attention_set_policy(int(policy))


def attention_fwd(qkv: Tensor, B: int, N: int, H: int, scale: float):
    """qkv [B*N, 3*H*64] -> (o [B*N, H*64], lse fp32 [B*H, N])."""
    D3 = qkv.shape[-1]
    D = D3 // 3
    assert qkv.is_contiguous() and qkv.numel() == B * N * D3
    o = torch.empty(B * N, D, dtype=qkv.dtype, device=qkv.device)
    lse = torch.empty(B * H, N, dtype=torch.float32, device=qkv.device)
    check(lib().vitmi_attention_fwd(dt(qkv.dtype), B, N, H, D // H, float(scale), _p(qkv), _p(o), _p(lse),
                                    _s()), "attention_fwd")
    return o, lse


def attention_fwd_x3(qkv: Tensor, B: int, N: int, H: int, scale: float):
    """bf16 qkv [B*N, 3*H*64] -> (o bf16 [B*N, H*64], o3 bf16 [B*N, 3*H*64] = [hi | hi | lo] rows of
    the fp32 output, lse fp32 [B*H, N]); N <= 256.  o and lse are attention_fwd's, bit for bit."""
    D = qkv.shape[-1] // 3
    assert qkv.is_contiguous() and qkv.dtype == torch.bfloat16 and qkv.numel() == B * N * 3 * D
    o = torch.empty(B * N, D, dtype=torch.bfloat16, device=qkv.device)
    o3 = torch.empty(B * N, 3 * D, dtype=torch.bfloat16, device=qkv.device)
    lse = torch.empty(B * H, N, dtype=torch.float32, device=qkv.device)
    check(lib().vitmi_attention_fwd_x3(B, N, H, D // H, float(scale), _p(qkv), _p(o), _p(o3), _p(lse), _s()),
          "attention_fwd_x3")
    return o, o3, lse


def attention_fwd_f8(qkv: Tensor, B: int, N: int, H: int, scale: float):
    """As attention_fwd_x3 for the bf16f8 knob: o8 is [B*N, 2*H*64] bf16 units, each row the
    VITMI_BF16F8 A-operand layout of the fp32 output."""
    D = qkv.shape[-1] // 3
    assert qkv.is_contiguous() and qkv.dtype == torch.bfloat16 and qkv.numel() == B * N * 3 * D
    o = torch.empty(B * N, D, dtype=torch.bfloat16, device=qkv.device)
    o8 = torch.empty(B * N, 2 * D, dtype=torch.bfloat16, device=qkv.device)
    lse = torch.empty(B * H, N, dtype=torch.float32, device=qkv.device)
    check(lib().vitmi_attention_fwd_f8(B, N, H, D // H, float(scale), _p(qkv), _p(o), _p(o8), _p(lse), _s()),
          "attention_fwd_f8")
    return o, o8, lse


def attention_bwd(qkv: Tensor, o: Tensor, do: Tensor, lse: Tensor, B: int, N: int, H: int,
                  scale: float, bias_grad: Optional[Tensor] = None, fused_bias: bool = True) -> Tensor:
    """dqkv; ``bias_grad`` (fp32 [3D]) += its column sums (the q/k/v bias gradient).

    ``fused_bias`` (default) forms the sums in the backward kernels from the LDS image each
    output tile is stored through (vitmi_attention_bwd_bias: one [3D] partial row per batch, or
    per (batch, 128-row block) for N > 256, folded in a fixed order), instead of a second pass
    over dqkv; ``fused_bias=False`` runs the
    separate column-sum pass (kernels without the fused sums fall back to it anyway)."""
    D = o.shape[-1]
    assert do.is_contiguous() and do.dtype == qkv.dtype
    dqkv = torch.empty_like(qkv)
    if bias_grad is not None and not fused_bias:
        dqkv = attention_bwd(qkv, o, do, lse, B, N, H, scale)
        bias_grad_(dqkv, bias_grad)
        return dqkv
    if bias_grad is not None:
        assert bias_grad.dtype == torch.float32 and bias_grad.numel() == 3 * D and bias_grad.is_contiguous()
        ws = _ws(lib().vitmi_attention_bwd_bias_workspace_size(B, N, H), qkv)
        check(lib().vitmi_attention_bwd_bias(dt(qkv.dtype), B, N, H, D // H, float(scale), _p(qkv), _p(o), _p(do),
                                             _p(lse), _p(dqkv), _p(bias_grad), _p(ws), ws.numel(), _s()),
              "attention_bwd_bias")
        return dqkv
    ws = _ws(lib().vitmi_attention_bwd_workspace_size(B, N, H), qkv)
    check(lib().vitmi_attention_bwd(dt(qkv.dtype), B, N, H, D // H, float(scale), _p(qkv), _p(o), _p(do),
                                    _p(lse), _p(dqkv), _p(ws), ws.numel(), _s()), "attention_bwd")
    return dqkv


# ---------------------------------------------------------------- patch embed / tokens
def patch_im2col(img: Tensor, P: int, out_dtype: torch.dtype) -> Tensor:
    B, C, S, S2 = img.shape
    assert S == S2 and img.dtype == torch.float32 and img.is_contiguous()
    G = S // P
    out = torch.empty(B * G * G, C * P * P, dtype=out_dtype, device=img.device)
    check(lib().vitmi_patch_im2col(dt(out_dtype), B, C, S, P, _p(img), _p(out), _s()), "patch_im2col")
    return out


def tokens_assemble(tok: Tensor, B: int, np_: int, cls: Optional[Tensor], pos: Optional[Tensor]) -> Tensor:
    D = tok.shape[-1]
    x = torch.empty(B, np_ + 1, D, dtype=torch.float32, device=tok.device)
    check(lib().vitmi_tokens_assemble(B, np_, D, _p(tok), _p(cls), _p(pos), _p(x), _s()), "tokens_assemble")
    return x


def tokens_assemble_bwd(dx: Tensor, B: int, np_: int, want_f32: bool, lp_dtype: Optional[torch.dtype],
                        dcls: Optional[Tensor], dpos: Optional[Tensor]):
    D = dx.shape[-1]
    dtok = torch.empty(B * np_, D, dtype=torch.float32, device=dx.device) if want_f32 else None
    dtok_lp = None
    if lp_dtype is not None and lp_dtype != torch.float32:
        dtok_lp = torch.empty(B * np_, D, dtype=lp_dtype, device=dx.device)
    check(lib().vitmi_tokens_assemble_bwd(B, np_, D, _p(dx.contiguous()), _p(dtok), _p(dtok_lp), _p(dcls),
                                          _p(dpos), _s()), "tokens_assemble_bwd")
    return dtok, dtok_lp


# ---------------------------------------------------------------- §8(b) per-op entry points
def patch_embed_fwd(img: Tensor, w: Tensor, bias: Optional[Tensor], cls: Optional[Tensor], pos: Optional[Tensor],
                    P: int, dtype: torch.dtype):
    """vitmi_patch_embed_fwd: Conv2D(k=P, s=P) + cls + pos -> (x fp32 [B, np+1, D], patches
    [B*np, C*P*P] of dtype, saved for the backward).  w: [D, C*P*P] of dtype."""
    B, C, S, S2 = img.shape
    assert S == S2 and img.dtype == torch.float32 and img.is_contiguous()
    D = w.shape[0]
    assert w.is_contiguous() and w.dtype == dtype and w.shape[1] == C * P * P
    G = S // P
    patches = torch.empty(B * G * G, C * P * P, dtype=dtype, device=img.device)
    x = torch.empty(B, G * G + 1, D, dtype=torch.float32, device=img.device)
    ws = _ws(lib().vitmi_patch_embed_fwd_workspace_size(dt(dtype), B, C, S, P, D), img)
    check(lib().vitmi_patch_embed_fwd(dt(dtype), B, C, S, P, D, _p(img), _p(w), _p(bias), _p(cls), _p(pos),
                                      _p(patches), _p(x), _p(ws), ws.numel(), _s()), "patch_embed_fwd")
    return x, patches


def patch_embed_bwd(dx: Tensor, patches: Tensor, B: int, C: int, S: int, P: int, dw: Optional[Tensor],
                    dbias: Optional[Tensor], dcls: Optional[Tensor], dpos: Optional[Tensor]) -> None:
    """vitmi_patch_embed_bwd: dw [D, C*P*P] / dbias / dcls / dpos (fp32) += their gradients."""
    dx = dx.contiguous()
    D = dx.shape[-1]
    dtype = patches.dtype
    ws = _ws(lib().vitmi_patch_embed_bwd_workspace_size(dt(dtype), B, C, S, P, D), dx)
    check(lib().vitmi_patch_embed_bwd(dt(dtype), B, C, S, P, D, _p(dx), _p(patches), _p(dw), _p(dbias), _p(dcls),
                                      _p(dpos), _p(ws), ws.numel(), _s()), "patch_embed_bwd")


def linear_bwd(dy: Tensor, x: Optional[Tensor], w: Optional[Tensor], dx_dtype: Optional[torch.dtype],
               dw: Optional[Tensor], db: Optional[Tensor]) -> Optional[Tensor]:
    """vitmi_linear_bwd: dx = dy W (when dx_dtype), dw += dy^T x, db += colsum(dy)."""
    assert dy.is_contiguous()
    M, N = dy.numel() // dy.shape[-1], dy.shape[-1]
    K = w.shape[1] if w is not None else x.shape[-1]
    dx = torch.empty(*dy.shape[:-1], K, dtype=dx_dtype, device=dy.device) if dx_dtype is not None else None
    ws = _ws(lib().vitmi_linear_bwd_workspace_size(dt(dy.dtype), M, N, K), dy)
    check(lib().vitmi_linear_bwd(dt(dy.dtype), M, N, K, _p(dy), _p(x), _p(w), _p(dx),
                                 dt(dx_dtype) if dx_dtype is not None else 0, _p(dw), _p(db), _p(ws), ws.numel(),
                                 _s()), "linear_bwd")
    return dx


def _loss_entry(name: str, logits: Tensor, target: Tensor, grad: bool) -> Tensor:
    B, C = logits.shape
    logits = logits.contiguous()
    out = torch.empty_like(logits) if grad else torch.empty((), dtype=torch.float32, device=logits.device)
    check(getattr(lib(), name)(B, C, _p(logits), _p(target.contiguous()), _p(out), _s()), name)
    return out


def xent_fwd(logits: Tensor, target: Tensor) -> Tensor:
    return _loss_entry("vitmi_xent_fwd", logits, target.to(torch.int64), False)


def xent_bwd(logits: Tensor, target: Tensor) -> Tensor:
    return _loss_entry("vitmi_xent_bwd", logits, target.to(torch.int64), True)


def mse_fwd(pred: Tensor, target: Tensor) -> Tensor:
    return _loss_entry("vitmi_mse_fwd", pred, target.to(torch.float32).reshape(pred.shape), False)


def mse_bwd(pred: Tensor, target: Tensor) -> Tensor:
    return _loss_entry("vitmi_mse_bwd", pred, target.to(torch.float32).reshape(pred.shape), True)


# ---------------------------------------------------------------- head / loss / cast
def head_fwd(y: Tensor, w: Tensor, b: Optional[Tensor]) -> Tensor:
    B, D = y.shape
    C = w.shape[0]
    logits = torch.empty(B, C, dtype=torch.float32, device=y.device)
    check(lib().vitmi_head_fwd(B, D, C, _p(y), y.stride(0), _p(w), _p(b), _p(logits), _s()), "head_fwd")
    return logits


def head_bwd(dlogits: Tensor, y: Tensor, w: Tensor, dw: Tensor, db: Optional[Tensor]) -> Tensor:
    B, D = y.shape
    C = w.shape[0]
    dy = torch.empty(B, D, dtype=torch.float32, device=y.device)
    check(lib().vitmi_head_bwd(B, D, C, _p(dlogits.contiguous()), _p(y), y.stride(0), _p(w), _p(dy), _p(dw),
                               _p(db), _s()), "head_bwd")
    return dy


def loss_fwd_bwd(logits: Tensor, target: Tensor, kind: int):
    B, C = logits.shape
    loss = torch.empty((), dtype=torch.float32, device=logits.device)
    dl = torch.empty_like(logits)
    if kind == LOSS_CE:
        target = target.to(torch.int64).contiguous()
    else:
        target = target.to(torch.float32).contiguous()
    check(lib().vitmi_loss_fwd_bwd(kind, B, C, _p(logits.contiguous()), _p(target), _p(loss), _p(dl), _s()),
          "loss")
    return loss, dl


def cast_bf16(src: Tensor, dst: Optional[Tensor] = None) -> Tensor:
    assert src.dtype == torch.float32 and src.is_contiguous()
    if dst is None:
        dst = torch.empty(src.shape, dtype=torch.bfloat16, device=src.device)
    check(lib().vitmi_cast_f32_bf16(src.numel(), _p(src), _p(dst), _s()), "cast")
    return dst


def split_bf16x3(x: Tensor, pattern: int, hi_copy: bool = False):
    """x fp32 [rows, K] (rows may be strided) -> (x3 bf16 [rows, 3K] laid out [hi | hi | lo]
    (pattern 0, a GEMM's A operand) or [hi | lo | hi] (pattern 1, its weight), hi bf16 [rows, K]
    or None): the split-bf16 operand of the precision knob (vitmi_split_bf16x3)."""
    assert x.dtype == torch.float32
    rows, ld = _rows(x)
    K = x.shape[-1]
    x3 = torch.empty(rows, 3 * K, dtype=torch.bfloat16, device=x.device)
    hi = torch.empty(rows, K, dtype=torch.bfloat16, device=x.device) if hi_copy else None
    check(lib().vitmi_split_bf16x3(rows, K, _p(x), ld, _p(x3), 3 * K, int(pattern), _p(hi), K, _s()),
          "split_bf16x3")
    return x3, hi


def split_bf16f8_weights(ws, patterns=None):
    """Dense fp32 weights [N_j, K_j] (up to 8) -> their pattern-1 VITMI_BF16F8 rows [N_j, 2 K_j] (or,
    where patterns[j] == 3, VITMI_BF16F8W rows [hi | lo8] [N_j, 1.5 K_j]), one launch
    (vitmi_split_bf16f8_weights_mixed)."""
    ws = [w.detach() for w in ws]
    n = len(ws)
    pats = list(patterns) if patterns is not None else [1] * n
    assert 1 <= n <= 8 and len(pats) == n and all(
        w.dtype == torch.float32 and w.is_contiguous() and w.dim() == 2 for w in ws)
    outs = [torch.empty(w.shape[0], (w.shape[1] * 3 // 2) if p == 3 else 2 * w.shape[1], dtype=torch.bfloat16,
                        device=w.device) for w, p in zip(ws, pats)]
    srcs = (ctypes.c_void_p * n)(*[_p(w) for w in ws])
    dsts = (ctypes.c_void_p * n)(*[_p(o) for o in outs])
    rows = (ctypes.c_int64 * n)(*[w.shape[0] for w in ws])
    ks = (ctypes.c_int64 * n)(*[w.shape[1] for w in ws])
    check(lib().vitmi_split_bf16f8_weights_mixed(n, srcs, dsts, rows, ks, (ctypes.c_int * n)(*pats), _s()),
          "split_bf16f8_weights")
    return outs


def split_bf16f8(x: Tensor, pattern: int, hi_copy: bool = False):
    """x fp32 [rows, K] (rows may be strided) -> (x8 [rows, 2K] bf16 units, the VITMI_BF16F8 rows
    [hi | hi8 | lo8] (pattern 0, a GEMM's A operand) or [hi | lo8 | hi8] (pattern 1, its weight),
    hi bf16 [rows, K] or None) (vitmi_split_bf16f8; hi8 = e4m3(hi), lo8 = e4m3((x - hi) 2^9))."""
    assert x.dtype == torch.float32
    rows, ld = _rows(x)
    K = x.shape[-1]
    width = K + K // 2 if pattern >= 2 else 2 * K   # patterns 2 / 3: VITMI_BF16F8W [hi | hi8] / [hi | lo8]
    x8 = torch.empty(rows, width, dtype=torch.bfloat16, device=x.device)
    hi = torch.empty(rows, K, dtype=torch.bfloat16, device=x.device) if hi_copy else None
    check(lib().vitmi_split_bf16f8(rows, K, _p(x), ld, _p(x8), width, int(pattern), _p(hi), K, _s()),
          "split_bf16f8")
    return x8, hi


def cast_f32(src: Tensor, dst: Optional[Tensor] = None) -> Tensor:
    """bf16 -> fp32 (vitmi_cast_bf16_f32)."""
    assert src.dtype == torch.bfloat16 and src.is_contiguous()
    if dst is None:
        dst = torch.empty(src.shape, dtype=torch.float32, device=src.device)
    check(lib().vitmi_cast_bf16_f32(src.numel(), _p(src), _p(dst), _s()), "cast_bf16_f32")
    return dst


# ---------------------------------------------------------------- CvT stages
def conv_same_geometry(H: int, W: int, k: int, s: int) -> Tuple[int, int, int, int]:
    """TF 'same' geometry of layers.Conv2D (models/CvT(Par).py:203-212): (Ho, Wo, pad_top, pad_left)."""
    import ctypes
    v = [ctypes.c_int(0) for _ in range(4)]
    check(lib().vitmi_conv_same_geometry(H, W, k, k, s, *[ctypes.addressof(t) for t in v]), "conv_same_geometry")
    return tuple(t.value for t in v)


def conv_im2col(x: Tensor, B: int, H: int, W: int, C: int, k: int, s: int, geo, Kp: int,
                out_dtype: torch.dtype, img_stride: Optional[int] = None, row_off: int = 0) -> Tensor:
    """Patch rows [B*Ho*Wo, Kp] (column order kh, kw, c; zero past kh*kw*C) of the NHWC fp32
    token rows of x (image b pixel (h, w) = row b*img_stride + row_off + h*W + w)."""
    Ho, Wo, pt, pl = geo
    _, ldx = _rows(x)
    img_stride = H * W if img_stride is None else img_stride
    out = torch.empty(B * Ho * Wo, Kp, dtype=out_dtype, device=x.device)
    check(lib().vitmi_conv_im2col(dt(out_dtype), B, H, W, C, k, k, s, pt, pl, Ho, Wo, _p(x), ldx, img_stride, row_off,
                                  _p(out), Kp, _s()), "conv_im2col")
    return out


def conv_col2im(dp: Tensor, B: int, H: int, W: int, C: int, k: int, s: int, geo, dx: Tensor,
                img_stride: Optional[int] = None, row_off: int = 0, accumulate: bool = False) -> Tensor:
    """dx (fp32 NHWC rows as in conv_im2col) (+)= the adjoint of im2col applied to dp [rows, Kp]."""
    Ho, Wo, pt, pl = geo
    _, ldx = _rows(dx)
    img_stride = H * W if img_stride is None else img_stride
    check(lib().vitmi_conv_col2im(dt(dp.dtype), B, H, W, C, k, k, s, pt, pl, Ho, Wo, _p(dp), dp.shape[-1], _p(dx), ldx,
                                  img_stride, row_off, int(accumulate), _s()), "conv_col2im")
    return dx


def dwconv_bn_fwd(x: Tensor, B: int, H: int, W: int, w9: Tensor, gamma: Tensor, beta: Tensor, eps: float,
                  momentum: float, training: bool, run_mean: Optional[Tensor], run_var: Optional[Tensor],
                  y: Tensor, x_img: Optional[int] = None, x_off: int = 0, y_img: Optional[int] = None,
                  y_off: int = 0):
    """Projection('dw_bn') (models/CvT(Par).py:92-94): y rows <- BN(depthwise3x3(x)); w9 [3,3,C].
    Returns the saved (z, mean, rstd)."""
    C = x.shape[-1]
    _, ldx = _rows(x)
    _, ldy = _rows(y)
    x_img = H * W if x_img is None else x_img
    y_img = H * W if y_img is None else y_img
    z = torch.empty(B * H * W, C, dtype=torch.float32, device=x.device)
    mean = torch.empty(C, dtype=torch.float32, device=x.device)
    rstd = torch.empty_like(mean)
    ws = _ws(lib().vitmi_dwconv_bn_workspace_size(B, H, W, C), x)
    check(lib().vitmi_dwconv_bn_fwd(B, H, W, C, _p(x), ldx, x_img, x_off, _p(w9), _p(gamma), _p(beta), float(eps),
                                    float(momentum), int(training), _p(run_mean), _p(run_var), _p(z), _p(mean),
                                    _p(rstd), _p(y), dt(y.dtype), ldy, y_img, y_off, _p(ws), ws.numel(), _s()),
          "dwconv_bn_fwd")
    return z, mean, rstd


def dwconv_bn_bwd(dy: Tensor, x: Tensor, B: int, H: int, W: int, w9: Tensor, gamma: Tensor, z: Tensor,
                  mean: Tensor, rstd: Tensor, dx: Tensor, dw9: Tensor, dgamma: Tensor, dbeta: Tensor,
                  x_img: Optional[int] = None, x_off: int = 0, dy_img: Optional[int] = None, dy_off: int = 0) -> None:
    """dx (rows as x) += d/dx; dw9/dgamma/dbeta += their gradients (fp32)."""
    C = x.shape[-1]
    _, ldx = _rows(x)
    _, lddy = _rows(dy)
    assert dx.stride() == x.stride()
    x_img = H * W if x_img is None else x_img
    dy_img = H * W if dy_img is None else dy_img
    ws = _ws(lib().vitmi_dwconv_bn_workspace_size(B, H, W, C), x)
    check(lib().vitmi_dwconv_bn_bwd(B, H, W, C, _p(dy), dt(dy.dtype), lddy, dy_img, dy_off, _p(x), ldx, x_img, x_off,
                                    _p(w9), _p(gamma), _p(z), _p(mean), _p(rstd), _p(dx), _p(dw9), _p(dgamma),
                                    _p(dbeta), _p(ws), ws.numel(), _s()), "dwconv_bn_bwd")


def avgpool3_fwd(x: Tensor, B: int, H: int, W: int, y: Tensor, x_img: Optional[int] = None, x_off: int = 0,
                 y_img: Optional[int] = None, y_off: int = 0, count_pad: bool = False) -> Tensor:
    """Projection('avg'): 3x3 stride-1 'same' average pooling (padding excluded from the count)
    of the fp32 rows x into the rows of y (bf16 | fp32)."""
    C = x.shape[-1]
    _, ldx = _rows(x)
    _, ldy = _rows(y)
    x_img = H * W if x_img is None else x_img
    y_img = H * W if y_img is None else y_img
    check(lib().vitmi_avgpool3_fwd(B, H, W, C, _p(x), ldx, x_img, x_off, _p(y), dt(y.dtype), ldy, y_img, y_off,
                                   int(count_pad), _s()), "avgpool3_fwd")
    return y


def avgpool3_bwd(dy: Tensor, B: int, H: int, W: int, dx: Tensor, dy_img: Optional[int] = None, dy_off: int = 0,
                 x_img: Optional[int] = None, x_off: int = 0, count_pad: bool = False) -> None:
    """dx (fp32 rows) += avgpool3^T(dy)."""
    C = dx.shape[-1]
    _, lddy = _rows(dy)
    _, ldx = _rows(dx)
    x_img = H * W if x_img is None else x_img
    dy_img = H * W if dy_img is None else dy_img
    check(lib().vitmi_avgpool3_bwd(B, H, W, C, _p(dy), dt(dy.dtype), lddy, dy_img, dy_off, _p(dx), ldx, x_img, x_off,
                                   int(count_pad), _s()), "avgpool3_bwd")


# ---------------------------------------------------------------- small fp32 Dense
ACT_LINEAR, ACT_RELU = 0, 1


def dense_f32_fwd(x: Tensor, w: Tensor, b: Optional[Tensor], act: int = ACT_LINEAR) -> Tensor:
    """y = act(x W^T + b) on the small fp32 Dense kernel (Proc_Dense_1/2)."""
    M, ldx = _rows(x)
    N, K = w.shape
    assert x.dtype == torch.float32 and w.is_contiguous() and x.shape[-1] == K
    y = torch.empty(M, N, dtype=torch.float32, device=x.device)
    check(lib().vitmi_dense_f32_fwd(M, N, K, _p(x), ldx, _p(w), _p(b), _p(y), N, act, _s()), "dense_f32_fwd")
    return y


def dense_f32_bwd(dy: Tensor, y: Tensor, x: Tensor, w: Tensor, dw: Tensor, db: Optional[Tensor],
                  act: int = ACT_LINEAR, want_dx: bool = True) -> Optional[Tensor]:
    M, lddy = _rows(dy)
    _, ldy = _rows(y)
    _, ldx = _rows(x)
    N, K = w.shape
    dx = torch.empty(M, K, dtype=torch.float32, device=x.device) if want_dx else None
    check(lib().vitmi_dense_f32_bwd(M, N, K, _p(dy), lddy, _p(y), ldy, _p(x), ldx, _p(w), _p(dx), K, _p(dw), _p(db),
                                    act, _s()), "dense_f32_bwd")
    return dx
