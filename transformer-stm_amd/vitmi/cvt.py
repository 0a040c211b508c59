"""CvT: the reference's convolutional transformer on the MI355X path.

``create_cvt_model`` (``models/CvT(Par).py:292-354``) with the stage spec ``:66-72``: per stage a
strided ``ConvEmbed`` (Conv2D 'same', ``:194-217``) and one ``ConvTransformerBlock``
(``:231-289``) whose q/k/v come from ``Projection('dw_bn')`` (depthwise 3x3 + BatchNorm,
``:83-112``; or 'avg' pooling / 'linear' identity, ``qkv_method``) followed by the q/k/v Dense layers composed with MultiHeadAttention's own
projections (``:132-137,178-185``).  Module tree and parameter names follow MS_CvT's
``ConvolutionalVisionTransformer`` (``old_codes/MS_CvT.py:491-623``)::

    CvT(cfg)
      stage{i}: CvTStageModule  (.embed: ConvEmbedSame (.norm if cfg.embed_norm), .cls_token,
                                 .blocks[j]: CvTBlock (.norm1, .attn: CvTAttention
                                 (.conv_proj_{q,k,v}: DwBnProjection (.bn), .proj_{q,k,v}, .proj),
                                 .norm2 unless tied, .mlp (.fc1, .fc2)))
      norm: LayerNorm, proc: ProcMlp (.fc1, .fc2; cfg.proc_dim > 0), head: Linear

Every op runs as a libvitmi kernel: conv-embed im2col + MFMA GEMM (+ col2im in the backward),
dw_bn fwd/bwd, LayerNorm, the q/k/v/out/MLP GEMMs with fused epilogues and the attention
kernels (N = 1024, 256 and 65 at 128x128 input).  Small glue (the cls-row copies) is torch
tensor indexing on the GPU.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from . import ops
from .modules import F32, LayerNorm, Linear, _check_cuda, _drop_args, _lp, _sink, cross_entropy, mse_loss  # noqa: F401

Tensor = torch.Tensor


@dataclass
class CvTStage:
    embed_dim: int
    patch_size: int
    stride: int
    num_heads: int
    with_cls_token: bool = False
    depth: int = 1
    padding: Optional[int] = None    # None: TF 'same' (Keras); an int: symmetric (torch / MS_CvT)
    qkv_method: str = "dw_bn"        # 'dw_bn' | 'avg' (q stays 'linear') | 'linear'  (:25,83-112,130-132)


def qkv_methods(st: CvTStage):
    """Per-projection methods: 'avg' keeps q linear (models/CvT(Par).py:130-132)."""
    m = st.qkv_method
    if m not in ("dw_bn", "avg", "linear"):
        raise ValueError(f"unknown qkv_method {m}")
    return ("linear" if m == "avg" else m, m, m)


def keras_spec() -> List[CvTStage]:
    """models/CvT(Par).py:66-72 (projection_method 'dw_bn' :25, cls_token_switch True :28)."""
    return [CvTStage(64, 7, 4, 1), CvTStage(128, 3, 2, 2), CvTStage(256, 3, 2, 4, with_cls_token=True)]


@dataclass
class CvTConfig:
    img_size: int = 128
    in_chans: int = 1
    num_classes: int = 1
    stages: List[CvTStage] = field(default_factory=keras_spec)
    mlp_ratio: float = 4.0
    attn_scale: str = "head"       # Keras MHA key_dim**-0.5; 'dim' = MS_CvT D**-0.5
    ln_eps: float = 1e-6
    bn_eps: float = 1e-3           # Keras BatchNormalization
    bn_momentum: float = 0.99      # Keras convention: running <- m running + (1 - m) batch
    qkv_bias: bool = True
    tie_norms: bool = True         # the Keras block applies its one norm1 twice (:272,278)
    embed_norm: bool = False       # the intended ConvEmbed LayerNorm is never built (:209)
    avg_count_pad: bool = False    # 'avg' divisor: TF 'same' in-bounds count (False) or torch's 9
    proc_dim: int = 0              # process parameters (5 in the reference, :392); 0 = image only
    proc_hidden: int = 256         # Proc_Dense_1/2 width (:343-344)
    # Dropout after the out-projection (:141,189) and after both MLP Dense layers (:255,257);
    # Keras default 0.1 in training.  0 = the parity / benchmark configuration.
    drop_rate: float = 0.0
    dtype: str = "bf16"
    # Keras' stacked Dense pairs as separate parameters (models/CvT(Par).py:132-137,180-188): the
    # q/k/v Dense then MultiHeadAttention's query/key/value projection, and MHA's output
    # projection then self.proj.  False: each pair is ONE linear map (their composition; the same
    # forward, fewer parameters, a different Adam trajectory).  True: both factors are parameters
    # (attn.proj_{q,k,v} / attn.mha_{q,k,v}, attn.mha_o / attn.proj); every forward composes them
    # (fp32 GEMMs, D^3 each) and the backward hands each factor its chain-rule gradient, so Adam
    # steps the same parameters Keras does.
    keras_dense: bool = False

    def replace(self, **kw) -> "CvTConfig":
        return dataclasses.replace(self, **kw)


def _kpad(K: int) -> int:
    return (K + 63) // 64 * 64   # the GEMM's K step (bf16 64, fp32 32)


def _geometry(H: int, k: int, s: int, padding: Optional[int]):
    """(Ho, Wo, pad_top, pad_left) for a square input."""
    if padding is None:
        return ops.conv_same_geometry(H, H, k, s)
    Ho = (H + 2 * padding - k) // s + 1
    return (Ho, Ho, padding, padding)


# ======================================================================= ConvEmbed
class ConvEmbedSame(nn.Module):
    """layers.Conv2D(D, kernel=k, strides=s, padding='same') (models/CvT(Par).py:203-212) on
    NHWC token rows, as im2col + MFMA GEMM.  ``weight`` keeps torch's [D, Cin, k, k] layout."""

    def __init__(self, cin: int, dim: int, k: int, s: int, padding: Optional[int], norm: bool, eps: float,
                 dtype: str):
        super().__init__()
        self.cin, self.dim, self.k, self.s, self.padding, self.dtype = cin, dim, k, s, padding, dtype
        self.weight = nn.Parameter(torch.zeros(dim, cin, k, k))
        self.bias = nn.Parameter(torch.zeros(dim))
        self.norm = LayerNorm(dim, eps) if norm else None

    def forward(self, x: Tensor, B: int, H: int, img_stride: Optional[int] = None, row_off: int = 0):
        """x: fp32 rows [.., Cin] (image b pixel (h, w) = row b*img_stride + row_off + h*H + w).
        Returns (tokens fp32 [B, Ho*Wo, D], Ho)."""
        geo = _geometry(H, self.k, self.s, self.padding)
        y = _ConvEmbedFn.apply(x, self, geo, B, H, img_stride, row_off, self.weight, self.bias)
        y = y.view(B, geo[0] * geo[1], self.dim)
        if self.norm is not None:
            y = self.norm(y)
        return y, geo[0]


class _ConvEmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mod, geo, B, H, img_stride, row_off, w, b):
        T = ops.torch_dtype(mod.dtype)
        C, D, k = mod.cin, mod.dim, mod.k
        K = k * k * C
        Kp = _kpad(K)
        patches = ops.conv_im2col(x, B, H, H, C, k, mod.s, geo, Kp, T, img_stride, row_off)
        wm = torch.zeros(D, Kp, dtype=T, device=x.device)          # [D][kh][kw][Cin], zero-padded
        wm[:, :K] = w.detach().permute(0, 2, 3, 1).reshape(D, K).to(T)
        y = ops.linear_fwd(patches, wm, b, F32)
        ctx.save_for_backward(x, patches, wm)
        ctx.mod, ctx.geo, ctx.dims = mod, geo, (B, H, img_stride, row_off)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, patches, wm = ctx.saved_tensors
        mod, geo, (B, H, img_stride, row_off) = ctx.mod, ctx.geo, ctx.dims
        T = patches.dtype
        C, D, k = mod.cin, mod.dim, mod.k
        K = k * k * C
        gs = _sink(ctx, 7, (mod.weight, mod.bias))
        dy = dy.contiguous().float()
        dy_lp = dy if T == F32 else ops.cast_bf16(dy)
        if gs.wants(mod.weight):
            dwm = torch.zeros(D, wm.shape[1], dtype=torch.float32, device=dy.device)
            ops.linear_wgrad(dy_lp, patches, dwm)
            gs(mod.weight).add_(dwm[:, :K].view(D, k, k, C).permute(0, 3, 1, 2))
        if gs.wants(mod.bias):
            ops.bias_grad(dy_lp, gs(mod.bias))
        dx = None
        if ctx.needs_input_grad[0]:
            dp = ops.linear_dgrad(dy_lp, wm, F32)
            dx = torch.zeros_like(x)
            ops.conv_col2im(dp, B, H, H, C, k, mod.s, geo, dx, img_stride, row_off)
        return (dx,) + (None,) * 6 + gs.grads((mod.weight, mod.bias))


# ======================================================================= dw_bn projection
class _BN(nn.Module):
    """layers.BatchNormalization parameters and moving statistics (models/CvT(Par).py:94)."""

    def __init__(self, dim: int):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(dim))
        self.bias = nn.Parameter(torch.zeros(dim))
        self.register_buffer("running_mean", torch.zeros(dim))
        self.register_buffer("running_var", torch.ones(dim))


class DwBnProjection(nn.Module):
    """Projection(method='dw_bn') (models/CvT(Par).py:83-112): DepthwiseConv2D(3, 'same', no
    bias) + BatchNormalization.  ``weight`` [D, 1, 3, 3] (torch grouped-conv layout)."""

    def __init__(self, dim: int):
        super().__init__()
        self.weight = nn.Parameter(torch.zeros(dim, 1, 3, 3))
        self.bn = _BN(dim)

    def w9(self) -> Tensor:
        return self.weight.detach().view(-1, 9).t().contiguous()   # [3][3][D]


class CvTAttention(nn.Module):
    def __init__(self, dim: int, num_heads: int, qkv_bias: bool, methods=("dw_bn",) * 3, keras_dense: bool = False):
        super().__init__()
        self.num_heads = num_heads
        self.methods = tuple(methods)
        self.keras_dense = keras_dense
        for c, m in zip("qkv", self.methods):
            if m == "dw_bn":
                setattr(self, f"conv_proj_{c}", DwBnProjection(dim))
        self.proj_q, self.proj_k, self.proj_v = (Linear(dim, dim, bias=qkv_bias) for _ in range(3))
        if keras_dense:   # MultiHeadAttention's own EinsumDense projections (use_bias=True)
            self.mha_q, self.mha_k, self.mha_v, self.mha_o = (Linear(dim, dim) for _ in range(4))
        self.proj = Linear(dim, dim)

    def linear_pair(self, c: str):
        """(outer, inner) Linear modules of projection c ('q', 'k', 'v' or 'o'): the map applied
        is outer(inner(x)).  None for inner when the pair is held composed."""
        if c == "o":
            return self.proj, (self.mha_o if self.keras_dense else None)
        lin = getattr(self, f"proj_{c}")
        return (getattr(self, f"mha_{c}"), lin) if self.keras_dense else (lin, None)


def _compose(outer: Linear, inner: Linear):
    """W = W_outer W_inner, b = W_outer b_inner + b_outer (fp32, the library's fp32 GEMM)."""
    A, B = outer.weight.detach(), inner.weight.detach()
    D_out, D_mid = A.shape
    D_in = B.shape[1]
    W = torch.empty(D_out, D_in, dtype=F32, device=A.device)
    ops.gemm(A, B, True, False, D_out, D_in, D_mid, W)                      # W[o, i] = sum_j A[o, j] B[j, i]
    b = torch.empty(1, D_out, dtype=F32, device=A.device)
    bi = inner.bias.detach() if inner.bias is not None else torch.zeros(D_mid, device=A.device)
    ops.gemm(bi.view(1, D_mid), A, True, True, 1, D_out, D_mid, b, bias=outer.bias)   # b[o] = sum_j A[o, j] bi[j] + bo[o]
    return W, b.view(D_out)


def _chain(outer: Linear, inner: Linear, G: Tensor, gb: Tensor, gs) -> None:
    """The factors' gradients from the composed map's (G = dL/dW, gb = dL/db):
    dW_outer += G W_inner^T + gb b_inner^T, dW_inner += W_outer^T G, db_outer += gb,
    db_inner += W_outer^T gb (all fp32 GEMMs of the library; the outer product rides in the
    first GEMM as one extra, zero-padded K column)."""
    A, B = outer.weight.detach(), inner.weight.detach()
    D_out, D_mid = A.shape
    D_in = B.shape[1]
    if gs.wants(outer.weight):
        Kp = D_in + 32
        Gp = torch.zeros(D_out, Kp, dtype=F32, device=G.device)
        Bp = torch.zeros(D_mid, Kp, dtype=F32, device=G.device)
        Gp[:, :D_in] = G
        Bp[:, :D_in] = B
        if inner.bias is not None:
            Gp[:, D_in] = gb
            Bp[:, D_in] = inner.bias.detach()
        ops.gemm(Gp, Bp, True, True, D_out, D_mid, Kp, gs(outer.weight), ops.EPI_ACCUM)
    if gs.wants(inner.weight):
        ops.gemm(A, G, False, False, D_mid, D_in, D_out, gs(inner.weight), ops.EPI_ACCUM)
    if gs.wants(outer.bias):
        gs(outer.bias).add_(gb)
    if inner.bias is not None and gs.wants(inner.bias):
        ops.gemm(gb.view(1, D_out), A, True, False, 1, D_mid, D_out, gs(inner.bias).view(1, D_mid), ops.EPI_ACCUM)


class _Mlp(nn.Module):
    def __init__(self, dim: int, hidden: int):
        super().__init__()
        self.fc1 = Linear(dim, hidden)
        self.fc2 = Linear(hidden, dim)


class CvTBlock(nn.Module):
    """ConvTransformerBlock (models/CvT(Par).py:231-289) with dw_bn q/k/v."""

    def __init__(self, dim: int, num_heads: int, cfg: CvTConfig, methods=("dw_bn",) * 3):
        super().__init__()
        self.norm1 = LayerNorm(dim, cfg.ln_eps)
        self.attn = CvTAttention(dim, num_heads, cfg.qkv_bias, methods, cfg.keras_dense)
        self.tie_norms = cfg.tie_norms
        if not cfg.tie_norms:
            self.norm2 = LayerNorm(dim, cfg.ln_eps)
        self.mlp = _Mlp(dim, int(dim * cfg.mlp_ratio))
        self.cfg = cfg
        self.dim = dim

    @property
    def _norm2(self) -> LayerNorm:
        return self.norm1 if self.tie_norms else self.norm2

    def forward(self, x: Tensor, H: int, W: int, with_cls: bool, drop=None) -> Tensor:
        _check_cuda(x)
        return _CvTBlockFn.apply(x, self, H, W, with_cls, drop, *self.parameters())


class _CvTBlockFn(torch.autograd.Function):
    """Fused CvT block: LN1 -> 3 x (dw_bn -> q/k/v GEMM) -> attention -> out-proj + residual ->
    LN(2 or tied 1) -> fc1 + GELU -> fc2 + residual.  The cls row (stage 3) bypasses dw_bn
    (models/CvT(Par).py:146-150,164-176)."""

    @staticmethod
    def forward(ctx, x, blk, H, W, with_cls, drop, *params):
        cfg = blk.cfg
        T = ops.torch_dtype(cfg.dtype)
        B, N, D = x.shape
        M = B * N
        off = 1 if with_cls else 0
        a_ = blk.attn
        Hh = a_.num_heads
        dh = D // Hh
        scale = dh ** -0.5 if cfg.attn_scale == "head" else D ** -0.5
        x2 = x.contiguous().view(M, D)
        n1, n2 = blk.norm1, blk._norm2
        h, m1, r1 = ops.layernorm_fwd(x2, n1.weight, n1.bias, cfg.ln_eps, F32)
        qkv = torch.empty(M, 3 * D, dtype=T, device=x.device)
        saved_proj = []
        h_lp = None
        def weight_of(c):
            """(operand weight in T, bias) of projection c: the Linear's, or the composed pair's"""
            outer, inner = a_.linear_pair(c)
            if inner is None:
                return _lp(blk, outer.weight, T), outer.bias
            W, b = _compose(outer, inner)
            return (W if T == F32 else ops.cast_bf16(W)), b
        for c_i, (c, meth) in enumerate(zip("qkv", a_.methods)):
            z = mean = rstd = None
            if meth == "linear":                       # identity projection: the LN output itself
                if h_lp is None:
                    h_lp = h if T == F32 else ops.cast_bf16(h)
                inp = h_lp
            else:
                inp = torch.empty(M, D, dtype=T, device=x.device)
                if with_cls:
                    inp.view(B, N, D)[:, 0] = h.view(B, N, D)[:, 0].to(T)
                if meth == "dw_bn":
                    cp = getattr(a_, f"conv_proj_{c}")
                    z, mean, rstd = ops.dwconv_bn_fwd(h, B, H, W, cp.w9(), cp.bn.weight, cp.bn.bias, cfg.bn_eps,
                                                      cfg.bn_momentum, blk.training, cp.bn.running_mean,
                                                      cp.bn.running_var, inp, x_img=N, x_off=off, y_img=N, y_off=off)
                else:                                  # 'avg'
                    ops.avgpool3_fwd(h, B, H, W, inp, x_img=N, x_off=off, y_img=N, y_off=off,
                                     count_pad=cfg.avg_count_pad)
            wl, bl = weight_of(c)
            ops.gemm(inp, wl, True, True, M, D, D, qkv[:, c_i * D:(c_i + 1) * D], ops.EPI_STORE, bias=bl)
            saved_proj += [inp, z, mean, rstd, wl]
        o, lse = ops.attention_fwd(qkv, B, N, Hh, scale)
        dr = [None, None, None]
        if drop is not None:   # (seed, rate, site0): sites site0 (proj), +1 (GELU), +2 (fc2)
            dr = [(drop[0], drop[2] + j, drop[1]) for j in range(3)]
        wo, bo = weight_of("o")
        x1 = ops.linear_fwd(o, wo, bo, F32, ops.EPI_RESIDUAL, residual=x2, dropout=dr[0])
        h2, m2, r2 = ops.layernorm_fwd(x1, n2.weight, n2.bias, cfg.ln_eps, T)
        w1, w2 = _lp(blk, blk.mlp.fc1.weight, T), _lp(blk, blk.mlp.fc2.weight, T)
        act, u = ops.linear_fwd(h2, w1, blk.mlp.fc1.bias, T, ops.EPI_BIAS_GELU, dropout=dr[1],
                                aux_tiled=T == torch.bfloat16)
        out = ops.linear_fwd(act, w2, blk.mlp.fc2.bias, F32, ops.EPI_RESIDUAL, residual=x1, dropout=dr[2])
        ctx.save_for_backward(x2, h, m1, r1, qkv, o, lse, x1, h2, m2, r2, u, act, wo, w1, w2, *saved_proj)
        ctx.blk, ctx.dims, ctx.drop = blk, (B, N, D, H, W, with_cls, scale), drop
        return out.view(B, N, D)

    @staticmethod
    def backward(ctx, dout):
        (x2, h, m1, r1, qkv, o, lse, x1, h2, m2, r2, u, act, wo, w1, w2, *sp) = ctx.saved_tensors
        blk = ctx.blk
        B, N, D, H, W, with_cls, scale = ctx.dims
        cfg = blk.cfg
        T = h2.dtype
        lpT = None if T == F32 else T
        M = B * N
        off = 1 if with_cls else 0
        a_, mlp = blk.attn, blk.mlp
        n1, n2 = blk.norm1, blk._norm2
        ps = list(blk.parameters())
        gs = _sink(ctx, 6, ps)
        g2 = dout.contiguous().view(M, D).float()
        drop = ctx.drop
        if drop is None:
            g2_lp = g2 if T == F32 else ops.cast_bf16(g2)
        else:   # the fc2 branch was dropped: its dgrad/wgrad/bias see g2 * mask / (1 - p)
            g2_lp = ops.dropout_apply(g2, drop[0], drop[2] + 2, drop[1], T)
        # MLP
        du = ops.linear_dgrad(g2_lp, w2, T, ops.EPI_DGELU, aux=u, bias_grad=gs(mlp.fc1.bias),
                              aux_tiled=T == torch.bfloat16)
        if gs.wants(mlp.fc2.weight):
            ops.linear_wgrad(g2_lp, act, gs(mlp.fc2.weight))
        if gs.wants(mlp.fc2.bias):
            ops.bias_grad(g2_lp, gs(mlp.fc2.bias))
        dh2 = ops.linear_dgrad(du, w1, T)
        if gs.wants(mlp.fc1.weight):
            ops.linear_wgrad(du, h2, gs(mlp.fc1.weight))
        dx1, dx1_lp = ops.layernorm_bwd(dh2, x1, m2, r2, n2.weight, gs(n2.weight), gs(n2.bias), dres=g2,
                                        lp_dtype=lpT if drop is None else None)
        if drop is not None:   # the out-projection branch was dropped
            dx1_lp = ops.dropout_apply(dx1, drop[0], drop[2], drop[1], T)
        elif dx1_lp is None:
            dx1_lp = dx1
        def grads_of(c):
            """(wants W, wants b, dW dst, db dst) of projection c's applied map: the Linear's own
            gradients, or zeroed buffers of the composed map that chain_of passes to the factors"""
            outer, inner = a_.linear_pair(c)
            if inner is None:
                return gs.wants(outer.weight), gs.wants(outer.bias), gs(outer.weight), gs(outer.bias)
            if not any(gs.wants(p) for p in (outer.weight, outer.bias, inner.weight, inner.bias)):
                return False, False, None, None
            Dn = outer.weight.shape[0]
            return (True, True, torch.zeros(Dn, inner.weight.shape[1], dtype=F32, device=g2.device),
                    torch.zeros(Dn, dtype=F32, device=g2.device))

        def chain_of(c, G, gb):
            outer, inner = a_.linear_pair(c)
            if inner is not None and G is not None:
                _chain(outer, inner, G, gb, gs)
        # attention + out-projection
        do = ops.linear_dgrad(dx1_lp, wo, T)
        ww, wb, dWo, dbo = grads_of("o")
        if ww:
            ops.linear_wgrad(dx1_lp, o, dWo)
        if wb:
            ops.bias_grad(dx1_lp, dbo)
        chain_of("o", dWo, dbo)
        dqkv = ops.attention_bwd(qkv, o, do, lse, B, N, a_.num_heads, scale)
        # q/k/v GEMMs, the cls rows, dw_bn: all into the LN1-output gradient dh
        dh = torch.zeros(M, D, dtype=torch.float32, device=g2.device)
        for c_i, (c, meth) in enumerate(zip("qkv", a_.methods)):
            inp, z, mean, rstd, wl = sp[5 * c_i:5 * c_i + 5]
            dq = dqkv[:, c_i * D:(c_i + 1) * D].contiguous()
            dinp = ops.linear_dgrad(dq, wl, F32)
            ww, wb, dW, db_ = grads_of(c)
            if ww:
                ops.linear_wgrad(dq, inp, dW)
            if wb and db_ is not None:
                ops.bias_grad(dq, db_)
            chain_of(c, dW, db_)
            if meth == "linear":
                dh.add_(dinp)
                continue
            if with_cls:
                dh.view(B, N, D)[:, 0] += dinp.view(B, N, D)[:, 0]
            if meth == "avg":
                ops.avgpool3_bwd(dinp, B, H, W, dh, dy_img=N, dy_off=off, x_img=N, x_off=off,
                                 count_pad=cfg.avg_count_pad)
                continue
            cp = getattr(a_, f"conv_proj_{c}")
            dw9 = torch.zeros(9, D, dtype=torch.float32, device=g2.device)
            # (the BN parameter gradients always have a destination: the kernel writes them)
            dg = gs(cp.bn.weight)
            db = gs(cp.bn.bias)
            dg = dg if dg is not None else torch.zeros(D, device=g2.device)
            db = db if db is not None else torch.zeros(D, device=g2.device)
            ops.dwconv_bn_bwd(dinp, h, B, H, W, cp.w9(), cp.bn.weight, z, mean, rstd, dh, dw9,
                              dg, db, x_img=N, x_off=off, dy_img=N, dy_off=off)
            if gs.wants(cp.weight):
                gs(cp.weight).add_(dw9.t().reshape(D, 1, 3, 3))
        dx, _ = ops.layernorm_bwd(dh, x2, m1, r1, n1.weight, gs(n1.weight), gs(n1.bias), dres=dx1, lp_dtype=None)
        return (dx.view(B, N, D), None, None, None, None, None) + gs.grads(ps)


class ProcMlp(nn.Module):
    """Proc_Dense_1/2: Dense(hidden, relu) x 2 on the standardised process parameters
    (models/CvT(Par).py:343-344), on the small fp32 Dense kernels."""

    def __init__(self, dim: int, hidden: int):
        super().__init__()
        self.fc1 = Linear(dim, hidden)
        self.fc2 = Linear(hidden, hidden)

    def forward(self, proc: Tensor) -> Tensor:
        _check_cuda(proc)
        return _ProcMlpFn.apply(proc, self, *self.parameters())


class _ProcMlpFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mod, *params):
        x = x.contiguous().float()
        h = ops.dense_f32_fwd(x, mod.fc1.weight.detach(), mod.fc1.bias, ops.ACT_RELU)
        y = ops.dense_f32_fwd(h, mod.fc2.weight.detach(), mod.fc2.bias, ops.ACT_RELU)
        ctx.save_for_backward(x, h, y)
        ctx.mod = mod
        return y

    @staticmethod
    def backward(ctx, dy):
        x, h, y = ctx.saved_tensors
        mod = ctx.mod
        ps = list(mod.parameters())
        gs = _sink(ctx, 2, ps)

        def dst(w):   # dense_f32_bwd always writes dW: a scratch buffer for a frozen weight
            d = gs(w)
            return d if d is not None else torch.zeros_like(w)
        dy = dy.contiguous().float()
        dh = ops.dense_f32_bwd(dy, y, h, mod.fc2.weight.detach(), dst(mod.fc2.weight), gs(mod.fc2.bias),
                               ops.ACT_RELU)
        dx = ops.dense_f32_bwd(dh, h, x, mod.fc1.weight.detach(), dst(mod.fc1.weight), gs(mod.fc1.bias),
                               ops.ACT_RELU, want_dx=ctx.needs_input_grad[0])
        return (dx, None) + gs.grads(ps)


class _CvTHeadFn(torch.autograd.Function):
    """Dense(num_classes) on the normed features (models/CvT(Par).py:350) on the small-C head kernel."""

    @staticmethod
    def forward(ctx, y, head, w, b):
        y = y.contiguous().float()
        ctx.save_for_backward(y)
        ctx.head = head
        return ops.head_fwd(y, w.detach(), b)

    @staticmethod
    def backward(ctx, dlogits):
        (y,) = ctx.saved_tensors
        head = ctx.head
        gs = _sink(ctx, 2, (head.weight, head.bias))
        dw = gs(head.weight)
        dy = ops.head_bwd(dlogits.float(), y, head.weight.detach(), dw if dw is not None else torch.zeros_like(head.weight),
                          gs(head.bias))
        return (dy, None) + gs.grads((head.weight, head.bias))


# ======================================================================= stages + model
class CvTStageModule(nn.Module):
    def __init__(self, cin: int, st: CvTStage, cfg: CvTConfig):
        super().__init__()
        self.spec = st
        self.embed = ConvEmbedSame(cin, st.embed_dim, st.patch_size, st.stride, st.padding, cfg.embed_norm,
                                   cfg.ln_eps, cfg.dtype)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, st.embed_dim)) if st.with_cls_token else None
        self.blocks = nn.ModuleList([CvTBlock(st.embed_dim, st.num_heads, cfg, qkv_methods(st))
                                     for _ in range(st.depth)])


class CvT(nn.Module):
    """create_cvt_model's image branch (models/CvT(Par).py:292-340) + LN(cls) -> Dense head.
    ``forward(x [B, Cin, S, S] fp32) -> logits [B, num_classes]``."""

    def __init__(self, cfg: CvTConfig):
        super().__init__()
        self.cfg = cfg
        self.drop_seed: Optional[int] = None   # fixed dropout seed (tests); None = drawn per forward
        cin = cfg.in_chans
        for i, st in enumerate(cfg.stages):
            self.add_module(f"stage{i}", CvTStageModule(cin, st, cfg))
            cin = st.embed_dim
        self.norm = LayerNorm(cin, cfg.ln_eps)
        if cfg.proc_dim:
            self.proc = ProcMlp(cfg.proc_dim, cfg.proc_hidden)
            cin += cfg.proc_hidden
        self.head = Linear(cin, cfg.num_classes)

    def stages(self) -> List[CvTStageModule]:
        return [getattr(self, f"stage{i}") for i in range(len(self.cfg.stages))]

    def forward_features(self, img: Tensor) -> Tensor:
        _check_cuda(img)
        B, C, S, _ = img.shape
        # NCHW image -> NHWC rows (Cin = 1 for the SLS grayscale input: a view)
        x = img.float().reshape(B * S * S, 1) if C == 1 else img.float().permute(0, 2, 3, 1).reshape(B * S * S, C)
        H, img_stride, row_off = S, S * S, 0
        tok = None
        t = None
        cap = getattr(self, "_capture_stage", None)
        stages = self.stages()
        drop = _drop_args(self, self.cfg.drop_rate, 0)
        bi = 0   # global block index: dropout sites 3*bi .. 3*bi+2
        for si, stg in enumerate(stages):
            st = stg.spec
            t, H = stg.embed(x, B, H, img_stride, row_off)          # [B, H*H, D] fp32
            D = st.embed_dim
            if stg.cls_token is not None:
                t = torch.cat([stg.cls_token.expand(B, 1, D), t], dim=1)
            for blk in stg.blocks:
                d = None if drop is None else (drop[0], drop[1], 3 * bi)
                t = blk(t, H, H, stg.cls_token is not None, d)
                bi += 1
            if cap is not None and si == cap % len(stages):     # Grad-CAM's activation (vitmi.gradcam)
                if t.requires_grad:
                    t.retain_grad()
                self._captured = (t, H, stg.cls_token is not None)
            N = t.shape[1]
            if stg.cls_token is not None:
                tok = t[:, 0]
                img_stride, row_off = N, 1
            else:
                img_stride, row_off = N, 0
            x = t.reshape(B * N, D)
        if tok is None:
            return self.norm(t).mean(dim=1)
        return self.norm(tok)

    def forward(self, img: Tensor, proc: Optional[Tensor] = None) -> Tensor:
        """Image features [++ Proc_Dense_2 features (:347)] -> Final_Dense (:350)."""
        f = self.forward_features(img)
        if self.cfg.proc_dim:
            if proc is None:
                raise ValueError("this CvT takes process parameters (cfg.proc_dim > 0): forward(img, proc)")
            f = torch.cat([f, self.proc(proc.to(f.device, torch.float32))], dim=1)
        return _CvTHeadFn.apply(f, self.head, self.head.weight, self.head.bias)

    def reset_parameters(self, seed: int = 0) -> None:
        """Keras initialisers: glorot_uniform kernels (Dense, Conv2D, DepthwiseConv2D; the
        MultiHeadAttention EinsumDense kernels with Keras' fans of their 3-d shapes), zero
        biases / betas / cls token, unit gammas."""
        g = torch.Generator().manual_seed(seed)
        with torch.no_grad():
            for name, p in self.named_parameters():
                leaf, parent = name.rsplit(".", 1)[-1], name.split(".")[-2]
                if parent in ("norm1", "norm2", "norm", "bn"):
                    t = torch.ones(p.shape) if leaf == "weight" else torch.zeros(p.shape)
                elif leaf == "bias":
                    t = torch.zeros(p.shape)
                elif leaf == "cls_token":              # add_weight(initializer='zeros'), :245
                    t = torch.zeros(p.shape)
                else:
                    rf = p.shape[2] * p.shape[3] if p.dim() == 4 else 1
                    fan_in, fan_out = p.shape[1] * rf, p.shape[0] * rf
                    if "conv_proj" in name:               # depthwise: one input channel per filter
                        fan_in, fan_out = rf, rf
                    if ".mha_" in name:   # EinsumDense kernels [D, H, dh] (q/k/v) and [H, dh, D] (output)
                        D, Hh = p.shape[0], self.cfg.stages[int(name[5:name.index(".")])].num_heads
                        fan_in, fan_out = (D, D * Hh) if ".mha_o." in name else (Hh * D, (D // Hh) * D)
                    lim = (6.0 / (fan_in + fan_out)) ** 0.5
                    t = (torch.rand(p.shape, generator=g) * 2 - 1) * lim
                p.copy_(t.to(p.device))
            for m in self.modules():
                if isinstance(m, _BN):
                    m.running_mean.zero_()
                    m.running_var.fill_(1.0)

    def load_param_dict(self, d: Dict[str, Tensor]) -> None:
        mine = dict(self.named_parameters())
        missing = set(mine) - set(d)
        if missing:
            raise KeyError(f"missing parameters: {sorted(missing)[:5]}")
        with torch.no_grad():
            for k, p in mine.items():
                p.copy_(d[k].reshape(p.shape).to(p.device, p.dtype))
