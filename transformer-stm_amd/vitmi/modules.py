"""nn.Module API of the MI355X ViT path.

Module tree and names follow the reference's layers (Keras ``ConvEmbed`` /
``ConvAttention`` / ``ConvTransformerBlock`` / ``create_cvt_model``,
``models/CvT(Par).py:194-354``) in the nn.Module form of the vendored Microsoft
CvT (``old_codes/MS_CvT.py``: ``Mlp`` :53, ``Attention`` :77, ``Block`` :289,
``ConvEmbed`` :336, ``VisionTransformer`` :372, head :605-623):

    VisionTransformer(cfg)
      patch_embed: ConvEmbed      (.proj Conv2d-shaped params, optional .norm)
      cls_token, pos_embed
      blocks[i]: Block            (.norm1, .attn: Attention(.qkv, .proj), .norm2, .mlp: Mlp(.fc1, .fc2))
      norm: LayerNorm, head: Linear

Every forward and backward runs the hand-written gfx950 kernels of libvitmi.so
through fused ``torch.autograd.Function``s (one per block: LN1 -> QKV -> attention
-> out-proj + residual -> LN2 -> fc1 + GELU -> fc2 + residual).  Parameters are
ordinary fp32 ``nn.Parameter``s, so ``torch.optim``, ``state_dict`` and the DP
reducer work unchanged.  The Functions RETURN their parameters' gradients to autograd
(``vitmi/grads.py``: the kernels accumulate each into its final buffer, for a model with a
ParamArena the arena view that AccumulateGrad then keeps as ``.grad``), so parameter hooks,
DistributedDataParallel and ``torch.autograd.grad`` see them, and frozen parameters get
none.  In ``bf16`` mode GEMM/attention operands are bf16 (fp32 accumulate,
fp32 residual stream, LN statistics, softmax and head); in ``fp32`` mode every
product is exact fp32 (f32-input MFMA).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from . import ops
from .config import ViTConfig
from .grads import GradSink

Tensor = torch.Tensor
F32 = torch.float32

# A backward that already holds a bf16 copy of the gradient it returns (the LayerNorm backward
# writes both) hands it to the next backward up the chain as an attribute of the returned
# tensor object, so that backward does not re-cast its incoming gradient.  The copy lives and
# dies with that tensor object (no address-keyed table that a later allocation could alias),
# and it is used only while the tensor is unmodified: autograd may accumulate another gradient
# into it in place, which bumps its version counter.
_LP_ATTR = "_vitmi_lp"
LP_STATS = {"hit": 0, "miss": 0}     # test hook: how often the handed-over copy was used


def _drop_args(mod: nn.Module, rate: float, site0: int):
    """(seed, rate, site0) for a training-mode forward with dropout, else None.  The seed is
    ``mod.drop_seed`` when set (parity tests), otherwise drawn from torch's default CPU
    generator, so ``torch.manual_seed`` makes the masks reproducible."""
    if not mod.training or rate <= 0.0 or not torch.is_grad_enabled():
        return None
    seed = getattr(mod, "drop_seed", None)
    if seed is None:
        seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())
    return (int(seed), float(rate), site0)


def _sink(ctx, first: int, params, arena=None, extra=()) -> GradSink:
    """GradSink over the Function inputs ``params`` starting at input index ``first`` (plus
    ``extra`` (index, param) pairs)."""
    return GradSink(ctx, [(first + i, q) for i, q in enumerate(params)] + list(extra), arena)


def _lp(mod: nn.Module, p: Tensor, T: torch.dtype) -> Tensor:
    """Operand copy of a weight in the compute dtype."""
    if T == F32:
        return p.detach()
    arena = getattr(mod, "_arena", None)
    if arena is not None:
        return arena.lp(p)
    return ops.cast_bf16(p.detach().contiguous())


def _take_lp(g: Tensor, T: torch.dtype, src: Optional[Tensor] = None) -> Tensor:
    """``g`` (fp32, contiguous) in the compute dtype.  ``src`` is the tensor object autograd
    passed in (``g`` may be a view of it): its handed-over bf16 copy is used when it is still
    current, otherwise ``g`` is cast."""
    if T == F32:
        return g
    src = g if src is None else src
    ent = src.__dict__.pop(_LP_ATTR, None)
    if ent is not None:
        lp, version, ptr = ent
        if src._version == version and src.data_ptr() == ptr and lp.numel() == g.numel() and lp.dtype == T:
            LP_STATS["hit"] += 1
            return lp.view(g.shape)
    LP_STATS["miss"] += 1
    return ops.cast_bf16(g.contiguous())


def _handover(g: Tensor, lp: Optional[Tensor]) -> Tensor:
    """Attach the bf16 copy ``lp`` of ``g`` to the tensor object a backward returns."""
    if lp is not None:
        g.__dict__[_LP_ATTR] = (lp, g._version, g.data_ptr())
    return g


def _is_vitmi_node(x: Tensor) -> bool:
    """x was produced by a vitmi Function: its backward consumes the handed-over bf16 copy of
    the gradient.  (A leaf or a torch op would keep the tensor object, e.g. as a leaf's .grad,
    and the copy with it: ADVICE r03.)"""
    fn = x.grad_fn
    return fn is not None and getattr(type(fn), "_forward_cls", None) in _HANDOVER_FNS


def _folds(backward):
    """Run a Function's backward with its partial-sum folds queued and launched together at
    its end (ops.deferred_folds): one fold launch per backward, and every parameter gradient it
    returns is final in stream order when it returns."""
    def run(ctx, *grads):
        with ops.deferred_folds():
            return backward(ctx, *grads)
    run.__doc__ = backward.__doc__
    return run


def _check_cuda(x: Tensor):
    if not x.is_cuda:
        raise RuntimeError("vitmi modules run only on the GPU (HIP); there is no CPU path")


# ======================================================================= leaves
class LayerNorm(nn.Module):
    """layers.LayerNormalization(epsilon=eps) over the last dim (models/CvT(Par).py:248)."""

    def __init__(self, dim: int, eps: float = 1e-6):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))
        self.bias = nn.Parameter(torch.zeros(dim))

    def forward(self, x: Tensor) -> Tensor:
        _check_cuda(x)
        return _LayerNormFn.apply(x, self, self.weight, self.bias)


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mod, w, b):
        xs = x.contiguous().float()
        y, mean, rstd = ops.layernorm_fwd(xs, w, b, mod.eps, F32)
        ctx.save_for_backward(xs, mean, rstd)
        ctx.mod = mod
        return y.view(x.shape)

    @staticmethod
    @_folds
    def backward(ctx, dy):
        xs, mean, rstd = ctx.saved_tensors
        mod = ctx.mod
        ps = (mod.weight, mod.bias)
        gs = _sink(ctx, 2, ps, getattr(mod, "_arena", None))
        dx, _ = ops.layernorm_bwd(dy.contiguous().float(), xs, mean, rstd, mod.weight, gs(mod.weight), gs(mod.bias))
        return (dx.view(xs.shape), None) + gs.grads(ps)


class Linear(nn.Linear):
    """Parameter container with nn.Linear's names/shapes (keras Dense); the math runs in
    the fused Functions below or, standalone, through vitmi GEMMs."""

    def forward(self, x: Tensor) -> Tensor:  # standalone use: fp32 GEMM
        _check_cuda(x)
        return _LinearFn.apply(x, self, self.weight, self.bias)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mod, w, b):
        xs = x.contiguous().float()
        y = ops.linear_fwd(xs.view(-1, xs.shape[-1]), w.detach(), b, F32)
        ctx.save_for_backward(xs)
        ctx.mod = mod
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        (xs,) = ctx.saved_tensors
        mod = ctx.mod
        ps = (mod.weight, mod.bias)
        gs = _sink(ctx, 2, ps, getattr(mod, "_arena", None))
        dy2 = dy.contiguous().float().view(-1, dy.shape[-1])
        x2 = xs.view(-1, xs.shape[-1])
        dx = ops.linear_dgrad(dy2, mod.weight.detach(), F32).view(xs.shape) if ctx.needs_input_grad[0] else None
        if gs.wants(mod.weight):
            ops.linear_wgrad(dy2, x2, gs(mod.weight))
        if gs.wants(mod.bias):
            ops.bias_grad(dy2, gs(mod.bias))
        return (dx, None) + gs.grads(ps)


# ======================================================================= attention / MLP
class Attention(nn.Module):
    """ConvAttention with identity ('linear') projections (models/CvT(Par).py:115-191):
    fused Q/K/V linear [D -> 3D], softmax(QK^T * scale) V, out-projection.
    ``forward(x, h, w)`` mirrors old_codes/MS_CvT.py:190 (h, w unused for 'linear')."""

    def __init__(self, dim: int, num_heads: int, qkv_bias: bool = True, attn_scale: str = "head",
                 dtype: str = "bf16"):
        super().__init__()
        if dim % num_heads or dim // num_heads != 64:
            raise ValueError("vitmi Attention needs head_dim == 64")
        self.dim, self.num_heads = dim, num_heads
        self.scale = (dim // num_heads) ** -0.5 if attn_scale == "head" else dim ** -0.5
        self.qkv = Linear(dim, 3 * dim, bias=qkv_bias)
        self.proj = Linear(dim, dim)
        self.dtype = dtype

    def forward(self, x: Tensor, h: Optional[int] = None, w: Optional[int] = None) -> Tensor:
        _check_cuda(x)
        return _AttentionFn.apply(x, self, *self._params())

    def _params(self):
        return [p for p in (self.qkv.weight, self.qkv.bias, self.proj.weight, self.proj.bias) if p is not None]


class _AttentionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mod, *params):
        T = ops.torch_dtype(mod.dtype)
        B, N, D = x.shape
        x2 = x.contiguous().float().view(B * N, D)
        xo = x2 if T == F32 else ops.cast_bf16(x2)
        wq, wo = _lp(mod, mod.qkv.weight, T), _lp(mod, mod.proj.weight, T)
        qkv = ops.linear_fwd(xo, wq, mod.qkv.bias, T)
        o, lse = ops.attention_fwd(qkv, B, N, mod.num_heads, mod.scale)
        y = ops.linear_fwd(o, wo, mod.proj.bias, F32)
        ctx.save_for_backward(xo, qkv, o, lse, wq, wo)
        ctx.mod, ctx.shape = mod, (B, N, D)
        return y.view(B, N, D)

    @staticmethod
    @_folds
    def backward(ctx, dy):
        xo, qkv, o, lse, wq, wo = ctx.saved_tensors
        mod, (B, N, D) = ctx.mod, ctx.shape
        ps = mod._params()
        gs = _sink(ctx, 2, ps, getattr(mod, "_arena", None))
        T = xo.dtype
        g = dy.contiguous().float().view(B * N, D)
        g_lp = _take_lp(g, T, dy)
        do = ops.linear_dgrad(g_lp, wo, T)
        if gs.wants(mod.proj.weight):
            ops.linear_wgrad(g_lp, o, gs(mod.proj.weight))
        if gs.wants(mod.proj.bias):
            ops.bias_grad(g_lp, gs(mod.proj.bias))
        dqkv = ops.attention_bwd(qkv, o, do, lse, B, N, mod.num_heads, mod.scale, bias_grad=gs(mod.qkv.bias))
        dx = ops.linear_dgrad(dqkv, wq, F32)
        if gs.wants(mod.qkv.weight):
            ops.linear_wgrad(dqkv, xo, gs(mod.qkv.weight))
        return (dx.view(B, N, D), None) + gs.grads(ps)


class Mlp(nn.Module):
    """Dense(hidden, exact GELU) -> Dense(out)  (models/CvT(Par).py:253-258; MS_CvT.py:53-74)."""

    def __init__(self, in_features: int, hidden_features: int, dtype: str = "bf16"):
        super().__init__()
        self.fc1 = Linear(in_features, hidden_features)
        self.fc2 = Linear(hidden_features, in_features)
        self.dtype = dtype

    def forward(self, x: Tensor) -> Tensor:
        _check_cuda(x)
        return _MlpFn.apply(x, self, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias)


class _MlpFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mod, *params):
        T = ops.torch_dtype(mod.dtype)
        shp = x.shape
        x2 = x.contiguous().float().view(-1, shp[-1])
        xo = x2 if T == F32 else ops.cast_bf16(x2)
        w1, w2 = _lp(mod, mod.fc1.weight, T), _lp(mod, mod.fc2.weight, T)
        a, u = ops.linear_fwd(xo, w1, mod.fc1.bias, T, ops.EPI_BIAS_GELU, aux_tiled=T != F32)
        y = ops.linear_fwd(a, w2, mod.fc2.bias, F32)
        ctx.save_for_backward(xo, a, u, w1, w2)
        ctx.mod, ctx.shape = mod, shp
        return y.view(shp)

    @staticmethod
    @_folds
    def backward(ctx, dy):
        xo, a, u, w1, w2 = ctx.saved_tensors
        mod = ctx.mod
        ps = (mod.fc1.weight, mod.fc1.bias, mod.fc2.weight, mod.fc2.bias)
        gs = _sink(ctx, 2, ps, getattr(mod, "_arena", None))
        T = xo.dtype
        g = dy.contiguous().float().view(-1, dy.shape[-1])
        g_lp = _take_lp(g, T, dy)
        du = ops.linear_dgrad(g_lp, w2, T, ops.EPI_DGELU, aux=u, bias_grad=gs(mod.fc1.bias), aux_tiled=T != F32)
        if gs.wants(mod.fc2.weight):
            ops.linear_wgrad(g_lp, a, gs(mod.fc2.weight))
        if gs.wants(mod.fc2.bias):
            ops.bias_grad(g_lp, gs(mod.fc2.bias))
        dx = ops.linear_dgrad(du, w1, F32)
        if gs.wants(mod.fc1.weight):
            ops.linear_wgrad(du, xo, gs(mod.fc1.weight))
        return (dx.view(ctx.shape), None) + gs.grads(ps)


# ======================================================================= block
class Block(nn.Module):
    """Pre-LN transformer block ``x += Attn(LN1(x)); x += MLP(LN2(x))``
    (ConvTransformerBlock.call, models/CvT(Par).py:261-289; Block.forward, MS_CvT.py:325-333).
    ``tie_norms=True`` reproduces the Keras model's single ``norm1`` used twice (:248,272,278)."""

    def __init__(self, dim: int, num_heads: int, mlp_ratio: float = 4.0, qkv_bias: bool = True,
                 eps: float = 1e-6, attn_scale: str = "head", tie_norms: bool = False, dtype: str = "bf16"):
        super().__init__()
        self.norm1 = LayerNorm(dim, eps)
        self.attn = Attention(dim, num_heads, qkv_bias, attn_scale, dtype)
        self.tie_norms = tie_norms
        if not tie_norms:
            self.norm2 = LayerNorm(dim, eps)
        self.mlp = Mlp(dim, int(dim * mlp_ratio), dtype)
        self.dtype = dtype
        # the precision knobs' qkv GEMM: split operands (True), plain bf16 (False) or, for 'bf16f8',
        # the weight-side correction alone ("weight", VITMI_BF16F8W).  Of the qkv GEMM's error, the
        # weight rounding's is the part that matters (every token's q and k move together; the
        # activations' rounding averages out): depth-12 ViT-B logits over 8 images, RMS / max, 1.7e-4
        # / 3.4e-4 with "weight" against 3.4e-4 / 7.1e-4 plain, smoke model 1.8e-4 against 9.6e-4
        # (tools/precision_sides.py, profiles/r06_sides/), at 1.5K- instead of 2K-equivalent work.
        # Default: split for 'bf16x3', "weight" for 'bf16f8' where dim % 128 == 0 (else plain);
        # ViTConfig.split_qkv overrides
        self.split_qkv = True if dtype == "bf16x3" else ("weight" if dtype == "bf16f8" and dim % 128 == 0 else False)
        self.eps = eps
        self.drop_rate = 0.0     # set by VisionTransformer / the caller (Keras default 0.1)
        self.drop_seed: Optional[int] = None   # fixed seed (tests); None = drawn per forward

    @property
    def _norm2(self) -> LayerNorm:
        return self.norm1 if self.tie_norms else self.norm2

    def forward(self, x: Tensor, h: Optional[int] = None, w: Optional[int] = None) -> Tensor:
        _check_cuda(x)
        return _BlockFn.apply(x, self, None, False, _drop_args(self, self.drop_rate, 0), _is_vitmi_node(x),
                              *self.parameters())


class _BlockFn(torch.autograd.Function):
    """Fused block.  ``handover``: the input was produced by a vitmi Function whose backward
    takes the bf16 copy of the input gradient (the LN1 backward writes it beside the fp32
    gradient).  ``prev_fc2_bias``: the fc2 bias of the block feeding this one; its gradient is
    colsum(d input), produced for free by this block's LN1 backward and returned for that input.
    ``fc2_bias_done``: this block's own fc2 bias gradient is supplied by its consumer (next block
    or head).  ``drop``: (seed, rate, site0) -> training-mode dropout
    (models/CvT(Par).py:189,255,257) at sites site0 (out-projection), site0+1 (GELU output),
    site0+2 (fc2), fused into the GEMM epilogues; the backward regenerates the masks
    (vitmi_dropout_apply)."""

    @staticmethod
    def forward(ctx, x, blk, prev_fc2_bias, fc2_bias_done, drop, handover, *params):
        T = ops.torch_dtype(blk.dtype)
        B, N, D = x.shape
        M = B * N
        H = blk.attn.num_heads
        x2 = x.contiguous().float().view(M, D)
        n1, n2 = blk.norm1, blk._norm2
        a_ = blk.attn
        wq, wo = _lp(blk, a_.qkv.weight, T), _lp(blk, a_.proj.weight, T)
        w1, w2 = _lp(blk, blk.mlp.fc1.weight, T), _lp(blk, blk.mlp.fc2.weight, T)
        ctx.blk, ctx.shape = blk, (B, N, D)
        ctx.prev_bias, ctx.bias_done, ctx.drop = prev_fc2_bias, fc2_bias_done, drop
        ctx.handover = handover
        ctx.aux_tiled = T != F32
        if blk.dtype in ("bf16x3", "bf16f8"):
            out = _BlockFn._forward_x3(ctx, x2, blk, B, N, D, H, drop, (wq, wo, w1, w2))
            return out.view(B, N, D)
        h1, m1, r1 = ops.layernorm_fwd(x2, n1.weight, n1.bias, blk.eps, T)
        qkv = ops.linear_fwd(h1, wq, a_.qkv.bias, T)
        o, lse = ops.attention_fwd(qkv, B, N, H, a_.scale)
        dr = [None, None, None]
        if drop is not None:
            seed, rate, site0 = drop
            dr = [(seed, site0 + j, rate) for j in range(3)]
        x1 = ops.linear_fwd(o, wo, a_.proj.bias, F32, ops.EPI_RESIDUAL, residual=x2, dropout=dr[0])
        h2, m2, r2 = ops.layernorm_fwd(x1, n2.weight, n2.bias, blk.eps, T)
        # gelu' stays in the tile-native layout between fc1's epilogue and fc2's dgrad (bf16)
        act, u = ops.linear_fwd(h2, w1, blk.mlp.fc1.bias, T, ops.EPI_BIAS_GELU, dropout=dr[1], aux_tiled=T != F32)
        out = ops.linear_fwd(act, w2, blk.mlp.fc2.bias, F32, ops.EPI_RESIDUAL, residual=x1, dropout=dr[2])
        ctx.save_for_backward(x2, h1, m1, r1, qkv, o, lse, x1, h2, m2, r2, u, act, wq, wo, w1, w2)
        return out.view(B, N, D)

    @staticmethod
    def _forward_x3(ctx, x2, blk, B, N, D, H, drop, wlp):
        """The precision knob's forward (ViTConfig dtype 'bf16x3'; tools/precision_emulate.py):
        the qkv, out-projection, fc1 and fc2 GEMMs take split-bf16 operands (weights and the
        LayerNorm / attention / GELU outputs as hi + lo, one GEMM over K' = 3K).  The LayerNorm
        and attention kernels write their outputs split (VITMI_BF16X3, vitmi_attention_fwd_x3);
        q, k, v and the softmax P are bf16 (emulated cost 1.5-1.8e-4 of logits at depth 12).  The
        backward is the bf16 one, on the hi parts (row-strided views of the split operands) and
        the attention forward's own bf16 O and lse (so P's rows in the backward sum to 1).

        dtype 'bf16f8' (tools/precision_emulate_fp8.py): the same operands as VITMI_BF16F8 rows,
        [hi | e4m3 hi8, lo8 * 2^9]: hi.hi in bf16 and both corrections as one block-scaled fp8
        product, 2K-equivalent MFMA work instead of 3K (emulated 1.8-2.3e-4 at depth 12).

        blk.split_qkv False: the qkv GEMM runs on plain bf16 operands (LN1 writes bf16, the
        weight's bf16 shadow); "weight" ('bf16f8'): LN1 writes VITMI_BF16F8W rows [hi | hi8] and the
        weight is split [hi | lo8], so the GEMM adds hi8 . lo8 / 2^9 to hi . hi (the weight-side
        correction alone, K/128 e4m3 K-steps); the other three GEMMs as above."""
        f8 = blk.dtype == "bf16f8"
        sq = blk.split_qkv is True
        wq8 = f8 and blk.split_qkv == "weight" and D % 128 == 0
        if drop is not None:
            raise ValueError(f"vitmi: dtype '{blk.dtype}' is the parity / evaluation knob; dropout is not supported")
        n1, n2 = blk.norm1, blk._norm2
        a_, mlp = blk.attn, blk.mlp
        split = ops.split_bf16f8 if f8 else ops.split_bf16x3
        ln_out = ops.BF16F8 if f8 else ops.BF16X3

        weights = ((a_.qkv.weight,) if sq or wq8 else ()) + (a_.proj.weight, mlp.fc1.weight, mlp.fc2.weight)
        if f8:   # the block's split weights in one launch
            pats = [3 if wq8 and i == 0 else 1 for i in range(len(weights))]
            split_w = dict(zip(map(id, weights), ops.split_bf16f8_weights(weights, pats)))

        def w3(p):
            return split_w[id(p)] if f8 else split(p.detach(), 1)[0]
        h1_3, m1, r1 = ops.layernorm_fwd(x2, n1.weight, n1.bias, blk.eps,
                                         ln_out if sq else ops.BF16F8W if wq8 else torch.bfloat16)
        # the qkv GEMM's operands: split, weight-side split, or plain bf16 (h1 and the weight's bf16 shadow)
        qa, qw, qf8 = ((h1_3, w3(a_.qkv.weight), f8) if sq else (h1_3, split_w[id(a_.qkv.weight)], "w") if wq8
                       else (h1_3, wlp[0], False))
        if N <= ops.ATTN_SEQ_MAX:   # q, k, v leave the GEMM epilogue in bf16
            qkv = ops.linear_fwd(qa, qw, a_.qkv.bias, torch.bfloat16, f8=qf8)
            o, o3, lse = (ops.attention_fwd_f8 if f8 else ops.attention_fwd_x3)(qkv, B, N, H, a_.scale)
        else:   # streamed kernels (N > 256): O from the fp32 kernel, o / lse from the bf16 one
            qkvf = ops.linear_fwd(qa, qw, a_.qkv.bias, F32, f8=qf8)
            qkv = ops.cast_bf16(qkvf)
            of, _ = ops.attention_fwd(qkvf, B, N, H, a_.scale)
            del qkvf
            o3, _ = split(of, 0)
            del of
            o, lse = ops.attention_fwd(qkv, B, N, H, a_.scale)
        x1 = ops.linear_fwd(o3, w3(a_.proj.weight), a_.proj.bias, F32, ops.EPI_RESIDUAL, residual=x2, f8=f8)
        del o3
        h2_3, m2, r2 = ops.layernorm_fwd(x1, n2.weight, n2.bias, blk.eps, ln_out)
        # GELU in the fc1 epilogue, its output split there (VITMI_EPI_SPLIT_X3 / _F8); gelu' saved
        # in the tile-native layout of the bf16 path
        act3, dg = ops.linear_fwd(h2_3, w3(mlp.fc1.weight), mlp.fc1.bias, torch.bfloat16, ops.EPI_BIAS_GELU,
                                  aux_tiled=True, split_x3=not f8, split_f8=f8, f8=f8)
        out = ops.linear_fwd(act3, w3(mlp.fc2.weight), mlp.fc2.bias, F32, ops.EPI_RESIDUAL, residual=x1, f8=f8)
        # the bf16 backward's operands: hi parts of the split activations (row-strided views)
        h1, h2, act = (h1_3[:, :D] if sq or wq8 else h1_3), h2_3[:, :D], act3[:, :mlp.fc1.weight.shape[0]]
        ctx.aux_tiled = True
        ctx.save_for_backward(x2, h1, m1, r1, qkv, o, lse, x1, h2, m2, r2, dg, act, *wlp)
        return out

    @staticmethod
    @_folds
    def backward(ctx, dout):
        (x2, h1, m1, r1, qkv, o, lse, x1, h2, m2, r2, u, act, wq, wo, w1, w2) = ctx.saved_tensors
        blk, (B, N, D) = ctx.blk, ctx.shape
        M = B * N
        T = h1.dtype
        lpT = None if T == F32 else T
        n1, n2 = blk.norm1, blk._norm2
        a_, mlp = blk.attn, blk.mlp
        ps = list(blk.parameters())
        prev = ctx.prev_bias
        gs = _sink(ctx, 6, ps, getattr(blk, "_arena", None), extra=[(2, prev)] if prev is not None else [])
        g2 = dout.contiguous().float().view(M, D)
        drop = ctx.drop
        if drop is None:
            g2_lp = _take_lp(g2, T, dout)
        else:
            # the fc2 branch was dropped: its dgrad/wgrad/bias see g2 * mask / (1 - p)
            dout.__dict__.pop(_LP_ATTR, None)
            seed, rate, site0 = drop
            g2_lp = ops.dropout_apply(g2, seed, site0 + 2, rate, T)
        # the block's weight gradients, grouped per ops.WGRAD_GROUP (default: the out-projection's
        # and qkv's in one split-K launch over both outputs' tiles and one reduction, at qkv's
        # point; the MLP pair where du has just been written)
        wg = []
        wr = _WgradRunner()
        # MLP branch
        # fc1's bias gradient = column sums of du, fused into the DGELU epilogue
        du = ops.linear_dgrad(g2_lp, w2, T, ops.EPI_DGELU, aux=u, bias_grad=gs(mlp.fc1.bias), aux_tiled=ctx.aux_tiled)
        if gs.wants(mlp.fc2.weight):
            wg.append((g2_lp, act, gs(mlp.fc2.weight)))
        if not ctx.bias_done and gs.wants(mlp.fc2.bias):
            ops.bias_grad(g2_lp, gs(mlp.fc2.bias))
        if gs.wants(mlp.fc1.weight):
            wg.append((du, h2, gs(mlp.fc1.weight)))
        if ops.WGRAD_GROUP in (0, 2, 3):
            wr.run(ops.linear_wgrad_group if ops.WGRAD_GROUP == 2 else _each_wgrad, wg)
            wg = []
        dh2 = ops.linear_dgrad(du, w1, T)
        # LN2 backward + residual; its column sums of dx1 are the out-proj bias grad
        if drop is None:
            dx1, dx1_lp = ops.layernorm_bwd(dh2, x1, m2, r2, n2.weight, gs(n2.weight), gs(n2.bias),
                                            dres=g2, lp_dtype=lpT, dxsum=gs(a_.proj.bias))
            if dx1_lp is None:
                dx1_lp = dx1
        else:
            dx1, _ = ops.layernorm_bwd(dh2, x1, m2, r2, n2.weight, gs(n2.weight), gs(n2.bias),
                                       dres=g2, lp_dtype=None)
            dx1_lp = ops.dropout_apply(dx1, seed, site0, rate, T)
            if gs.wants(a_.proj.bias):
                ops.bias_grad(dx1_lp, gs(a_.proj.bias))
        # attention branch
        do = ops.linear_dgrad(dx1_lp, wo, T)
        if gs.wants(a_.proj.weight):
            wg.append((dx1_lp, o, gs(a_.proj.weight)))
        if ops.WGRAD_GROUP == 0:
            wr.run(_each_wgrad, wg)
            wg = []
        # the qkv bias gradient (column sums of dqkv) comes out of the attention backward kernels
        dqkv = ops.attention_bwd(qkv, o, do, lse, B, N, a_.num_heads, a_.scale, bias_grad=gs(a_.qkv.bias))
        if gs.wants(a_.qkv.weight):
            wg.append((dqkv, h1, gs(a_.qkv.weight)))
        if ops.WGRAD_GROUP == 0:
            wr.run(_each_wgrad, wg)
            wg = []
        dh1 = ops.linear_dgrad(dqkv, wq, T)
        wr.run(ops.linear_wgrad_group, wg)
        # the bf16 copy of dx is for a consumer that takes it (the block below); the patch
        # embedding's backward reads dx in fp32
        want_lp = drop is None and ctx.handover
        dx, dx_lp = ops.layernorm_bwd(dh1, x2, m1, r1, n1.weight, gs(n1.weight), gs(n1.bias),
                                      dres=dx1, lp_dtype=lpT if want_lp else None, dxsum=gs(prev))
        wr.join()
        out = _handover(dx.view(B, N, D), dx_lp)
        return (out, None, gs.grads([prev])[0], None, None, None) + gs.grads(ps)


# the block backward's weight gradients on a side stream (VITMI_WGRAD_STREAM=0: the current one).
# They depend on nothing the dgrad chain computes after them, so their launches fill the tails
# and ramps of the chain's: C3 backward 22.98-23.02 -> 22.77-22.83 ms (profiles/r06_side/)
_WG_SIDE = os.environ.get("VITMI_WGRAD_STREAM", "1") == "1"
_SIDE_STREAMS: Dict[int, "torch.cuda.Stream"] = {}


class _WgradRunner:
    """Runs weight-gradient launches on a side stream ordered after the current stream's work so
    far (or on the current stream); join() orders the current stream after all of them, so every
    gradient the backward returns is final in stream order.  Their operands are the backward's
    locals and saved tensors, alive until it returns (after join): no cross-stream reuse."""

    def __init__(self):
        self.main = torch.cuda.current_stream()
        self.side = None
        if _WG_SIDE:
            dev = self.main.device.index
            if dev not in _SIDE_STREAMS:
                _SIDE_STREAMS[dev] = torch.cuda.Stream(device=self.main.device)
            self.side = _SIDE_STREAMS[dev]

    def run(self, fn, items):
        if not items:
            return
        if self.side is None:
            fn(items)
            return
        ev = torch.cuda.Event()
        ev.record(self.main)
        self.side.wait_event(ev)
        with torch.cuda.stream(self.side):
            fn(items)

    def join(self):
        if self.side is not None:
            ev = torch.cuda.Event()
            ev.record(self.side)
            self.main.wait_event(ev)


def _each_wgrad(items):
    for dy, x, dw in items:
        ops.linear_wgrad(dy, x, dw)


# ======================================================================= embedding
class ConvEmbed(nn.Module):
    """Conv2D(embed_dim, k=patch, s=patch) patch embedding (models/CvT(Par).py:194-217;
    old_codes/MS_CvT.py:336-369).  ``forward(x[B,C,H,W]) -> [B,D,h,w]`` like MS_CvT."""

    def __init__(self, patch_size: int = 16, in_chans: int = 3, embed_dim: int = 768,
                 norm: bool = False, eps: float = 1e-6, dtype: str = "bf16"):
        super().__init__()
        self.patch_size = patch_size
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.norm = LayerNorm(embed_dim, eps) if norm else None
        self.dtype = dtype

    def forward(self, x: Tensor) -> Tensor:
        _check_cuda(x)
        B, C, S, _ = x.shape
        G = S // self.patch_size
        tok = _EmbedFn.apply(x, self, None, None, *self.parameters())  # [B, 1+np, D] w/o cls
        return tok[:, 1:].transpose(1, 2).reshape(B, -1, G, G)


class _EmbedFn(torch.autograd.Function):
    """im2col -> patch GEMM (+bias) [-> LN] -> cls concat + pos-embed, one token tensor."""

    @staticmethod
    def forward(ctx, img, emb, cls, pos, *params):
        T = ops.torch_dtype(emb.dtype)
        B, C, S, _ = img.shape
        P = emb.patch_size
        G = S // P
        np_ = G * G
        D = emb.proj.weight.shape[0]
        w = _lp(emb, emb.proj.weight, T).reshape(D, -1)
        cls_ = cls.detach().reshape(-1) if cls is not None else None
        pos_ = pos.detach().reshape(-1) if pos is not None else None
        if emb.norm is None and emb.dtype in ("bf16x3", "bf16f8"):
            # the precision knob: patches and weight as split-bf16 pairs (tools/precision_emulate.py:
            # the bf16 patch weight alone costs 1.1e-3 of ViT-B logits error); the backward reads hi
            f8 = emb.dtype == "bf16f8"
            split = ops.split_bf16f8 if f8 else ops.split_bf16x3
            pf = ops.patch_im2col(img.contiguous().float(), P, F32)
            p3, patches = split(pf, 0, hi_copy=True)
            del pf
            w3, _ = split(emb.proj.weight.detach().reshape(D, -1), 1)
            tok = ops.linear_fwd(p3, w3, emb.proj.bias, F32, f8=f8)
            x = ops.tokens_assemble(tok, B, np_, cls_, pos_)
            saved = [patches]
        elif emb.norm is None:
            # the §8(b) entry point: im2col -> patch GEMM (+bias) -> cls concat + pos-embed
            x, patches = ops.patch_embed_fwd(img.contiguous().float(), w, emb.proj.bias, cls_, pos_, P, T)
            saved = [patches]
        else:
            patches = ops.patch_im2col(img.contiguous().float(), P, T)
            conv = ops.linear_fwd(patches, w, emb.proj.bias, F32)
            y, mean, rstd = ops.layernorm_fwd(conv, emb.norm.weight, emb.norm.bias, emb.norm.eps, F32)
            saved = [patches, conv, mean, rstd]
            x = ops.tokens_assemble(y, B, np_, cls_, pos_)
        ctx.save_for_backward(*saved)
        ctx.emb, ctx.cls, ctx.pos, ctx.dims = emb, cls, pos, (B, np_, D)
        ctx.img_shape = (B, C, S, P)
        return x

    @staticmethod
    @_folds
    def backward(ctx, dx):
        emb, cls, pos, (B, np_, D) = ctx.emb, ctx.cls, ctx.pos, ctx.dims
        ps = list(emb.parameters())
        gs = _sink(ctx, 4, ps, getattr(emb, "_arena", None), extra=[(2, cls), (3, pos)])
        saved = ctx.saved_tensors
        patches = saved[0]
        T = patches.dtype
        lpT = None if T == F32 else T
        dx = dx.contiguous()
        dcls, dpos = gs(cls), gs(pos)
        dcls = dcls.view(-1) if dcls is not None else None
        dpos = dpos.view(-1) if dpos is not None else None
        dw = gs(emb.proj.weight)
        dw = dw.view(D, -1) if dw is not None else None
        if emb.norm is not None:
            conv, mean, rstd = saved[1:]
            dy, _ = ops.tokens_assemble_bwd(dx, B, np_, True, None, dcls, dpos)
            dconv, dconv_lp = ops.layernorm_bwd(dy, conv, mean, rstd, emb.norm.weight,
                                                gs(emb.norm.weight), gs(emb.norm.bias), lp_dtype=lpT)
            g = dconv_lp if dconv_lp is not None else dconv
            if dw is not None:
                ops.linear_wgrad(g, patches, dw)
            if gs.wants(emb.proj.bias):
                ops.bias_grad(g, gs(emb.proj.bias))
        else:
            Bi, C, S, P = ctx.img_shape
            ops.patch_embed_bwd(dx, patches, Bi, C, S, P, dw, gs(emb.proj.bias), dcls, dpos)
        return (None, None, gs.grads([cls])[0], gs.grads([pos])[0]) + gs.grads(ps)


# ======================================================================= head + loss
class _HeadFn(torch.autograd.Function):
    """LN(cls) -> Dense(num_classes)  (models/CvT(Par).py:326-329,350).  ``last_fc2_bias``: the
    fc2 bias of the last block, whose gradient (colsum of the head's input gradient) the LN
    backward forms here."""

    @staticmethod
    def forward(ctx, x, model, last_fc2_bias, *params):
        norm, head = model.norm, model.head
        xc = x[:, 0]                                      # strided rows [B, D]
        y, mean, rstd = ops.layernorm_fwd(xc, norm.weight, norm.bias, norm.eps, F32)
        logits = ops.head_fwd(y, head.weight.detach(), head.bias)
        ctx.save_for_backward(x, y, mean, rstd)
        ctx.model, ctx.last_bias = model, last_fc2_bias
        ctx.handover = _is_vitmi_node(x)
        return logits

    @staticmethod
    @_folds
    def backward(ctx, dlogits):
        x, y, mean, rstd = ctx.saved_tensors
        model, last = ctx.model, ctx.last_bias
        norm, head = model.norm, model.head
        ps = list(norm.parameters()) + list(head.parameters())
        gs = _sink(ctx, 3, ps, model._arena, extra=[(2, last)] if last is not None else [])
        dy = ops.head_bwd(dlogits.float(), y, head.weight.detach(), gs(head.weight), gs(head.bias))
        dx = torch.zeros_like(x)
        # the last block's GEMMs take dx in the compute dtype: its zero rows are a fill and the
        # cls rows come from the LN backward (no cast pass over dx)
        T = ops.torch_dtype(model.cfg.dtype)
        lp = (torch.zeros(x.shape[0] * x.shape[1], x.shape[2], dtype=T, device=x.device)
              if T != F32 and ctx.handover else None)
        ops.layernorm_bwd(dy, x[:, 0], mean, rstd, norm.weight, gs(norm.weight), gs(norm.bias),
                          dx=dx[:, 0], dxsum=gs(last), lp_dtype=None if lp is None else T,
                          dx_lp=None if lp is None else lp.view(x.shape[0], x.shape[1], x.shape[2])[:, 0])
        _handover(dx, lp)
        return (dx, None, gs.grads([last])[0]) + gs.grads(ps)


class _LossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, kind):
        loss, dl = ops.loss_fwd_bwd(logits.float(), target, kind)
        ctx.save_for_backward(dl)
        return loss

    @staticmethod
    def backward(ctx, g):
        (dl,) = ctx.saved_tensors
        return dl * g, None, None


# the Functions whose backward takes a handed-over bf16 copy of their output gradient
_HANDOVER_FNS = (_BlockFn, _AttentionFn, _MlpFn)


def cross_entropy(logits: Tensor, target: Tensor) -> Tensor:
    """Mean softmax cross-entropy on the vitmi loss kernel."""
    return _LossFn.apply(logits, target, ops.LOSS_CE)


def mse_loss(logits: Tensor, target: Tensor) -> Tensor:
    """Keras 'mean_squared_error' (models/CvT(Par).py:464-466) on the vitmi loss kernel."""
    t = target.reshape(logits.shape[0], -1)
    return _LossFn.apply(logits, t, ops.LOSS_MSE)


# ======================================================================= parameter arena
class ParamArena:
    """All parameters of a model as views into ONE fp32 buffer (plus one fp32 gradient
    buffer and one bf16 operand shadow with the same offsets), laid out in the order
    the backward finishes them (head first, patch-embed last) so DP buckets become
    ready front to back."""

    ALIGN = 64  # elements: 256 B fp32 / 128 B bf16

    def __init__(self, ordered: List[nn.Parameter], device, want_lp: bool):
        self.params = ordered
        offs, n = [], 0
        for p in ordered:
            offs.append(n)
            n += (p.numel() + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        self.numel = n
        self.offsets = {id(p): o for p, o in zip(ordered, offs)}
        self.flat = torch.zeros(n, dtype=F32, device=device)
        self.grad = torch.zeros(n, dtype=F32, device=device)
        self.flat_lp = torch.empty(n, dtype=torch.bfloat16, device=device) if want_lp else None
        self._lp_version: Optional[int] = None
        self._ids = frozenset(id(p) for p in ordered)
        self._fresh: set = set()   # parameters whose gradient view is zero and not handed out
        with torch.no_grad():
            for p, o in zip(ordered, offs):
                self.flat[o:o + p.numel()].copy_(p.detach().reshape(-1))
                p.data = self.flat[o:o + p.numel()].view(p.shape)
        self._grad_views = [self.grad[o:o + p.numel()].view(p.shape) for p, o in zip(ordered, offs)]

    def owns(self, ps: List[nn.Parameter]) -> bool:
        for p in ps:
            o = self.offsets.get(id(p))
            if o is None or p.data_ptr() != self.flat.data_ptr() + 4 * o:
                return False
        return True

    def view(self, buf: Tensor, p: Tensor) -> Tensor:
        o = self.offsets[id(p)]
        return buf[o:o + p.numel()].view(p.shape)

    def lp(self, p: Tensor) -> Tensor:
        return self.view(self.flat_lp, p)

    def _stamp(self) -> int:
        # version counters only grow: any in-place torch write to the flat buffer or to a
        # parameter (p.data is a view of it but keeps its own counter) raises this sum
        return self.flat._version + sum(p._version for p in self.params)

    def refresh_lp(self) -> None:
        """Re-cast the bf16 shadow unless it is current: no in-place torch write since the
        last cast or since vitmi Adam wrote params and shadow together."""
        if self.flat_lp is None:
            return
        stamp = self._stamp()
        if self._lp_version == stamp:
            return
        ops.cast_bf16(self.flat, self.flat_lp)
        self._lp_version = stamp

    def mark_lp_fresh(self) -> None:
        """The fused optimizer wrote params and shadow through raw pointers (no version bump)."""
        self._lp_version = self._stamp()

    def begin_step(self) -> None:
        """A forward that will be differentiated: when no parameter holds a gradient (the
        set_to_none convention of torch's zero_grad), zero the flat gradient buffer once and
        offer every parameter's view as its backward destination (``take``); AccumulateGrad
        then keeps that view as ``.grad``.  Otherwise (gradients being accumulated across
        backwards) the Functions allocate fresh buffers that autograd adds into ``.grad``."""
        if all(p.grad is None for p in self.params):
            self.grad.zero_()
            self._fresh = set(self._ids)
        else:
            self._fresh = set()

    def take(self, p: Tensor) -> Optional[Tensor]:
        """p's zeroed gradient view, once per ``begin_step``, while ``p.grad`` is None."""
        if id(p) in self._fresh and p.grad is None:
            self._fresh.discard(id(p))
            return self.view(self.grad, p)
        return None

    def bind_grads(self, fill_missing: bool = True) -> None:
        """Make every ``.grad`` the parameter's view of the flat gradient buffer (copying a
        gradient that lives elsewhere): the fused optimizer and the DP buckets read the flat
        buffer.  A missing gradient counts as zero (``fill_missing``) or is left missing.  After a
        backward from ``begin_step`` this only checks pointers."""
        ps, views = self.params, self._grad_views
        if fill_missing and all(p.grad is None for p in ps):
            self.grad.zero_()
            for p, v in zip(ps, views):
                p.grad = v
            return
        for p, v in zip(ps, views):
            g = p.grad
            if g is None:
                if fill_missing:
                    v.zero_()
                    p.grad = v
            elif g.data_ptr() != v.data_ptr():
                v.copy_(g)
                p.grad = v

    def runs(self, select: List[bool]) -> List[tuple]:
        """(start, end) element ranges of the flat buffers covering the selected parameters, one per
        run of consecutive selected parameters (alignment padding included: it holds zeros)."""
        out: List[tuple] = []
        for p, sel in zip(self.params, select):
            if not sel:
                continue
            o = self.offsets[id(p)]
            e = o + (p.numel() + self.ALIGN - 1) // self.ALIGN * self.ALIGN
            if out and out[-1][1] == o:
                out[-1] = (out[-1][0], e)
            else:
                out.append((o, e))
        return out


# ======================================================================= model
class VisionTransformer(nn.Module):
    """One-stage ViT in the reference's vocabulary: ConvEmbed(P, s=P) -> depth x
    ConvTransformerBlock(qkv_method='linear') -> LN(cls) -> Dense(num_classes)
    (create_cvt_model, models/CvT(Par).py:292-354; MS_CvT VisionTransformer :372-488 +
    head :605-623).  ``forward(x) -> logits``."""

    def __init__(self, cfg: ViTConfig):
        super().__init__()
        if not cfg.with_cls_token:
            raise NotImplementedError("vitmi: only the cls-token head is implemented")
        self.cfg = cfg
        D = cfg.embed_dim
        self.patch_embed = ConvEmbed(cfg.patch_size, cfg.in_chans, D, cfg.embed_norm, cfg.ln_eps, cfg.dtype)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, D))
        self.pos_embed = nn.Parameter(torch.zeros(1, cfg.seq_len, D)) if cfg.pos_embed else None
        self.blocks = nn.ModuleList([
            Block(D, cfg.num_heads, cfg.mlp_ratio, cfg.qkv_bias, cfg.ln_eps, cfg.attn_scale, cfg.tie_norms,
                  cfg.dtype) for _ in range(cfg.depth)])
        if cfg.split_qkv is not None:
            for blk in self.blocks:
                blk.split_qkv = cfg.split_qkv
        self.norm = LayerNorm(D, cfg.ln_eps)
        self.head = Linear(D, cfg.num_classes)
        self._arena: Optional[ParamArena] = None
        self.drop_seed: Optional[int] = None   # fixed dropout seed (tests); None = drawn per forward
        self._fc2_bias_fused = True
        self.reset_parameters()

    # -- init: trunc_normal(.02) weights, zero biases, LN (1, 0)  (old_codes/MS_CvT.py:437-454)
    def reset_parameters(self, seed: Optional[int] = None) -> None:
        g = torch.Generator().manual_seed(seed) if seed is not None else None
        with torch.no_grad():
            for name, p in self.named_parameters():
                if "norm" in name:
                    p.fill_(1.0 if name.endswith("weight") else 0.0)
                elif name.endswith("bias"):
                    p.zero_()
                else:
                    t = torch.randn(p.shape, generator=g).clamp_(-2, 2) * 0.02
                    p.copy_(t)

    def named_param_dict(self) -> Dict[str, nn.Parameter]:
        return dict(self.named_parameters())

    def load_param_dict(self, d: Dict[str, Tensor]) -> None:
        mine = self.named_param_dict()
        missing = set(mine) - set(d)
        if missing:
            raise KeyError(f"missing parameters: {sorted(missing)[:5]}")
        with torch.no_grad():
            for k, p in mine.items():
                p.copy_(d[k].reshape(p.shape).to(p.device, p.dtype))

    # -- arena
    def backward_order(self) -> List[nn.Parameter]:
        order: List[nn.Parameter] = []
        order += list(self.head.parameters()) + list(self.norm.parameters())
        for blk in reversed(self.blocks):
            order += list(blk.parameters())
        order += list(self.patch_embed.parameters())
        order += [self.cls_token] + ([self.pos_embed] if self.pos_embed is not None else [])
        assert len(order) == len(list(self.parameters()))
        return order

    def arena(self) -> ParamArena:
        ps = self.backward_order()
        if self._arena is None or not self._arena.owns(ps) or self._arena.flat.device != ps[0].device:
            self._arena = ParamArena(ps, ps[0].device, self.cfg.dtype != "fp32")
            for m in self.modules():
                if m is not self:
                    object.__setattr__(m, "_arena", self._arena)
        return self._arena

    # -- forward
    def forward_features(self, x: Tensor, _head_takes_bias: bool = False) -> Tensor:
        """Token stream after the last block, [B, N, D] fp32.  (``_head_takes_bias``: forward()'s
        head forms the last block's fc2 bias gradient.)"""
        _check_cuda(x)
        arena = self.arena()
        arena.refresh_lp()
        if torch.is_grad_enabled():
            arena.begin_step()
        pe = self.patch_embed
        t = _EmbedFn.apply(x, pe, self.cls_token, self.pos_embed, *pe.parameters())
        # bias-grad fusion: block i's LN1 backward produces colsum(d input) = the fc2 bias grad
        # of block i-1; the head's LN backward does it for the last block.
        drop = _drop_args(self, self.cfg.drop_rate, 0)
        # with dropout the fc2/proj bias grads are column sums of MASKED gradients: no fusion
        self._fc2_bias_fused = drop is None
        L = len(self.blocks)
        for i, blk in enumerate(self.blocks):
            prev_bias = self.blocks[i - 1].mlp.fc2.bias if i > 0 and drop is None else None
            done = drop is None and (i < L - 1 or _head_takes_bias)
            d = None if drop is None else (drop[0], drop[1], 3 * i)
            # block 0's input gradient goes to the patch embedding's backward, which reads fp32
            t = _BlockFn.apply(t, blk, prev_bias, done, d, i > 0, *blk.parameters())
        return t

    def forward(self, x: Tensor) -> Tensor:
        t = self.forward_features(x, _head_takes_bias=True)
        last = self.blocks[-1].mlp.fc2.bias if len(self.blocks) and self._fc2_bias_fused else None
        return _HeadFn.apply(t, self, last, *self.norm.parameters(), *self.head.parameters())


def build_model(cfg: ViTConfig, device="cuda") -> VisionTransformer:
    return VisionTransformer(cfg).to(device)


__all__ = ["LayerNorm", "Linear", "Attention", "Mlp", "Block", "ConvEmbed", "VisionTransformer",
           "cross_entropy", "mse_loss", "build_model", "ParamArena"]

