"""ORACLE — CPU restatement of the reference ViT forward/backward (TEST INFRASTRUCTURE ONLY).

This module is the parity checker for the MI355X path.  It is never imported by
the product package (``transformer-stm_amd/vitmi``); only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it.

It restates, in plain PyTorch fp32 on the CPU, the algorithm of the
reference's transformer stage:

* ``ConvEmbed``           ``models/CvT(Par).py:194-217``   (Conv2D k=P, s=P; the
  LayerNorm the Keras code intends is never built, ``:209``; MS_CvT applies it,
  ``old_codes/MS_CvT.py:358,365-366`` -> ``embed_norm`` knob)
* cls-token prepend       ``models/CvT(Par).py:244-245,264-268``;
  ``old_codes/MS_CvT.py:473-477``
* ``ConvTransformerBlock`` ``models/CvT(Par).py:261-289``: pre-LN block
  ``x += Attn(LN(x)); x += MLP(LN(x))`` (``old_codes/MS_CvT.py:325-333``)
* ``ConvAttention`` with ``Projection(method='linear')`` ``models/CvT(Par).py:144-191``:
  Q/K/V linears (fused here into one [3D, D] weight: a composition of linears is a
  linear), softmax(QK^T * scale) V, out-projection
  (``old_codes/MS_CvT.py:198-211``)
* ``Mlp``                 ``models/CvT(Par).py:253-258``: Dense(4D, exact-erf GELU) -> Dense(D)
* head                    ``models/CvT(Par).py:326-329,350``: LN(cls) -> Dense(num_classes);
  ``old_codes/MS_CvT.py:605-623``
* loss                    ``models/CvT(Par).py:464-466`` (MSE for 1 output); softmax-CE
  for >= 2 classes (BASELINE configs)

Knobs follow ``vitmi.config.ViTConfig`` (attn_scale, ln_eps, qkv_bias,
embed_norm, pos_embed, tie_norms); any object with those attributes works.

Parity pinning: ``tests/golden/`` holds vectors generated in the survey
container from (i) the reference's own PyTorch module ``old_codes/MS_CvT.py``
(imported with stubs for its absent ``timm``/``registry``/``torch._six``
imports) and (ii) ``transformers.ViTForImageClassification`` built offline
from a config; ``tests/test_oracle_golden.py`` checks this restatement against
both.  The TF/Keras boundary itself is unpinned (TensorFlow is not installed).
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

Tensor = torch.Tensor


def param_shapes(cfg) -> Dict[str, tuple]:
    """Canonical parameter names/shapes shared with ``vitmi.modules``."""
    D, C, P = cfg.embed_dim, cfg.in_chans, cfg.patch_size
    F_, L = int(cfg.embed_dim * cfg.mlp_ratio), cfg.depth
    N = (cfg.img_size // P) ** 2 + (1 if cfg.with_cls_token else 0)
    s = {"patch_embed.proj.weight": (D, C, P, P), "patch_embed.proj.bias": (D,)}
    if cfg.embed_norm:
        s["patch_embed.norm.weight"] = (D,)
        s["patch_embed.norm.bias"] = (D,)
    if cfg.with_cls_token:
        s["cls_token"] = (1, 1, D)
    if cfg.pos_embed:
        s["pos_embed"] = (1, N, D)
    for i in range(L):
        p = f"blocks.{i}."
        s[p + "norm1.weight"] = (D,)
        s[p + "norm1.bias"] = (D,)
        s[p + "attn.qkv.weight"] = (3 * D, D)
        if cfg.qkv_bias:
            s[p + "attn.qkv.bias"] = (3 * D,)
        s[p + "attn.proj.weight"] = (D, D)
        s[p + "attn.proj.bias"] = (D,)
        if not cfg.tie_norms:
            s[p + "norm2.weight"] = (D,)
            s[p + "norm2.bias"] = (D,)
        s[p + "mlp.fc1.weight"] = (F_, D)
        s[p + "mlp.fc1.bias"] = (F_,)
        s[p + "mlp.fc2.weight"] = (D, F_)
        s[p + "mlp.fc2.bias"] = (D,)
    s["norm.weight"] = (D,)
    s["norm.bias"] = (D,)
    s["head.weight"] = (cfg.num_classes, D)
    s["head.bias"] = (cfg.num_classes,)
    return s


def init_params(cfg, seed: int = 0, randomize_all: bool = True) -> Dict[str, Tensor]:
    """Deterministic parameters.

    ``trunc_normal(std=.02)`` for weights / cls / pos (``old_codes/MS_CvT.py:437-454``).
    With ``randomize_all`` (parity runs) LN gamma/beta and biases are random too, so
    every term of the backward is exercised; otherwise biases 0, gamma 1, beta 0.
    """
    g = torch.Generator().manual_seed(seed)
    out = {}
    for name, shape in param_shapes(cfg).items():
        leaf = name.rsplit(".", 1)[-1]
        is_norm = ".norm" in name or name.startswith("norm.") or "norm1" in name or "norm2" in name
        if is_norm:
            if randomize_all:
                t = (1.0 + 0.1 * torch.randn(shape, generator=g)) if leaf == "weight" else 0.1 * torch.randn(shape, generator=g)
            else:
                t = torch.ones(shape) if leaf == "weight" else torch.zeros(shape)
        elif leaf == "bias":
            t = 0.02 * torch.randn(shape, generator=g) if randomize_all else torch.zeros(shape)
        else:
            t = torch.randn(shape, generator=g).clamp_(-2.0, 2.0) * 0.02
        out[name] = t.float().contiguous()
    return out


# ---------------------------------------------------------------- dropout
# layers.Dropout at models/CvT(Par).py:189 (after the out-projection), :255 (after the GELU)
# and :257 (after fc2); Keras' rate 0.1, active in training only.  Keras draws its mask from
# TF's stateful RNG (unreproducible here, and TF is absent); the build defines the mask as a
# counter hash of (seed, site, row, col) -- restated here bit for bit from the C ABI's
# vitmi_dropout_hash (include/vitmi.h) -- so the oracle and the device path drop the SAME
# elements.  Sites: block i -> 3i (proj), 3i+1 (GELU), 3i+2 (fc2); rows = b*N + token.
_M32 = np.uint64(0xFFFFFFFF)


def _fmix32(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x85EBCA6B)) & _M32
    x ^= x >> np.uint64(13)
    x = (x * np.uint64(0xC2B2AE35)) & _M32
    x ^= x >> np.uint64(16)
    return x


def dropout_hash(seed: int, site: int, rows: np.ndarray, cols: np.ndarray) -> np.ndarray:
    """uint32 hash of every (row, col) pair of the broadcast of rows[:, None], cols[None, :]."""
    rows = np.asarray(rows, dtype=np.uint64)
    cols = np.asarray(cols, dtype=np.uint64)
    base = np.uint64(seed & 0xFFFFFFFF) ^ ((np.uint64(site) * np.uint64(0x9E3779B1)) & _M32)
    rk = _fmix32(base ^ _fmix32((rows + np.uint64(0x7F4A7C15)) & _M32))
    return _fmix32(rk[:, None] ^ ((cols[None, :] * np.uint64(0x85EBCA77)) & _M32))


def dropout_params(p: float) -> Tuple[int, float]:
    """(thresh, scale): keep iff hash >= thresh = round(p * 2^32); kept values * 1/(1-p)."""
    return min(int(round(p * 2.0 ** 32)), 0xFFFFFFFF), 1.0 / (1.0 - p)


def dropout(x: Tensor, seed: int, site: int, p: float) -> Tensor:
    """x [..., C] with rows = the flattened leading dims (token-major, like the device GEMMs)."""
    shape = x.shape
    x2 = x.reshape(-1, shape[-1])
    thresh, scale = dropout_params(p)
    keep = dropout_hash(seed, site, np.arange(x2.shape[0]), np.arange(x2.shape[1])) >= thresh
    return (x2 * torch.from_numpy(keep.astype(np.float32)) * scale).reshape(shape)


def layer_norm(x: Tensor, w: Tensor, b: Tensor, eps: float) -> Tensor:
    # models/CvT(Par).py:248 (LayerNormalization over the channel axis)
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


def attention(x: Tensor, p: Dict[str, Tensor], pre: str, cfg, drop=None) -> Tensor:
    """ConvAttention.call with identity projections (models/CvT(Par).py:144-191)."""
    B, N, D = x.shape
    H = cfg.num_heads
    dh = D // H
    qkv = F.linear(x, p[pre + "attn.qkv.weight"], p.get(pre + "attn.qkv.bias"))
    q, k, v = qkv.split(D, dim=-1)
    q = q.reshape(B, N, H, dh).transpose(1, 2)
    k = k.reshape(B, N, H, dh).transpose(1, 2)
    v = v.reshape(B, N, H, dh).transpose(1, 2)
    scale = cfg.head_dim ** -0.5 if cfg.attn_scale == "head" else cfg.embed_dim ** -0.5
    s = torch.matmul(q, k.transpose(-1, -2)) * scale           # old_codes/MS_CvT.py:202
    a = torch.softmax(s, dim=-1)                                # :203
    o = torch.matmul(a, v).transpose(1, 2).reshape(B, N, D)     # :206-207
    out = F.linear(o, p[pre + "attn.proj.weight"], p[pre + "attn.proj.bias"])  # :209
    if drop is not None:                                        # proj_dropout, CvT(Par).py:189
        out = dropout(out, drop[0], drop[1], drop[2])
    return out


def mlp(x: Tensor, p: Dict[str, Tensor], pre: str, drop=None) -> Tensor:
    """Mlp: Dense(4D, gelu) -> Dropout -> Dense(D) -> Dropout (models/CvT(Par).py:253-258).
    ``drop`` = (seed, first site, rate) or None (inference / rate 0)."""
    h = F.linear(x, p[pre + "mlp.fc1.weight"], p[pre + "mlp.fc1.bias"])
    h = F.gelu(h)  # exact erf GELU (tf.nn.gelu default approximate=False)
    if drop is not None:
        h = dropout(h, drop[0], drop[1], drop[2])
    y = F.linear(h, p[pre + "mlp.fc2.weight"], p[pre + "mlp.fc2.bias"])
    if drop is not None:
        y = dropout(y, drop[0], drop[1] + 1, drop[2])
    return y


def block(x: Tensor, p: Dict[str, Tensor], i: int, cfg, drop_seed: Optional[int] = None) -> Tensor:
    """ConvTransformerBlock.call (models/CvT(Par).py:261-289).  ``drop_seed``: training-mode
    dropout at ``cfg.drop_rate`` (sites 3i, 3i+1, 3i+2)."""
    pre = f"blocks.{i}."
    n2 = "norm1" if cfg.tie_norms else "norm2"
    rate = getattr(cfg, "drop_rate", 0.0)
    on = drop_seed is not None and rate > 0
    da = (drop_seed, 3 * i, rate) if on else None
    dm = (drop_seed, 3 * i + 1, rate) if on else None
    x = x + attention(layer_norm(x, p[pre + "norm1.weight"], p[pre + "norm1.bias"], cfg.ln_eps), p, pre, cfg, da)
    x = x + mlp(layer_norm(x, p[pre + n2 + ".weight"], p[pre + n2 + ".bias"], cfg.ln_eps), p, pre, dm)
    return x


def embed(img: Tensor, p: Dict[str, Tensor], cfg) -> Tensor:
    """ConvEmbed + cls concat + (optional) learned position embedding."""
    x = F.conv2d(img, p["patch_embed.proj.weight"], p["patch_embed.proj.bias"],
                 stride=cfg.patch_size)                         # models/CvT(Par).py:203-212
    B, D = x.shape[0], x.shape[1]
    x = x.flatten(2).transpose(1, 2)                            # b c h w -> b (h w) c
    if cfg.embed_norm:
        x = layer_norm(x, p["patch_embed.norm.weight"], p["patch_embed.norm.bias"], cfg.ln_eps)
    if cfg.with_cls_token:
        x = torch.cat([p["cls_token"].expand(B, 1, D), x], dim=1)
    if cfg.pos_embed:
        x = x + p["pos_embed"]
    return x


def forward_features(img: Tensor, p: Dict[str, Tensor], cfg, drop_seed: Optional[int] = None) -> Tensor:
    x = embed(img, p, cfg)
    for i in range(cfg.depth):
        x = block(x, p, i, cfg, drop_seed)
    return x


def forward(img: Tensor, p: Dict[str, Tensor], cfg, drop_seed: Optional[int] = None) -> Tensor:
    """Logits [B, num_classes] (head: models/CvT(Par).py:326-329,350)."""
    x = forward_features(img, p, cfg, drop_seed)
    cls = x[:, 0] if cfg.with_cls_token else x.mean(dim=1)
    cls = layer_norm(cls, p["norm.weight"], p["norm.bias"], cfg.ln_eps)
    return F.linear(cls, p["head.weight"], p["head.bias"])


def loss_fn(logits: Tensor, target: Tensor, num_classes: int) -> Tensor:
    """MSE for the reference's 1-output regressor (models/CvT(Par).py:464-466), CE otherwise."""
    if num_classes == 1:
        return F.mse_loss(logits.squeeze(-1), target.float())
    return F.cross_entropy(logits, target.long())


def forward_backward(img: Tensor, target: Tensor, p: Dict[str, Tensor], cfg, drop_seed: Optional[int] = None):
    """One fwd+bwd step on the CPU: returns (logits, loss, {name: grad})."""
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in p.items()}
    logits = forward(img, leaves, cfg, drop_seed)
    loss = loss_fn(logits, target, cfg.num_classes)
    loss.backward()
    grads = {k: v.grad.detach() for k, v in leaves.items()}
    return logits.detach(), loss.detach(), grads


def per_image_grad_scale(img: Tensor, target: Tensor, p: Dict[str, Tensor], cfg) -> Dict[str, float]:
    """{name: sum_i ||g_i||}: the norms of each image's contribution g_i to the batch-mean gradient
    g = sum_i g_i, summed.  kappa = sum_i ||g_i|| / ||g|| measures how much the contributions cancel;
    a low-precision backward rounds each contribution, so its error scales with this sum, not with
    ||g|| (tests/test_gpu_model.py uses it as the denominator of the conditioned error)."""
    B = img.shape[0]
    out: Dict[str, float] = {}
    for i in range(B):
        _, _, g = forward_backward(img[i:i + 1], target[i:i + 1], p, cfg)
        for k, v in g.items():
            out[k] = out.get(k, 0.0) + v.double().norm().item() / B
    return out


def synthetic_batch(cfg, batch: int, seed: int = 1234):
    """Images in [0,1) like the reference's /255 normalisation (models/CvT(Par).py:423)."""
    g = torch.Generator().manual_seed(seed)
    img = torch.rand(batch, cfg.in_chans, cfg.img_size, cfg.img_size, generator=g)
    if cfg.num_classes == 1:
        tgt = torch.randn(batch, generator=g)
    else:
        tgt = torch.randint(0, cfg.num_classes, (batch,), generator=g)
    return img, tgt


def rel_err(a: Tensor, b: Tensor) -> float:
    a = a.double()
    b = b.double()
    den = b.norm().item()
    return (a - b).norm().item() / (den if den > 0 else 1.0)


__all__ = [
    "param_shapes", "init_params", "forward", "forward_features", "forward_backward",
    "loss_fn", "synthetic_batch", "rel_err", "per_image_grad_scale", "layer_norm", "attention", "mlp", "block", "embed",
    "dropout", "dropout_hash", "dropout_params",
]

