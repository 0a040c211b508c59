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

from typing import Dict

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


def layer_norm(x: Tensor, w: Tensor, b: Tensor, eps: float) -> Tensor:
    # models/CvT(Par).py:248 (LayerNormalization over the channel axis)
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


def attention(x: Tensor, p: Dict[str, Tensor], pre: str, cfg) -> Tensor:
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
    return F.linear(o, p[pre + "attn.proj.weight"], p[pre + "attn.proj.bias"])  # :209


def mlp(x: Tensor, p: Dict[str, Tensor], pre: str) -> Tensor:
    """Mlp: Dense(4D, gelu) -> Dense(D) (models/CvT(Par).py:253-258)."""
    h = F.linear(x, p[pre + "mlp.fc1.weight"], p[pre + "mlp.fc1.bias"])
    h = F.gelu(h)  # exact erf GELU (tf.nn.gelu default approximate=False)
    return F.linear(h, p[pre + "mlp.fc2.weight"], p[pre + "mlp.fc2.bias"])


def block(x: Tensor, p: Dict[str, Tensor], i: int, cfg) -> Tensor:
    """ConvTransformerBlock.call (models/CvT(Par).py:261-289)."""
    pre = f"blocks.{i}."
    n2 = "norm1" if cfg.tie_norms else "norm2"
    x = x + attention(layer_norm(x, p[pre + "norm1.weight"], p[pre + "norm1.bias"], cfg.ln_eps), p, pre, cfg)
    x = x + mlp(layer_norm(x, p[pre + n2 + ".weight"], p[pre + n2 + ".bias"], cfg.ln_eps), p, pre)
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


def forward_features(img: Tensor, p: Dict[str, Tensor], cfg) -> Tensor:
    x = embed(img, p, cfg)
    for i in range(cfg.depth):
        x = block(x, p, i, cfg)
    return x


def forward(img: Tensor, p: Dict[str, Tensor], cfg) -> Tensor:
    """Logits [B, num_classes] (head: models/CvT(Par).py:326-329,350)."""
    x = forward_features(img, p, cfg)
    cls = x[:, 0] if cfg.with_cls_token else x.mean(dim=1)
    cls = layer_norm(cls, p["norm.weight"], p["norm.bias"], cfg.ln_eps)
    return F.linear(cls, p["head.weight"], p["head.bias"])


def loss_fn(logits: Tensor, target: Tensor, num_classes: int) -> Tensor:
    """MSE for the reference's 1-output regressor (models/CvT(Par).py:464-466), CE otherwise."""
    if num_classes == 1:
        return F.mse_loss(logits.squeeze(-1), target.float())
    return F.cross_entropy(logits, target.long())


def forward_backward(img: Tensor, target: Tensor, p: Dict[str, Tensor], cfg):
    """One fwd+bwd step on the CPU: returns (logits, loss, {name: grad})."""
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in p.items()}
    logits = forward(img, leaves, cfg)
    loss = loss_fn(logits, target, cfg.num_classes)
    loss.backward()
    grads = {k: v.grad.detach() for k, v in leaves.items()}
    return logits.detach(), loss.detach(), grads


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
    "loss_fn", "synthetic_batch", "rel_err", "layer_norm", "attention", "mlp", "block", "embed",
]

