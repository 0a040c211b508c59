"""ORACLE — CPU restatement of the reference's CvT stages (TEST INFRASTRUCTURE ONLY).

Only ``tests/`` use this module; the product package never imports it.

SURVEY §8f row 1: the convolutional model the reference actually trains on its SLS images,
``create_cvt_model`` (``models/CvT(Par).py:292-354``) with the stage spec ``:66-72``:

=======  ==========================================  =============================
stage    ConvEmbed (Conv2D 'same', ``:194-217``)      ConvTransformerBlock (``:231-289``)
=======  ==========================================  =============================
1        D=64,  k7 s4                                 1 head,  dw_bn q/k/v, no cls
2        D=128, k3 s2                                 2 heads, dw_bn, no cls
3        D=256, k3 s2                                 4 heads, dw_bn, cls token
=======  ==========================================  =============================

* ConvEmbed: ``layers.Conv2D(D, k, s, padding='same')`` (TF asymmetric 'same' padding); the
  LayerNorm it means to apply is never built (``norm_layer == "LayerNormalization"`` compares
  a class to a string, ``:209``) -> ``embed_norm`` knob, True for MS_CvT (``old_codes/MS_CvT.py:358``).
* ``Projection('dw_bn')`` (``:83-112``): DepthwiseConv2D(3, stride 1, 'same', no bias) +
  BatchNormalization (training: batch statistics; Keras eps 1e-3), applied to the spatial
  tokens of q, k and v; the cls token bypasses it (``:146-150,164-176``).
* ``ConvAttention.call`` (``:144-191``): q/k/v Dense(D) then MultiHeadAttention(q, v, k) whose
  own query/key/value EinsumDense projections compose with them into one linear each (the
  build holds the composition ``proj_{q,k,v}``), softmax(QK^T / sqrt(D/H)) V, output Dense
  composed with ``self.proj`` into ``proj``.  ``keras_dense``: both factors of every pair as
  parameters (``proj_c`` then ``mha_c``; ``mha_o`` then ``proj``), applied one after the other.
* block: ``x += Attn(LN1(x)); x += MLP(LN1(x))`` with the SAME norm1 used twice (``:248,272,278``).
* ``Projection('avg')``: AveragePooling2D(3, 1, 'same') for k and v, q stays linear
  (``:95-96,107-108,130-132``); ``'linear'``: identity (``qkv_method`` per stage).
* head: LN(cls) (eps 1e-6, ``:328``) [ ++ the process-parameter MLP Dense(256, relu) x 2,
  ``:343-347``, when ``proc_dim`` > 0, SURVEY §8f row 2 ] -> Dense(num_classes) (``:350``).

Knobs (``CvTConfig``) cover MS_CvT's semantics too (``old_codes/MS_CvT.py``: symmetric conv
padding, embed LayerNorm, attention scale 1/sqrt(D) ``:100``, no q/k/v bias ``:82``, BN eps 1e-5,
separate norm1/norm2), which is how ``tests/golden/mscvt_cvt_dwbn.npz`` -- generated from the
reference's own module -- pins this restatement.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor


@dataclass
class CvTStage:
    embed_dim: int
    patch_size: int
    stride: int
    num_heads: int
    with_cls_token: bool = False
    depth: int = 1
    padding: Optional[int] = None    # None: TF 'same'; an int: symmetric (MS_CvT PATCH_PADDING)
    qkv_method: str = "dw_bn"        # 'dw_bn' | 'avg' (q stays 'linear') | 'linear'  (:25,83-112,130-132)


def keras_spec() -> List[CvTStage]:
    """models/CvT(Par).py:66-72 (cls_token_switch = True, :28)."""
    return [CvTStage(64, 7, 4, 1), CvTStage(128, 3, 2, 2), CvTStage(256, 3, 2, 4, with_cls_token=True)]


@dataclass
class CvTConfig:
    img_size: int = 128               # SLS images resized to 128x128 grayscale (:413-423)
    in_chans: int = 1
    num_classes: int = 1              # the reference regresses one value (MSE, :464-466)
    stages: List[CvTStage] = field(default_factory=keras_spec)
    mlp_ratio: float = 4.0
    attn_scale: str = "head"          # 'head' 1/sqrt(D/H) Keras; 'dim' 1/sqrt(D) MS_CvT
    ln_eps: float = 1e-6
    bn_eps: float = 1e-3              # Keras BatchNormalization default; torch 1e-5
    bn_momentum: float = 0.99         # Keras convention (running <- m running + (1-m) batch)
    qkv_bias: bool = True
    tie_norms: bool = True
    embed_norm: bool = False
    avg_count_pad: bool = False       # 'avg' divisor: False = TF 'same' in-bounds count; True = torch's 9
    proc_dim: int = 0                 # process parameters (5 in the reference, :392); 0 = image only
    proc_hidden: int = 256            # Proc_Dense_1/2 width (:343-344)
    drop_rate: float = 0.0            # Dropout after proj (:141,189) and both MLP Dense (:255,257)
    dtype: str = "bf16"
    keras_dense: bool = False         # the Dense pairs as separate factors (mha_{q,k,v,o}; see block)

    def replace(self, **kw) -> "CvTConfig":
        return dataclasses.replace(self, **kw)


def conv_geometry(H: int, k: int, s: int, padding: Optional[int]) -> Tuple[int, int, int]:
    """(Ho, pad_before, pad_after): TF 'same' when padding is None, else symmetric."""
    if padding is None:
        Ho = -(-H // s)
        tot = max((Ho - 1) * s + k - H, 0)
        return Ho, tot // 2, tot - tot // 2
    Ho = (H + 2 * padding - k) // s + 1
    return Ho, padding, padding


def param_shapes(cfg: CvTConfig) -> Dict[str, tuple]:
    s = {}
    cin = cfg.in_chans
    for i, st in enumerate(cfg.stages):
        D, k = st.embed_dim, st.patch_size
        p = f"stage{i}."
        s[p + "embed.weight"] = (D, cin, k, k)        # torch conv layout
        s[p + "embed.bias"] = (D,)
        if cfg.embed_norm:
            s[p + "embed.norm.weight"] = (D,)
            s[p + "embed.norm.bias"] = (D,)
        if st.with_cls_token:
            s[p + "cls_token"] = (1, 1, D)
        for j in range(st.depth):
            b = f"{p}blocks.{j}."
            s[b + "norm1.weight"] = (D,)
            s[b + "norm1.bias"] = (D,)
            for c in "qkv":
                if st.qkv_method == "dw_bn":
                    s[b + f"attn.conv_proj_{c}.weight"] = (D, 1, 3, 3)
                    s[b + f"attn.conv_proj_{c}.bn.weight"] = (D,)
                    s[b + f"attn.conv_proj_{c}.bn.bias"] = (D,)
                s[b + f"attn.proj_{c}.weight"] = (D, D)
                if cfg.qkv_bias:
                    s[b + f"attn.proj_{c}.bias"] = (D,)
            if cfg.keras_dense:   # MultiHeadAttention's query/key/value/output EinsumDense (use_bias)
                for c in "qkvo":
                    s[b + f"attn.mha_{c}.weight"] = (D, D)
                    s[b + f"attn.mha_{c}.bias"] = (D,)
            s[b + "attn.proj.weight"] = (D, D)
            s[b + "attn.proj.bias"] = (D,)
            if not cfg.tie_norms:
                s[b + "norm2.weight"] = (D,)
                s[b + "norm2.bias"] = (D,)
            Fh = int(D * cfg.mlp_ratio)
            s[b + "mlp.fc1.weight"] = (Fh, D)
            s[b + "mlp.fc1.bias"] = (Fh,)
            s[b + "mlp.fc2.weight"] = (D, Fh)
            s[b + "mlp.fc2.bias"] = (D,)
        cin = D
    D = cfg.stages[-1].embed_dim
    s["norm.weight"] = (D,)
    s["norm.bias"] = (D,)
    if cfg.proc_dim:
        Hp = cfg.proc_hidden
        s["proc.fc1.weight"] = (Hp, cfg.proc_dim)
        s["proc.fc1.bias"] = (Hp,)
        s["proc.fc2.weight"] = (Hp, Hp)
        s["proc.fc2.bias"] = (Hp,)
        D += Hp
    s["head.weight"] = (cfg.num_classes, D)
    s["head.bias"] = (cfg.num_classes,)
    return s


def qkv_methods(st: CvTStage) -> Tuple[str, str, str]:
    """Per-projection methods: 'avg' keeps q linear (models/CvT(Par).py:130-132)."""
    m = st.qkv_method
    if m not in ("dw_bn", "avg", "linear"):
        raise ValueError(f"unknown qkv_method {m}")
    return ("linear" if m == "avg" else m, m, m)


def init_params(cfg: CvTConfig, seed: int = 0) -> Dict[str, Tensor]:
    """Random parameters for parity runs (every gamma/beta/bias random)."""
    g = torch.Generator().manual_seed(seed)
    out = {}
    for name, shape in param_shapes(cfg).items():
        leaf = name.rsplit(".", 1)[-1]
        parent = name.split(".")[-2]
        if parent in ("norm1", "norm2", "norm", "bn"):
            t = (1.0 + 0.1 * torch.randn(shape, generator=g)) if leaf == "weight" else 0.1 * torch.randn(shape, generator=g)
        elif leaf == "bias":
            t = 0.02 * torch.randn(shape, generator=g)
        elif "conv_proj" in name:
            t = 0.2 * torch.randn(shape, generator=g)
        elif leaf == "cls_token":
            t = 0.02 * torch.randn(shape, generator=g)
        else:
            fan_in = shape[1] * (shape[2] * shape[3] if len(shape) == 4 else 1)
            t = torch.randn(shape, generator=g) * (1.0 / fan_in) ** 0.5
        out[name] = t.float().contiguous()
    return out


def conv_embed(x: Tensor, w: Tensor, b: Tensor, st: CvTStage) -> Tensor:
    """layers.Conv2D(D, k, s, padding='same') (models/CvT(Par).py:203-212). x NCHW -> NCHW."""
    k, s = st.patch_size, st.stride
    _, pt, pb = conv_geometry(x.shape[2], k, s, st.padding)
    _, pl, pr = conv_geometry(x.shape[3], k, s, st.padding)
    return F.conv2d(F.pad(x, (pl, pr, pt, pb)), w, b, stride=s)


def dw_bn(x: Tensor, w: Tensor, gamma: Tensor, beta: Tensor, eps: float) -> Tensor:
    """Projection('dw_bn') (models/CvT(Par).py:92-94,104-106): x NCHW, training-mode BN."""
    z = F.conv2d(x, w, None, stride=1, padding=1, groups=x.shape[1])
    return F.batch_norm(z, None, None, gamma, beta, training=True, eps=eps)


def block(x: Tensor, hw: Tuple[int, int], p: Dict[str, Tensor], pre: str, cfg: CvTConfig, st: CvTStage,
          drop=None) -> Tensor:
    """ConvTransformerBlock.call (models/CvT(Par).py:261-289) on tokens [B, N, D].  ``drop`` =
    (seed, rate, site0): training-mode Dropout with the build's counter-hash masks
    (oracle/vit_ref.py ``dropout``) at sites site0 (proj), +1 (GELU output), +2 (fc2)."""
    from oracle.vit_ref import dropout as _dropout
    dp = (lambda t, j: t) if drop is None else (lambda t, j: _dropout(t, drop[0], drop[2] + j, drop[1]))
    B, N, D = x.shape
    H, W = hw
    Hh = st.num_heads
    dh = D // Hh
    n1w, n1b = p[pre + "norm1.weight"], p[pre + "norm1.bias"]
    n2w, n2b = (n1w, n1b) if cfg.tie_norms else (p[pre + "norm2.weight"], p[pre + "norm2.bias"])
    h = F.layer_norm(x, (D,), n1w, n1b, cfg.ln_eps)
    cls, sp = (h[:, :1], h[:, 1:]) if st.with_cls_token else (None, h)
    img = sp.transpose(1, 2).reshape(B, D, H, W)
    proj = []
    for c, m in zip("qkv", qkv_methods(st)):
        a = pre + f"attn.conv_proj_{c}."
        if m == "dw_bn":
            t = dw_bn(img, p[a + "weight"], p[a + "bn.weight"], p[a + "bn.bias"], cfg.bn_eps)
        elif m == "avg":   # AveragePooling2D(3, 1, 'same') (:95-96,107-108)
            t = F.avg_pool2d(img, 3, 1, 1, count_include_pad=cfg.avg_count_pad)
        else:
            t = img
        t = t.flatten(2).transpose(1, 2)
        if cls is not None:
            t = torch.cat([cls, t], dim=1)
        t = F.linear(t, p[pre + f"attn.proj_{c}.weight"], p.get(pre + f"attn.proj_{c}.bias"))
        if cfg.keras_dense:   # then MHA's own query/key/value projection (:185; Keras MHA internals)
            t = F.linear(t, p[pre + f"attn.mha_{c}.weight"], p[pre + f"attn.mha_{c}.bias"])
        proj.append(t)
    q, k, v = (t.reshape(B, N, Hh, dh).transpose(1, 2) for t in proj)
    scale = dh ** -0.5 if cfg.attn_scale == "head" else D ** -0.5
    a = torch.softmax(torch.matmul(q, k.transpose(-1, -2)) * scale, dim=-1)
    o = torch.matmul(a, v).transpose(1, 2).reshape(B, N, D)
    if cfg.keras_dense:       # MHA's output projection, then self.proj (:188)
        o = F.linear(o, p[pre + "attn.mha_o.weight"], p[pre + "attn.mha_o.bias"])
    x = x + dp(F.linear(o, p[pre + "attn.proj.weight"], p[pre + "attn.proj.bias"]), 0)
    y = F.layer_norm(x, (D,), n2w, n2b, cfg.ln_eps)
    y = dp(F.gelu(F.linear(y, p[pre + "mlp.fc1.weight"], p[pre + "mlp.fc1.bias"])), 1)
    y = dp(F.linear(y, p[pre + "mlp.fc2.weight"], p[pre + "mlp.fc2.bias"]), 2)
    return x + y


def forward_features(img: Tensor, p: Dict[str, Tensor], cfg: CvTConfig, capture: Optional[list] = None,
                     drop_seed: Optional[int] = None) -> Tensor:
    """Stages 1..S; returns LN(final cls token) [B, D] (the token mean without cls, :337-340)."""
    x = img
    tok = None
    t = None
    bi = 0
    for i, st in enumerate(cfg.stages):
        pre = f"stage{i}."
        x = conv_embed(x, p[pre + "embed.weight"], p[pre + "embed.bias"], st)
        B, D, H, W = x.shape
        t = x.flatten(2).transpose(1, 2)
        if cfg.embed_norm:
            t = F.layer_norm(t, (D,), p[pre + "embed.norm.weight"], p[pre + "embed.norm.bias"], cfg.ln_eps)
        if st.with_cls_token:
            t = torch.cat([p[pre + "cls_token"].expand(B, 1, D), t], dim=1)
        for j in range(st.depth):
            drop = None if (drop_seed is None or cfg.drop_rate <= 0) else (drop_seed, cfg.drop_rate, 3 * bi)
            t = block(t, (H, W), p, f"{pre}blocks.{j}.", cfg, st, drop)
            bi += 1
        if capture is not None:
            capture.append((t, H, st.with_cls_token))
        if st.with_cls_token:
            tok, t = t[:, 0], t[:, 1:]
        x = t.transpose(1, 2).reshape(B, D, H, W)
    if tok is None:
        return F.layer_norm(t, (t.shape[-1],), p["norm.weight"], p["norm.bias"], cfg.ln_eps).mean(dim=1)
    return F.layer_norm(tok, (tok.shape[-1],), p["norm.weight"], p["norm.bias"], cfg.ln_eps)


def proc_features(proc: Tensor, p: Dict[str, Tensor]) -> Tensor:
    """Proc_Dense_1/2: Dense(256, relu) x 2 on the standardised process parameters (:343-344)."""
    h = F.relu(F.linear(proc, p["proc.fc1.weight"], p["proc.fc1.bias"]))
    return F.relu(F.linear(h, p["proc.fc2.weight"], p["proc.fc2.bias"]))


def forward(img: Tensor, p: Dict[str, Tensor], cfg: CvTConfig, proc: Optional[Tensor] = None,
            capture: Optional[list] = None, drop_seed: Optional[int] = None) -> Tensor:
    """Image features (+ concatenated process features, :347) -> Final_Dense (:350)."""
    f = forward_features(img, p, cfg, capture, drop_seed)
    if cfg.proc_dim:
        f = torch.cat([f, proc_features(proc, p)], dim=1)
    return F.linear(f, p["head.weight"], p["head.bias"])


def loss_fn(logits: Tensor, target: Tensor, num_classes: int) -> Tensor:
    if num_classes == 1:
        return F.mse_loss(logits.squeeze(-1), target.float())
    return F.cross_entropy(logits, target.long())


def forward_backward(img: Tensor, target: Tensor, p: Dict[str, Tensor], cfg: CvTConfig,
                     proc: Optional[Tensor] = None, drop_seed: Optional[int] = None):
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in p.items()}
    logits = forward(img, leaves, cfg, proc, drop_seed=drop_seed)
    loss = loss_fn(logits, target, cfg.num_classes)
    loss.backward()
    return logits.detach(), loss.detach(), {k: v.grad.detach() for k, v in leaves.items()}


def synthetic_proc(cfg: CvTConfig, batch: int, seed: int = 4321) -> Tensor:
    """Standardised process parameters (zero mean / unit variance like StandardScaler, :402-403)."""
    g = torch.Generator().manual_seed(seed)
    return torch.randn(batch, cfg.proc_dim, generator=g)


def synthetic_batch(cfg: CvTConfig, batch: int, seed: int = 1234):
    g = torch.Generator().manual_seed(seed)
    img = torch.rand(batch, cfg.in_chans, cfg.img_size, cfg.img_size, generator=g)
    if cfg.num_classes == 1:
        tgt = torch.randn(batch, generator=g)
    else:
        tgt = torch.randint(0, cfg.num_classes, (batch,), generator=g)
    return img, tgt


def gradcam(img: Tensor, p: Dict[str, Tensor], cfg: CvTConfig, proc: Optional[Tensor] = None, stage: int = -1,
            batch_size: int = 1) -> Tensor:
    """make_gradcam_heatmap (tools/grad_cam_CvT.py:422-481) per batch of ``batch_size``: grads of
    predictions[:, 0] wrt the stage's spatial output A [b, H, W, C]; pooled = mean over (0, 1, 2);
    heatmap = sum_c pooled[c] A[0, :, :, c]; max(heatmap, 0) / max(heatmap).  (BatchNorm in
    training mode here: use it with 'avg' / 'linear' projections for an inference-mode match.)"""
    p = {k: v.detach().clone().requires_grad_(True) for k, v in p.items()}
    out = []
    for lo in range(0, img.shape[0], batch_size):
        cap = []
        pr = None if proc is None else proc[lo:lo + batch_size]
        logits = forward(img[lo:lo + batch_size], p, cfg, pr, capture=cap)
        t, H, has_cls = cap[stage]
        g = torch.autograd.grad(logits[:, 0].sum(), t)[0]
        A, G = (t[:, 1:], g[:, 1:]) if has_cls else (t, g)
        n, _, C = A.shape
        A, G = A.reshape(n, H, H, C), G.reshape(n, H, H, C)
        pooled = G.mean(dim=(0, 1, 2))
        hm = (pooled * A[0]).sum(-1)
        out.append((torch.clamp(hm, min=0) / hm.max()).detach())
    return torch.stack(out, 0)
