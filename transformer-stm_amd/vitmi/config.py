"""ViT configuration for the MI355X training path.

The reference builds its transformer stage from a ``spec`` dict of module-level
constants (``models/CvT(Par).py:66-72``) and the Keras layer arguments of
``ConvEmbed`` / ``ConvTransformerBlock`` (``models/CvT(Par).py:194-289``).  A ViT
in that vocabulary is one stage with ``patch_size == stride == 16`` and
``qkv_method='linear'`` (identity convolutional projection,
``models/CvT(Par).py:97-98,109-110``).  ``ViTConfig`` carries exactly those knobs
plus the semantic switches on which the reference's two implementations
disagree:

=================  ==============================  ==============================
knob               Keras CvT (the model that ran)  MS_CvT (``old_codes/MS_CvT.py``)
=================  ==============================  ==============================
attn_scale         'head'  1/sqrt(D/H)  (:137)      'dim'  1/sqrt(D)  (:100)
ln_eps             1e-6 (:248)                      1e-5 (:633)
qkv_bias           True (Dense default :132-134)    False (:82)
embed_norm         False (norm never built, :209)   True (:358,365-366)
tie_norms          True (one norm1 used twice)      False (norm1/norm2)
=================  ==============================  ==============================
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass


@dataclass
class ViTConfig:
    img_size: int = 224
    patch_size: int = 16
    in_chans: int = 3
    embed_dim: int = 768
    depth: int = 12
    num_heads: int = 12
    mlp_ratio: float = 4.0
    num_classes: int = 2
    # semantic knobs (see module docstring)
    attn_scale: str = "head"      # 'head' -> dh**-0.5 (Keras), 'dim' -> D**-0.5 (MS_CvT)
    ln_eps: float = 1e-6
    qkv_bias: bool = True
    embed_norm: bool = False
    pos_embed: bool = True
    tie_norms: bool = False
    with_cls_token: bool = True
    # dropout after the out-projection and in the MLP (models/CvT(Par).py:141,189,255,257;
    # Keras default 0.1, training mode only).  0 = the parity / benchmark configuration.
    drop_rate: float = 0.0
    # compute dtype of the device path: 'bf16' (MFMA bf16, fp32 accumulate and
    # fp32 residual stream), 'bf16x3' (the precision knob: as bf16, with the forward GEMMs'
    # weights, LayerNorm outputs, attention output and GELU output carried as split hi + lo
    # bf16 pairs and the attention forward in fp32; logits within 1e-3 of the fp32 reference),
    # 'bf16f8' (the same knob with the two correction products as one block-scaled e4m3 GEMM
    # product: 2K- instead of 3K-equivalent forward GEMM work, include/vitmi.h VITMI_BF16F8)
    # or 'fp32' (f32-input MFMA, exact fp32 products)
    dtype: str = "bf16"
    # the precision knobs' qkv GEMM on split operands (True), plain bf16 (False) or, for 'bf16f8',
    # with the weight-side correction alone ("weight": VITMI_BF16F8W, needs embed_dim % 128 == 0);
    # None = the knob's default: split for 'bf16x3', "weight" for 'bf16f8' (plain where
    # embed_dim % 128 != 0).  vitmi/modules.py Block.split_qkv
    split_qkv: "bool | str | None" = None

    @property
    def grid(self) -> int:
        return self.img_size // self.patch_size

    @property
    def num_patches(self) -> int:
        return self.grid * self.grid

    @property
    def seq_len(self) -> int:
        return self.num_patches + (1 if self.with_cls_token else 0)

    @property
    def head_dim(self) -> int:
        return self.embed_dim // self.num_heads

    @property
    def mlp_dim(self) -> int:
        return int(self.embed_dim * self.mlp_ratio)

    @property
    def scale(self) -> float:
        if self.attn_scale == "head":
            return self.head_dim ** -0.5
        if self.attn_scale == "dim":
            return self.embed_dim ** -0.5
        raise ValueError(f"Unknown attn_scale: {self.attn_scale}")

    def replace(self, **kw) -> "ViTConfig":
        return dataclasses.replace(self, **kw)

    def flops_per_image_fwd(self) -> float:
        """Algorithmic forward FLOPs per image (2 x MAC over every dense contraction).

        Counts patch-embed, QKV, QK^T, PV, out-proj, fc1, fc2 and head, as
        BASELINE.md prescribes (LN/softmax/GELU excluded).  Mirrors the MAC
        convention of ``Attention.compute_macs`` (``old_codes/MS_CvT.py:214-286``).
        """
        D, N, F, L = self.embed_dim, self.seq_len, self.mlp_dim, self.depth
        P2C = self.patch_size * self.patch_size * self.in_chans
        macs = self.num_patches * P2C * D
        per_block = N * D * 3 * D + 2 * N * N * D + N * D * D + 2 * N * D * F
        macs += L * per_block + D * self.num_classes
        return 2.0 * macs

    def flops_per_image_fwd_bwd(self) -> float:
        return 3.0 * self.flops_per_image_fwd()


PRESETS = {
    # name: (img, patch, dim, depth, heads)
    "vit_tiny_16": dict(embed_dim=192, depth=12, num_heads=3),
    "vit_small_16": dict(embed_dim=384, depth=12, num_heads=6),
    "vit_base_16": dict(embed_dim=768, depth=12, num_heads=12),
    "vit_large_16": dict(embed_dim=1024, depth=24, num_heads=16),
}


def preset(name: str, **kw) -> ViTConfig:
    base = dict(PRESETS[name])
    base.update(kw)
    return ViTConfig(**base)


# BASELINE.json configs (C1..C5)
def config_c1(**kw) -> ViTConfig:
    return preset("vit_tiny_16", **{**dict(img_size=64, num_classes=2, dtype="fp32"), **kw})


def config_c2(**kw) -> ViTConfig:
    return preset("vit_small_16", **{**dict(img_size=224, num_classes=2, dtype="fp32"), **kw})


def config_c3(**kw) -> ViTConfig:
    return preset("vit_base_16", **{**dict(img_size=224, num_classes=2, dtype="bf16"), **kw})


def config_c5(**kw) -> ViTConfig:
    return preset("vit_large_16", **{**dict(img_size=384, num_classes=2, dtype="bf16"), **kw})
