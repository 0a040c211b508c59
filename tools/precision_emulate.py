"""Where the bf16 logits error of the ViT path comes from: a CPU emulation.

The fp32 oracle forward (oracle/vit_ref.py, models/CvT(Par).py:261-289 restated) with bf16
rounding r(x) = float(bf16(x)) inserted exactly where the GPU path rounds an operand or a stored
activation, one class of roundings switched on or off at a time:

    W     every GEMM weight (patch, qkv, proj, fc1, fc2)      -- the bf16 operand shadow
    WB    the block GEMM weights (qkv, proj, fc1, fc2)
    WP    the patch-embedding weight alone
    P     the im2col patches                                   -- patch GEMM A operand
    LN    the LayerNorm outputs h1, h2                         -- qkv / fc1 A operands
    QKV   the stored q, k, v                                   -- attention inputs
    PR    the softmax probabilities fed to P.V                 -- inside the attention kernel
    O     the stored attention output                          -- out-projection A operand
    ACT   the stored GELU output                               -- fc2 A operand

Accumulation, LayerNorm statistics, softmax, the residual stream and the head stay fp32, as on
the GPU.  An operand carried as two bf16 terms (hi + lo, the "bf16x3" products of the precision
knob) is emulated as not rounded: its residual error (2^-16 relative per product) is far below
what is measured here.

    python tools/precision_emulate.py [--depth 12] [--batch 2] [--init random|default]

Prints one line per setting: logits max-abs against the unrounded fp32 forward.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))

from oracle import vit_ref  # noqa: E402
from vitmi.config import preset  # noqa: E402

ALL = ("W", "P", "LN", "QKV", "PR", "O", "ACT")
BLOCK_W = ("attn.qkv.weight", "attn.proj.weight", "mlp.fc1.weight", "mlp.fc2.weight")


def r(x, on):
    return x.bfloat16().float() if on else x


def forward(img, p, cfg, rnd):
    R = lambda key, x: r(x, key in rnd)  # noqa: E731
    w = {k: (R("W", v) if k.endswith("weight") and ("proj" in k or "qkv" in k or "fc" in k) else v) for k, v in p.items()}
    w["patch_embed.proj.weight"] = R("WP", w["patch_embed.proj.weight"])   # WP: the patch weight alone
    w = {k: (R("WB", v) if k.endswith(BLOCK_W) else v) for k, v in w.items()}
    B = img.shape[0]
    D, H = cfg.embed_dim, cfg.num_heads
    dh = D // H
    Pz = cfg.patch_size
    patches = F.unfold(img, Pz, stride=Pz).transpose(1, 2)                       # [B, np, C*P*P]
    x = R("P", patches) @ w["patch_embed.proj.weight"].reshape(D, -1).t() + p["patch_embed.proj.bias"]
    x = torch.cat([p["cls_token"].expand(B, 1, D), x], dim=1)
    if cfg.pos_embed:
        x = x + p["pos_embed"]
    N = x.shape[1]
    scale = dh ** -0.5 if cfg.attn_scale == "head" else D ** -0.5
    for i in range(cfg.depth):
        pre = f"blocks.{i}."
        h = R("LN", vit_ref.layer_norm(x, p[pre + "norm1.weight"], p[pre + "norm1.bias"], cfg.ln_eps))
        qkv = R("QKV", h @ w[pre + "attn.qkv.weight"].t() + p[pre + "attn.qkv.bias"])
        q, k, v = (t.reshape(B, N, H, dh).transpose(1, 2) for t in qkv.split(D, dim=-1))
        a = torch.softmax((q @ k.transpose(-1, -2)) * scale, dim=-1)
        o = R("O", (R("PR", a) @ v).transpose(1, 2).reshape(B, N, D))
        x = x + o @ w[pre + "attn.proj.weight"].t() + p[pre + "attn.proj.bias"]
        n2 = "norm1" if cfg.tie_norms else "norm2"
        h2 = R("LN", vit_ref.layer_norm(x, p[pre + n2 + ".weight"], p[pre + n2 + ".bias"], cfg.ln_eps))
        act = R("ACT", F.gelu(h2 @ w[pre + "mlp.fc1.weight"].t() + p[pre + "mlp.fc1.bias"]))
        x = x + act @ w[pre + "mlp.fc2.weight"].t() + p[pre + "mlp.fc2.bias"]
    c = vit_ref.layer_norm(x[:, 0], p["norm.weight"], p["norm.bias"], cfg.ln_eps)
    return c @ p["head.weight"].t() + p["head.bias"]


SETTINGS = [
    ("all bf16 (the default path)", set(ALL)),
    ("weights only", {"W"}),
    ("LN outputs only", {"LN"}),
    ("attention output O only", {"O"}),
    ("GELU output only", {"ACT"}),
    ("q, k, v only", {"QKV"}),
    ("softmax P only", {"PR"}),
    ("patches only", {"P"}),
    ("the knob as built: GEMM operands split; q/k/v and P bf16", {"QKV", "PR"}),
    ("bf16x3 on W, P, LN, ACT; O, q/k/v and P bf16", {"QKV", "PR", "O"}),
    ("bf16x3 on W, LN, O, ACT; patches, q/k/v and P bf16", {"QKV", "PR", "P"}),
    ("bf16x3 on the block GEMMs; the patch GEMM (patches, weight) bf16", {"QKV", "PR", "P", "WP"}),
    ("the patch weight only", {"WP"}),
    ("block weights only", {"WB"}),
    ("split O, GELU, patch GEMM; LN outputs and block weights bf16", {"QKV", "PR", "LN", "WB"}),
    ("split W, O, GELU, patch GEMM; LN outputs bf16", {"QKV", "PR", "LN"}),
    ("split LN, O, GELU, patch GEMM; block weights bf16", {"QKV", "PR", "WB"}),
    ("split GELU, patch GEMM; LN, O, block weights bf16", {"QKV", "PR", "LN", "WB", "O"}),
    ("split O, GELU, W; LN outputs and the patches bf16", {"QKV", "PR", "LN", "P"}),
    ("none (GEMM operands split and attention in fp32)", set()),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--init", choices=["random", "default"], default="random",
                    help="random: the parity stress case (randomised gamma/beta/biases, init_params(seed=0)); "
                         "default: trunc_normal weights, zero biases, LN (1, 0)")
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 1))
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    cfg = preset("vit_base_16", img_size=224, num_classes=2, dtype="fp32", depth=args.depth)
    params = vit_ref.init_params(cfg, seed=0, randomize_all=args.init == "random")
    img, _ = vit_ref.synthetic_batch(cfg, args.batch)
    with torch.no_grad():
        ref = vit_ref.forward(img, params, cfg)
        base = forward(img, params, cfg, set())
        print(f"ViT-B/16 224px depth {args.depth} bs {args.batch}, {args.init} init; "
              f"emulator without rounding vs oracle: {(base - ref).abs().max().item():.2e}")
        print(f"{'bf16 rounding of':<66} logits max-abs vs fp32")
        for name, rnd in SETTINGS:
            err = (forward(img, params, cfg, rnd) - ref).abs().max().item()
            print(f"{name:<66} {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
