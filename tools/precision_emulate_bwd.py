"""Where does the bf16 path's GRADIENT error come from?  A CPU emulation (round 5).

The fp32 oracle (oracle/vit_ref.py, models/CvT(Par).py:261-289 restated) run through autograd with
bf16 rounding inserted where the GPU path rounds, one class at a time:

  forward operands (rounded values; the backward sees the rounded operand, as on the GPU):
    W     every GEMM weight                    A     the bf16 GEMM activation operands (patches,
                                                     LN outputs, attention output, GELU output)
    QKV   q, k, v (and P in P.V)
  backward gradient operands (identity forward, gradient rounded to bf16 on its way back):
    GBR   the branch-output gradients the GEMMs read (g2_lp into fc2, dx1_lp into the out-proj)
    GDU   du = dL/du of the GELU input (the DGELU epilogue's bf16 output)
    GDH   dL/dh of the LayerNorm outputs (the dgrad GEMMs' bf16 outputs, read by the LN backward)
    GDO   dL/dO of the attention output
    GQKV  dL/d(q, k, v) (the attention backward's bf16 output)

Prints, per setting, the worst and the median relative gradient error over all parameter
tensors against the unrounded fp32 oracle, plus the logits error.
usage: python tools/precision_emulate_bwd.py [--config c1|vitb] [--batch B] [--labels zero|seed] [--knob]"""
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
from vitmi.config import config_c1, preset  # noqa: E402

FWD = ("W", "A", "QKV")
BWD = ("GBR", "GDU", "GDH", "GDO", "GQKV")


def rb(x):
    return x.bfloat16().float()


class RoundVal(torch.autograd.Function):
    """bf16-rounded value, straight-through gradient."""
    @staticmethod
    def forward(ctx, x):
        return rb(x)

    @staticmethod
    def backward(ctx, g):
        return g


class RoundGrad(torch.autograd.Function):
    """Identity value, bf16-rounded gradient."""
    @staticmethod
    def forward(ctx, x):
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        return rb(g)


def forward(img, p, cfg, on):
    V = lambda key, x: RoundVal.apply(x) if key in on else x      # noqa: E731
    G = lambda key, x: RoundGrad.apply(x) if key in on else x     # noqa: E731
    B = img.shape[0]
    D, H = cfg.embed_dim, cfg.num_heads
    dh = D // H
    Pz = cfg.patch_size
    wp = V("W", p["patch_embed.proj.weight"].reshape(D, -1))
    patches = V("A", F.unfold(img, Pz, stride=Pz).transpose(1, 2))
    x = patches @ wp.t() + p["patch_embed.proj.bias"]
    x = torch.cat([p["cls_token"].expand(B, 1, D), x], dim=1)
    if cfg.pos_embed:
        x = x + p["pos_embed"]
    N = x.shape[1]
    scale = dh ** -0.5 if cfg.attn_scale == "head" else D ** -0.5
    for i in range(cfg.depth):
        pre = f"blocks.{i}."
        h = G("GDH", V("A", vit_ref.layer_norm(x, p[pre + "norm1.weight"], p[pre + "norm1.bias"], cfg.ln_eps)))
        qkv = h @ V("W", p[pre + "attn.qkv.weight"]).t() + p[pre + "attn.qkv.bias"]
        qkv = G("GQKV", V("QKV", qkv))
        q, k, v = (t.reshape(B, N, H, dh).transpose(1, 2) for t in qkv.split(D, dim=-1))
        a = torch.softmax((q @ k.transpose(-1, -2)) * scale, dim=-1)
        o = (V("QKV", a) @ v).transpose(1, 2).reshape(B, N, D)
        o = G("GDO", V("A", o))
        br = o @ V("W", p[pre + "attn.proj.weight"]).t() + p[pre + "attn.proj.bias"]
        x = x + G("GBR", br)
        h2 = G("GDH", V("A", vit_ref.layer_norm(x, p[pre + "norm2.weight"], p[pre + "norm2.bias"], cfg.ln_eps)))
        u = G("GDU", h2 @ V("W", p[pre + "mlp.fc1.weight"]).t() + p[pre + "mlp.fc1.bias"])
        act = V("A", F.gelu(u))
        br2 = act @ V("W", p[pre + "mlp.fc2.weight"]).t() + p[pre + "mlp.fc2.bias"]
        x = x + G("GBR", br2)
    c = vit_ref.layer_norm(x[:, 0], p["norm.weight"], p["norm.bias"], cfg.ln_eps)
    return c @ p["head.weight"].t() + p["head.bias"]


def grads(img, tgt, params, cfg, on):
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in params.items()}
    logits = forward(img, leaves, cfg, on)
    vit_ref.loss_fn(logits, tgt, cfg.num_classes).backward()
    return logits.detach(), {k: v.grad.detach() for k, v in leaves.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=["c1", "vitb"], default="c1")
    ap.add_argument("--batch", type=int, default=5)
    ap.add_argument("--labels", choices=["seed", "zero"], default="seed")
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--knob", action="store_true", help="settings around the bf16x3 knob's roundings")
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    if args.config == "c1":
        cfg = config_c1(dtype="fp32")
        params = vit_ref.init_params(cfg, seed=3)
    else:
        cfg = preset("vit_base_16", img_size=224, num_classes=2, dtype="fp32")
        params = vit_ref.init_params(cfg, seed=0)
    img, tgt = vit_ref.synthetic_batch(cfg, args.batch)
    if args.labels == "zero":
        tgt = torch.zeros_like(tgt)
    l_ref, g_ref = grads(img, tgt, params, cfg, set())
    settings = [("all (the GPU bf16 path)", set(FWD + BWD)), ("forward roundings only", set(FWD)),
                ("backward gradient roundings only", set(BWD))]
    settings += [(f"only {k}", {k}) for k in FWD + BWD]
    settings += [(f"all but {k}", set(FWD + BWD) - {k}) for k in FWD + BWD]
    if args.knob:   # the bf16x3 knob: split (unrounded) W and A, bf16 q/k/v/P and bf16 backward
        knob = {"QKV"} | set(BWD)
        settings = [("knob (QKV + backward)", knob)] + [(f"knob but {k}", knob - {k}) for k in ("QKV",) + BWD]
    print(f"{args.config} bs {args.batch} labels {tgt.tolist()}")
    print(f"{'bf16 rounding of':<40} {'worst grad rel':>14} {'(tensor)':<28} {'median':>9} {'logits':>9}")
    for name, on in settings:
        l, g = grads(img, tgt, params, cfg, on)
        errs = sorted((vit_ref.rel_err(g[k], g_ref[k]), k) for k in g_ref)
        worst = errs[-1]
        med = errs[len(errs) // 2][0]
        print(f"{name:<40} {worst[0]:14.3e} {worst[1]:<28} {med:9.2e} {(l - l_ref).abs().max().item():9.2e}",
              flush=True)


if __name__ == "__main__":
    main()
