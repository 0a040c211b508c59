#!/usr/bin/env python
"""CvT training-step throughput: the vitmi CvT (Keras spec
models/CvT(Par).py:66-72, 128x128x1, dw_bn) against the same network written in plain
PyTorch-ROCm eager ops (MIOpen conv / batch_norm, hipBLASLt linears, SDPA) under bf16 autocast,
both with a fused Adam step, on one GPU.  Prints one JSON line.

    python tools/cvt_bench.py [--batch 256 --steps 20 --warmup 5 --no-torch]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from vitmi import cvt  # noqa: E402
from vitmi.modules import mse_loss  # noqa: E402


def same_pad(x, k, s):
    H = x.shape[-1]
    Ho, _, pt, pl = cvt._geometry(H, k, s, None)
    tot = max((Ho - 1) * s + k - H, 0)
    return F.pad(x, (pl, tot - pl, pt, tot - pt))


def torch_forward(p, bufs, img, cfg: cvt.CvTConfig):
    """The same CvT in eager torch ops (NCHW), BN in training mode with moving stats."""
    x = img
    tok = None
    for i, st in enumerate(cfg.stages):
        pre = f"stage{i}."
        x = F.conv2d(same_pad(x, st.patch_size, st.stride), p[pre + "embed.weight"], p[pre + "embed.bias"],
                     stride=st.stride)
        B, D, H, W = x.shape
        t = x.flatten(2).transpose(1, 2)
        if st.with_cls_token:
            t = torch.cat([p[pre + "cls_token"].expand(B, 1, D).to(t.dtype), t], dim=1)
        for j in range(st.depth):
            b = f"{pre}blocks.{j}."
            h = F.layer_norm(t.float(), (D,), p[b + "norm1.weight"], p[b + "norm1.bias"], cfg.ln_eps)
            cls, sp = (h[:, :1], h[:, 1:]) if st.with_cls_token else (None, h)
            im = sp.transpose(1, 2).reshape(B, D, H, W)
            qkv = []
            for c in "qkv":
                a = b + f"attn.conv_proj_{c}."
                z = F.conv2d(im, p[a + "weight"], None, padding=1, groups=D)
                z = F.batch_norm(z, bufs[a + "bn.running_mean"], bufs[a + "bn.running_var"], p[a + "bn.weight"],
                                 p[a + "bn.bias"], training=True, momentum=1 - cfg.bn_momentum, eps=cfg.bn_eps)
                z = z.flatten(2).transpose(1, 2)
                if cls is not None:
                    z = torch.cat([cls.to(z.dtype), z], dim=1)
                qkv.append(F.linear(z, p[b + f"attn.proj_{c}.weight"], p[b + f"attn.proj_{c}.bias"]))
            Hh = st.num_heads
            q, k, v = (u.reshape(B, -1, Hh, D // Hh).transpose(1, 2) for u in qkv)
            o = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, -1, D)
            t = t + F.linear(o, p[b + "attn.proj.weight"], p[b + "attn.proj.bias"])
            y = F.layer_norm(t.float(), (D,), p[b + "norm1.weight"], p[b + "norm1.bias"], cfg.ln_eps)
            y = F.linear(F.gelu(F.linear(y, p[b + "mlp.fc1.weight"], p[b + "mlp.fc1.bias"])),
                         p[b + "mlp.fc2.weight"], p[b + "mlp.fc2.bias"])
            t = t + y
        if st.with_cls_token:
            tok, t = t[:, 0], t[:, 1:]
        x = t.transpose(1, 2).reshape(B, D, H, W)
    f = F.layer_norm(tok.float(), (tok.shape[-1],), p["norm.weight"], p["norm.bias"], cfg.ln_eps)
    return F.linear(f, p["head.weight"], p["head.bias"])


def timeit(step, warmup, steps):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--img", type=int, default=128)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-torch", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = cvt.CvTConfig(img_size=args.img, num_classes=1, dtype="bf16")
    B = args.batch
    g = torch.Generator(device=dev).manual_seed(1234)
    img = torch.rand(B, 1, args.img, args.img, device=dev, generator=g)
    tgt = torch.randn(B, device=dev, generator=g)

    model = cvt.CvT(cfg).to(dev)
    model.reset_parameters(0)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4, fused=True)

    def step_vitmi():
        opt.zero_grad()
        loss = mse_loss(model(img), tgt)
        loss.backward()
        opt.step()

    t_v = timeit(step_vitmi, args.warmup, args.steps)
    out = {"workload": f"CvT Keras spec (dw_bn, cls in stage 3) {args.img}x{args.img}x1 fwd + MSE + bwd + Adam",
           "batch": B, "vitmi_ms_per_step": round(t_v * 1e3, 3), "vitmi_images_per_sec": round(B / t_v, 1)}
    if not args.no_torch:
        p = {k: v.detach().clone().requires_grad_(True) for k, v in model.named_parameters()}
        bufs = {k: v.clone() for k, v in model.named_buffers()}
        topt = torch.optim.Adam(list(p.values()), lr=1e-4, fused=True)

        def step_torch():
            topt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = torch_forward(p, bufs, img, cfg)
            loss = F.mse_loss(y.float().squeeze(-1), tgt)
            loss.backward()
            topt.step()

        t_t = timeit(step_torch, args.warmup, args.steps)
        out.update({"torch_eager_ms_per_step": round(t_t * 1e3, 3), "torch_eager_images_per_sec": round(B / t_t, 1),
                    "speedup": round(t_t / t_v, 3)})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
