"""Does every block need the bf16f8 knob's corrections?  (a CPU emulation, round 6)

ViT-B/16 depth 12 on 8 images with randomised parameters: the knob as built (qkv with the
weight-side correction, the other classes both corrections) against plans that run the first /
last k blocks on plain bf16 operands, or one class plain in the first six blocks.  Prints logits
max-abs (first 2 images, all) and RMS against the fp32 oracle (profiles/r06_sides/).
usage: python tools/precision_blocks_f8.py"""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "transformer-stm_amd")):
    sys.path.insert(0, _p)
import precision_emulate_fp8 as pe  # noqa: E402
from oracle import vit_ref  # noqa: E402
from vitmi.config import preset  # noqa: E402
torch.set_num_threads(8)
rb = pe.rb
m = {k: pe.make_mm(v, 0) for k, v in {"f": "f8fixed", "x": "f8x", "w": "f8w", "b": "bf16"}.items()}

def forward(img, p, cfg, plan):
    """plan(block i, class) -> mm"""
    B = img.shape[0]; D, H = cfg.embed_dim, cfg.num_heads; dh = D // H; Pz = cfg.patch_size
    patches = F.unfold(img, Pz, stride=Pz).transpose(1, 2)
    x = m["f"](patches, p["patch_embed.proj.weight"].reshape(D, -1)) + p["patch_embed.proj.bias"]
    x = torch.cat([p["cls_token"].expand(B, 1, D), x], dim=1)
    if cfg.pos_embed: x = x + p["pos_embed"]
    N = x.shape[1]
    scale = dh ** -0.5 if cfg.attn_scale == "head" else D ** -0.5
    for i in range(cfg.depth):
        pre = f"blocks.{i}."
        h = vit_ref.layer_norm(x, p[pre + "norm1.weight"], p[pre + "norm1.bias"], cfg.ln_eps)
        qkv = rb(plan(i, "qkv")(h, p[pre + "attn.qkv.weight"]) + p[pre + "attn.qkv.bias"])
        q, k, v = (t.reshape(B, N, H, dh).transpose(1, 2) for t in qkv.split(D, dim=-1))
        a = rb(torch.softmax((q @ k.transpose(-1, -2)) * scale, dim=-1))
        o = (a @ v).transpose(1, 2).reshape(B, N, D)
        x = x + plan(i, "proj")(o, p[pre + "attn.proj.weight"]) + p[pre + "attn.proj.bias"]
        h2 = vit_ref.layer_norm(x, p[pre + "norm2.weight"], p[pre + "norm2.bias"], cfg.ln_eps)
        act = F.gelu(plan(i, "fc1")(h2, p[pre + "mlp.fc1.weight"]) + p[pre + "mlp.fc1.bias"])
        x = x + plan(i, "fc2")(act, p[pre + "mlp.fc2.weight"]) + p[pre + "mlp.fc2.bias"]
    c = vit_ref.layer_norm(x[:, 0], p["norm.weight"], p["norm.bias"], cfg.ln_eps)
    return c @ p["head.weight"].t() + p["head.bias"]

cfg = preset("vit_base_16", img_size=224, num_classes=2, dtype="fp32", depth=12)
params = vit_ref.init_params(cfg, seed=0, randomize_all=True)
img, _ = vit_ref.synthetic_batch(cfg, 8)
with torch.no_grad():
    ref = vit_ref.forward(img, params, cfg)
    def run(name, plan):
        d = forward(img, params, cfg, plan) - ref
        print(f"{name:<44} max2 {d[:2].abs().max().item():.2e}  max {d.abs().max().item():.2e}  rms {d.pow(2).mean().sqrt().item():.2e}", flush=True)
    base = lambda i, c: m["w"] if c == "qkv" else m["f"]
    run("default (qkv w, rest f)", base)
    for k in (2, 4, 6):
        run(f"first {k} blocks plain (qkv w kept)", lambda i, c, k=k: (m["w"] if c == "qkv" else m["b"]) if i < k else base(i, c))
        run(f"last {k} blocks plain (qkv w kept)", lambda i, c, k=k: (m["w"] if c == "qkv" else m["b"]) if i >= 12 - k else base(i, c))
    run("fc2 plain in the first 6", lambda i, c: m["b"] if (c == "fc2" and i < 6) else base(i, c))
    run("fc1 plain in the first 6", lambda i, c: m["b"] if (c == "fc1" and i < 6) else base(i, c))
