"""Which side of each forward GEMM's bf16 rounding costs the logits? (a CPU emulation, round 6)

Per GEMM class (qkv, proj, fc1, fc2, patch) the corrections of the bf16f8 knob run both (f: hi.lo_w
+ lo_x.hi_w in fixed-scale e4m3, as built), only the weight side (w: hi_x.lo_w), only the activation
side (x: lo_x.hi_w) or none (b: plain bf16), on the fp32 oracle's forward (tools/
precision_emulate_fp8.py's emulator).  Prints logits max-abs over the first 2 images (the bench's
parity sample), over all images, and the RMS, against the fp32 oracle.
usage: python tools/precision_sides.py vitb|smoke COMBO[,COMBO...] [images]
       COMBO = five letters for qkv, proj, fc1, fc2, patch, e.g. wffff (profiles/r06_sides/)"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "transformer-stm_amd")):
    sys.path.insert(0, _p)
import precision_emulate_fp8 as pe  # noqa: E402
from oracle import vit_ref  # noqa: E402
from vitmi.config import ViTConfig, preset  # noqa: E402

torch.set_num_threads(8)
code = {"f": "f8fixed", "x": "f8x", "w": "f8w", "b": "bf16"}
m = {k: pe.make_mm(v, 0) for k, v in code.items()}
combos = sys.argv[2].split(",")
which = sys.argv[1]
if which == "vitb":
    cfg = preset("vit_base_16", img_size=224, num_classes=2, dtype="fp32", depth=12)
    params = vit_ref.init_params(cfg, seed=0, randomize_all=True)
    img, _ = vit_ref.synthetic_batch(cfg, int(sys.argv[3]) if len(sys.argv) > 3 else 2)
elif which == "smoke":
    cfg = ViTConfig(img_size=32, patch_size=8, embed_dim=128, depth=2, num_heads=2, num_classes=2, dtype="fp32")
    params = vit_ref.init_params(cfg, seed=0)
    img, _ = vit_ref.synthetic_batch(cfg, 4)
with torch.no_grad():
    ref = vit_ref.forward(img, params, cfg)
    for cb in combos:
        per = {c: m[v] for c, v in zip(("qkv", "proj", "fc1", "fc2", "patch"), cb)}
        d = pe.forward(img, params, cfg, m["f"], per) - ref
        # max-abs on the first 2 images (the bench's sample) and over all
        print(f"{which} qkv,proj,fc1,fc2,patch={cb}  max2 {d[:2].abs().max().item():.2e}  max {d.abs().max().item():.2e}  rms {d.pow(2).mean().sqrt().item():.2e}", flush=True)
