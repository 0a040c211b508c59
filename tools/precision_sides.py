import sys, os, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tools'); sys.path.insert(0, '/root/repo/transformer-stm_amd')
import precision_emulate_fp8 as pe
from oracle import vit_ref
from vitmi.config import preset, ViTConfig
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
