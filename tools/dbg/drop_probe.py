"""Probe of the fused GELU-dropout epilogue at the ViT shape: which dropped elements come out
nonzero, and where (found the SGPR hazard of the asm epilogue stores).
usage: python tools/dbg/drop_probe.py"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd")); sys.path.insert(0, ROOT)
import numpy as np, torch
from vitmi import ops
from oracle import vit_ref
g = torch.Generator(device="cuda").manual_seed(0)
M, D, F = 197 * 16, 768, 3072
x = (torch.rand(M, D, device="cuda", generator=g) - 0.5).to(torch.bfloat16)
w = ((torch.rand(F, D, device="cuda", generator=g) - 0.5) * 0.1).to(torch.bfloat16)
b = torch.zeros(F, device="cuda")
a0, u0 = ops.linear_fwd(x, w, b, torch.bfloat16, ops.EPI_BIAS_GELU)
a1, u1 = ops.linear_fwd(x, w, b, torch.bfloat16, ops.EPI_BIAS_GELU, dropout=(7, 1, 0.1))
keep = vit_ref.dropout_hash(7, 1, np.arange(M), np.arange(F)) >= vit_ref.dropout_params(0.1)[0]
kt = torch.from_numpy(keep).cuda()
for name, t in (("a", a1), ("u", u1)):
    bad = (t != 0) & ~kt
    print(name, "dropped-but-nonzero:", int(bad.sum()), "of", int((~kt).sum()))
    idx = bad.nonzero()[:8].tolist()
    print(" ", [(r, c, float(t[r, c]), float(a0[r, c]), float(u0[r, c])) for r, c in idx])
    rows = bad.any(1).nonzero().flatten()
    cols = bad.any(0).nonzero().flatten()
    print("  rows", rows[:10].tolist(), len(rows), "cols", cols[:10].tolist(), len(cols))
ref = (a0.float() / 0.9)
kb = kt
print("kept rel max", float(((a1.float() - ref).abs() / (ref.abs() + 1e-3))[kb].max()))
