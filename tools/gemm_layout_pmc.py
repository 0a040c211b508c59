"""Run the ViT-B wgrad (TN), dgrad (NN) and fc1 store (NT) GEMMs a few times each: the target of
rocprofv3 --pmc passes comparing the three operand layouts.  usage: python tools/gemm_layout_pmc.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402

M, D, F = 256 * 197, 768, 3072
BF = torch.bfloat16
g = torch.Generator(device="cuda").manual_seed(0)
r = lambda *s: (torch.rand(*s, device="cuda", generator=g) * 2 - 1).to(BF)  # noqa: E731
x, h = r(M, D), r(M, F)
w1 = r(F, D) * 0.05
b1 = torch.zeros(F, device="cuda")
dw = torch.zeros(F, D, device="cuda")
for _ in range(3):
    ops.linear_fwd(x, w1, b1, BF)          # NT
    ops.linear_dgrad(h, w1, BF)            # NN
    ops.linear_wgrad(h, x, dw)             # TN (+ split-K reduce)
torch.cuda.synchronize()
print("done")
