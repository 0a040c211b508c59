"""Run one NT (qkv fwd), NN (fc1 dgrad) and TN (fc1 wgrad) ViT GEMM a few times: the target of
rocprofv3 --pmc passes comparing the three operand layouts of gemm256.
usage: python tools/gemm_pmc_one.py [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402

M, D, F = 256 * 197, 768, 3072
BF = torch.bfloat16


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    g = torch.Generator(device="cuda").manual_seed(0)
    x = ((torch.rand(M, D, device="cuda", generator=g) * 2 - 1)).to(BF)
    h = ((torch.rand(M, F, device="cuda", generator=g) * 2 - 1)).to(BF)
    w1 = ((torch.rand(F, D, device="cuda", generator=g) * 2 - 1) * 0.05).to(BF)
    b1 = torch.zeros(F, device="cuda")
    dw = torch.zeros(F, D, device="cuda")
    for _ in range(iters):
        ops.linear_fwd(x, w1, b1, BF)        # NT  [M x 3072 x 768]
        ops.linear_dgrad(h, w1, BF)          # NN  [M x 768 x 3072]
        ops.linear_wgrad(h, x, dw)           # TN  [3072 x 768 x M]
    torch.cuda.synchronize()
    print("done", iters)


if __name__ == "__main__":
    main()
