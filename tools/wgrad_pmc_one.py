"""One ViT-B/16 bs=256 weight-gradient GEMM shape (ops.linear_wgrad, the split-K TN gemm256) a few
times: the target of rocprofv3 --pmc passes (tools/gpu/wgrad_pmc.sh).
usage: python tools/wgrad_pmc_one.py fc1|fc2|qkv|proj [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402

BF = torch.bfloat16
M = 256 * 197
SHAPES = {"proj": (768, 768), "qkv": (2304, 768), "fc1": (3072, 768), "fc2": (768, 3072)}


def main():
    name = sys.argv[1]
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    n, k = SHAPES[name]
    g = torch.Generator(device="cuda").manual_seed(0)
    dy = (torch.rand(M, n, device="cuda", generator=g) - 0.5).to(BF)
    x = (torch.rand(M, k, device="cuda", generator=g) - 0.5).to(BF)
    dw = torch.zeros(n, k, device="cuda")
    for _ in range(iters):
        ops.linear_wgrad(dy, x, dw)
    torch.cuda.synchronize()
    print("done", name, iters)


if __name__ == "__main__":
    main()
