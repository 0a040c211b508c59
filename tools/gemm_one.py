"""Run ONE GEMM configuration a few times (the target of a rocprofv3 --pmc pass).
usage: python tools/gemm_one.py [fc1_gelu|fc1_store|fc2_res] [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402

M, D, F = 256 * 197, 768, 3072     # ViT-B/16, 256 images of 197 tokens (bench workload)
BF = torch.bfloat16


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "fc1_gelu"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    g = torch.Generator(device="cuda").manual_seed(0)
    x = (torch.rand(M, D, device="cuda", generator=g) * 2 - 1).to(BF)
    h = (torch.rand(M, F, device="cuda", generator=g) * 2 - 1).to(BF)
    w1 = ((torch.rand(F, D, device="cuda", generator=g) * 2 - 1) * 0.05).to(BF)
    w2 = ((torch.rand(D, F, device="cuda", generator=g) * 2 - 1) * 0.05).to(BF)
    b1, b2 = torch.zeros(F, device="cuda"), torch.zeros(D, device="cuda")
    res = torch.rand(M, D, device="cuda")
    fn = {"fc1_gelu": lambda: ops.linear_fwd(x, w1, b1, BF, ops.EPI_BIAS_GELU, aux_tiled=True),   # as the model
          "fc1_store": lambda: ops.linear_fwd(x, w1, b1, BF),
          "fc2_res": lambda: ops.linear_fwd(h, w2, b2, torch.float32, ops.EPI_RESIDUAL, res)}[which]
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    print("done", which, iters)


if __name__ == "__main__":
    main()
