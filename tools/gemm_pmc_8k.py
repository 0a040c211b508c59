"""8192^3 bf16 GEMM in the NN (A k-major, B n-major: the dgrad layout) and TN (both operands
m/n-major: the weight-gradient layout) forms of gemm256, a few times each: the target of the
rocprofv3 --pmc passes of tools/gpu/gemm_tn_pmc.sh (verdict r04 item 4: why the TN loop is slower).
usage: python tools/gemm_pmc_8k.py [iters] [nn|tn|both]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402

BF = torch.bfloat16
S = 8192


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    which = sys.argv[2] if len(sys.argv) > 2 else "both"
    g = torch.Generator(device="cuda").manual_seed(0)
    a = (torch.rand(S, S, device="cuda", generator=g) * 2 - 1).to(BF)
    b = (torch.rand(S, S, device="cuda", generator=g) * 2 - 1).to(BF)
    c = torch.empty(S, S, device="cuda", dtype=BF)
    for _ in range(iters):
        if which in ("nn", "both"):
            ops.gemm(a, b, True, False, S, S, S, c)     # NN: A [M][K], B [K][N]
        if which in ("tn", "both"):
            ops.gemm(a, b, False, False, S, S, S, c)    # TN: A [K][M], B [K][N]
    torch.cuda.synchronize()
    print("done", which, iters)


if __name__ == "__main__":
    main()
