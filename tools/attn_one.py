"""Run the bf16 whole-sequence attention forward + backward at the ViT-B/16 bs=256 shape a few
times (the target of a rocprofv3 --pmc pass).  usage: python tools/attn_one.py [iters] [B N H]
(default shape ViT-B/16 bs 256: 256 197 12; C5 is 64 577 16)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    B, N, H = (int(a) for a in sys.argv[2:5]) if len(sys.argv) >= 5 else (256, 197, 12)
    D = 64 * H
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = (torch.randn(B * N, 3 * D, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    do = torch.randn(B * N, D, device="cuda", generator=g).to(torch.bfloat16)
    for _ in range(iters):
        o, lse = ops.attention_fwd(qkv, B, N, H, 0.125)
        ops.attention_bwd(qkv, o, do, lse, B, N, H, 0.125)
    torch.cuda.synchronize()
    print("done", iters)


if __name__ == "__main__":
    main()
