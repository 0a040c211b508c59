"""Time the bf16 attention kernels at the ViT-B/16 bs=256 shape: the whole-sequence path (its
single-pass backward, policy 0; its two-kernel backward, policy 3) vs the streamed path (policy 1).
usage: python tools/attn_bench.py [B] [N] [H]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402


def t(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    B, N, H = (int(a) for a in (sys.argv[1:] + ["256", "197", "12"][len(sys.argv) - 1:]))
    D = 64 * H
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = (torch.randn(B * N, 3 * D, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    do = torch.randn(B * N, D, device="cuda", generator=g).to(torch.bfloat16)
    pairs = B * H * N * N
    for path, pol in (("seq", 0), ("seq2k", 3), ("stream", 1)):
        ops.attention_set_policy(pol)
        o, lse = ops.attention_fwd(qkv, B, N, H, 0.125)
        tf = t(lambda: ops.attention_fwd(qkv, B, N, H, 0.125))
        tb = t(lambda: ops.attention_bwd(qkv, o, do, lse, B, N, H, 0.125))
        print(f"{path:6s} fwd {tf:7.1f} us ({4 * 64 * pairs / tf / 1e6:6.1f} TF)  "
              f"bwd {tb:7.1f} us ({10 * 64 * pairs / tb / 1e6:6.1f} TF)", flush=True)
    ops.attention_set_policy(0)


if __name__ == "__main__":
    main()
