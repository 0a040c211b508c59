"""Does the token-major q|k|v layout cost the whole-sequence attention kernels?  The same work
(ViT-B bs 256: B*H = 3072 pairs, N = 197, dh 64) timed on the step's layout ([B*N][3*768], a head's
row is 128 B of a 4608-B row) and on a head-major one ([B*H*N][3*64]: every pair reads contiguous
384-B rows), via B' = B*H, H' = 1.  usage: python tools/attn_layout.py"""
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
    B, N, H = 256, 197, 12
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, (b, h) in (("token-major [B*N][3*768]", (B, H)), ("head-major [B*H*N][3*64]", (B * H, 1))):
        D = 64 * h
        qkv = (torch.randn(b * N, 3 * D, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
        do = torch.randn(b * N, D, device="cuda", generator=g).to(torch.bfloat16)
        o, lse = ops.attention_fwd(qkv, b, N, h, 0.125)
        tf = t(lambda: ops.attention_fwd(qkv, b, N, h, 0.125))
        tb = t(lambda: ops.attention_bwd(qkv, o, do, lse, b, N, h, 0.125))
        print(f"{name:28s} fwd {tf:7.1f} us  bwd {tb:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
