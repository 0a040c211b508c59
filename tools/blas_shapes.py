"""Time hipBLASLt (torch.mm, bf16 in/out) on the ViT-B/16 bs=256 GEMM shapes, for comparison with
tools/gemm_shapes.py (gemm256).  usage: python tools/blas_shapes.py"""
import torch

M, D, F = 256 * 197, 768, 3072
BF = torch.bfloat16


def timed(fn, iters=20):
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
    g = torch.Generator(device="cuda").manual_seed(0)

    def r(*s):
        return (torch.rand(*s, device="cuda", generator=g) * 2 - 1).to(BF)

    x, h, dq = r(M, D), r(M, F), r(M, 3 * D)
    wqkv, w1, w2 = r(3 * D, D), r(F, D), r(D, F)
    cases = [
        ("NT qkv fwd  [M x 2304 x 768]", 2 * M * 3 * D * D, lambda: torch.mm(x, wqkv.t())),
        ("NT fc1 fwd  [M x 3072 x 768]", 2 * M * F * D, lambda: torch.mm(x, w1.t())),
        ("NT fc2 fwd  [M x 768 x 3072]", 2 * M * D * F, lambda: torch.mm(h, w2.t())),
        ("NN fc1 dgrad [M x 768 x 3072]", 2 * M * D * F, lambda: torch.mm(h, w1)),
        ("NN qkv dgrad [M x 768 x 2304]", 2 * M * D * 3 * D, lambda: torch.mm(dq, wqkv)),
        ("TN fc1 wgrad [3072 x 768 x M]", 2 * M * F * D, lambda: torch.mm(h.t(), x)),
        ("TN qkv wgrad [2304 x 768 x M]", 2 * M * 3 * D * D, lambda: torch.mm(dq.t(), x)),
    ]
    for name, fl, fn in cases:
        us = timed(fn)
        print(f"{name:34s} {us:8.1f} us  {fl / us / 1e6:7.1f} TF", flush=True)


if __name__ == "__main__":
    main()
