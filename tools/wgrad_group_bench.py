"""Time a ViT block's four weight gradients (bf16, C3: M = 256 x 197 tokens) as one grouped launch
(ops.linear_wgrad_group: one split-K launch + one reduction) against one ops.linear_wgrad each.
usage: python tools/wgrad_group_bench.py [depth-like config: b (ViT-B, default) | l (ViT-L C5)]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402


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
    cfg = sys.argv[1] if len(sys.argv) > 1 else "b"
    M, D, F = (256 * 197, 768, 3072) if cfg == "b" else (64 * 577, 1024, 4096)
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s: (torch.randn(*s, device="cuda", generator=g) * 0.5).to(torch.bfloat16)  # noqa: E731
    shapes = [(D, F), (F, D), (D, D), (3 * D, D)]   # fc2, fc1, proj, qkv: dW[N, K] += dy[M, N]^T x[M, K]
    items = [(r(M, n), r(M, k), torch.zeros(n, k, device="cuda")) for n, k in shapes]
    t_sep = timed(lambda: [ops.linear_wgrad(dy, x, dw) for dy, x, dw in items])
    t_grp = timed(lambda: ops.linear_wgrad_group(items))
    flops = sum(2.0 * M * n * k for n, k in shapes)
    print(f"{cfg}: M={M}  separate {t_sep:8.1f} us ({flops / t_sep / 1e6:6.1f} TF)   grouped {t_grp:8.1f} us "
          f"({flops / t_grp / 1e6:6.1f} TF)")


if __name__ == "__main__":
    main()
