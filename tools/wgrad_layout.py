"""Weight-gradient GEMM rates of the four operand layouts on the ViT-B/16 bs=256 shapes:
TN (both operands token-major: the current vitmi_linear_wgrad), B^T given (x stored [K_in][M]),
A^T given (dy stored [N_out][M]) and both given (NT), all with the split-K fp32 accumulate.
usage: python tools/wgrad_layout.py [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402

BF = torch.bfloat16


def t(fn, iters):
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
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    M = 256 * 197
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s: (torch.rand(*s, device="cuda", generator=g) * 2 - 1).to(BF)  # noqa: E731
    for name, (n_out, k_in) in {"qkv": (2304, 768), "proj": (768, 768), "fc1": (3072, 768),
                                "fc2": (768, 3072)}.items():
        dy, x = r(M, n_out), r(M, k_in)
        dyT, xT = dy.t().contiguous(), x.t().contiguous()
        dw = torch.zeros(n_out, k_in, device="cuda")
        ref = torch.zeros_like(dw)
        ops.linear_wgrad(dy, x, ref)
        res = {}
        cases = {
            "TN": lambda: ops.linear_wgrad(dy, x, dw),
            "B^T": lambda: ops.gemm(dy, xT, False, True, n_out, k_in, M, dw, ops.EPI_ACCUM),
            "A^T": lambda: ops.gemm(dyT, x, True, False, n_out, k_in, M, dw, ops.EPI_ACCUM),
            "NT": lambda: ops.gemm(dyT, xT, True, True, n_out, k_in, M, dw, ops.EPI_ACCUM),
        }
        for k, fn in cases.items():
            dw.zero_()
            fn()
            err = ((dw - ref).abs().max() / ref.abs().max()).item()
            us = min(t(fn, iters) for _ in range(2))
            res[k] = (us, err)
        fl = 2.0 * M * n_out * k_in
        print(f"{name:5s} " + "  ".join(f"{k} {us:7.1f} us {fl / us / 1e6:6.0f} TF (err {e:.1e})"
                                        for k, (us, e) in res.items()), flush=True)


if __name__ == "__main__":
    main()
