"""Time every GEMM of the ViT-B/16 bs=256 step in isolation (HIP events, 20 launches each) with
the library VITMI_LIB points at (default: the in-tree build).  One line per GEMM: us/launch and
TFLOP/s.  usage: python tools/gemm_shapes.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402

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

    def r(*s, dt=BF, sc=1.0):
        return ((torch.rand(*s, device="cuda", generator=g) * 2 - 1) * sc).to(dt)

    x, h4 = r(M, D), r(M, F)
    dq = r(M, 3 * D)
    wqkv, wo, w1, w2 = r(3 * D, D, sc=0.05), r(D, D, sc=0.05), r(F, D, sc=0.05), r(D, F, sc=0.05)
    bq, bo, b1, b2 = (torch.zeros(n, device="cuda") for n in (3 * D, D, F, D))
    res = torch.rand(M, D, device="cuda")
    gp = r(M, F)
    dw_qkv, dw_1, dw_2, dw_o = (torch.zeros(*w.shape, device="cuda") for w in (wqkv, w1, w2, wo))
    cases = [
        ("qkv fwd  [M x 2304 x 768] +bias", 2 * M * 3 * D * D, lambda: ops.linear_fwd(x, wqkv, bq, BF)),
        ("proj fwd [M x 768 x 768] +res", 2 * M * D * D, lambda: ops.linear_fwd(x, wo, bo, torch.float32, ops.EPI_RESIDUAL, res)),
        ("fc1 fwd  [M x 3072 x 768] +GELU", 2 * M * F * D, lambda: ops.linear_fwd(x, w1, b1, BF, ops.EPI_BIAS_GELU, aux_tiled=True)),
        ("fc2 fwd  [M x 768 x 3072] +res", 2 * M * D * F, lambda: ops.linear_fwd(h4, w2, b2, torch.float32, ops.EPI_RESIDUAL, res)),
        ("fc2 dgrad [M x 3072 x 768] DGELU", 2 * M * F * D, lambda: ops.linear_dgrad(x, w2, BF, ops.EPI_DGELU, gp, aux_tiled=True)),
        ("fc1 dgrad [M x 768 x 3072]", 2 * M * D * F, lambda: ops.linear_dgrad(h4, w1, BF)),
        ("qkv dgrad [M x 768 x 2304]", 2 * M * D * 3 * D, lambda: ops.linear_dgrad(dq, wqkv, BF)),
        ("proj dgrad [M x 768 x 768]", 2 * M * D * D, lambda: ops.linear_dgrad(x, wo, BF)),
        ("fc1 wgrad [3072 x 768 x M]", 2 * M * F * D, lambda: ops.linear_wgrad(h4, x, dw_1)),
        ("fc2 wgrad [768 x 3072 x M]", 2 * M * F * D, lambda: ops.linear_wgrad(x, h4, dw_2)),
        ("qkv wgrad [2304 x 768 x M]", 2 * M * 3 * D * D, lambda: ops.linear_wgrad(dq, x, dw_qkv)),
        ("proj wgrad [768 x 768 x M]", 2 * M * D * D, lambda: ops.linear_wgrad(x, x, dw_o)),
    ]
    tot = 0.0
    for name, fl, fn in cases:
        us = timed(fn)
        tot += us
        print(f"{name:34s} {us:8.1f} us  {fl / us / 1e6:7.1f} TF", flush=True)
    print(f"{'sum (one block: x12 per step)':34s} {tot:8.1f} us")


if __name__ == "__main__":
    main()
