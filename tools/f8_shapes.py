"""Time the forward GEMMs of the bf16f8 knob (VITMI_BF16F8 operand rows) and their bf16 twins on
the ViT-B/16 bs=256 shapes, in isolation (HIP events, 20 launches each), with the library VITMI_LIB
points at.  usage: python tools/f8_shapes.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402

M, D, F = 256 * 197, 768, 3072
BF = torch.bfloat16


def timed(fn, iters=20):
    for _ in range(5):
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
    r = lambda *s: (torch.rand(*s, device="cuda", generator=g) * 2 - 1)  # noqa: E731
    x, h = r(M, D), r(M, F)
    w1, w2, wo = r(F, D) * 0.05, r(D, F) * 0.05, r(D, D) * 0.05
    b1, b2, bo = torch.zeros(F, device="cuda"), torch.zeros(D, device="cuda"), torch.zeros(D, device="cuda")
    res = torch.rand(M, D, device="cuda")
    x8, _ = ops.split_bf16f8(x, 0)
    h8, _ = ops.split_bf16f8(h, 0)
    w18, _ = ops.split_bf16f8(w1, 1)
    w28, _ = ops.split_bf16f8(w2, 1)
    wo8, _ = ops.split_bf16f8(wo, 1)
    xb, hb, w1b, w2b, wob = x.to(BF), h.to(BF), w1.to(BF), w2.to(BF), wo.to(BF)
    cases = [
        ("proj f8 +res", 2 * M * D * D, lambda: ops.linear_fwd(x8, wo8, bo, torch.float32, ops.EPI_RESIDUAL, res, f8=True)),
        ("proj bf16 +res", 2 * M * D * D, lambda: ops.linear_fwd(xb, wob, bo, torch.float32, ops.EPI_RESIDUAL, res)),
        ("fc1 f8 +GELU split", 2 * M * F * D, lambda: ops.linear_fwd(x8, w18, b1, BF, ops.EPI_BIAS_GELU, aux_tiled=True,
                                                                     split_f8=True, f8=True)),
        ("fc1 f8 store", 2 * M * F * D, lambda: ops.linear_fwd(x8, w18, b1, BF, f8=True)),
        ("fc1 bf16 +GELU", 2 * M * F * D, lambda: ops.linear_fwd(xb, w1b, b1, BF, ops.EPI_BIAS_GELU, aux_tiled=True)),
        ("fc1 bf16 store", 2 * M * F * D, lambda: ops.linear_fwd(xb, w1b, b1, BF)),
        ("fc2 f8 +res", 2 * M * F * D, lambda: ops.linear_fwd(h8, w28, b2, torch.float32, ops.EPI_RESIDUAL, res, f8=True)),
        ("fc2 bf16 +res", 2 * M * F * D, lambda: ops.linear_fwd(hb, w2b, b2, torch.float32, ops.EPI_RESIDUAL, res)),
    ]
    for name, fl, fn in cases:
        us = timed(fn)
        print(f"{name:<24} {us:8.1f} us  {fl / us / 1e6:7.1f} TF (product)", flush=True)


if __name__ == "__main__":
    main()
