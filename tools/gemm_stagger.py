"""EXPERIMENT: does desynchronising the persistent GEMM's blocks (delayed starts) shorten the
epilogue-heavy ViT GEMMs?  usage: python tools/gemm_stagger.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import _lib, ops  # noqa: E402

M, D, F = 256 * 197, 768, 3072
BF = torch.bfloat16


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
    lib = _lib.lib()
    lib.vitmi_gemm_experiment.argtypes = [ctypes.c_int, ctypes.c_int]
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s: (torch.rand(*s, device="cuda", generator=g) * 2 - 1).to(BF)  # noqa: E731
    x, h = r(M, D), r(M, F)
    w1, w2, wq = r(F, D) * 0.05, r(D, F) * 0.05, r(3 * D, D) * 0.05
    b1, b2, bq = torch.zeros(F, device="cuda"), torch.zeros(D, device="cuda"), torch.zeros(3 * D, device="cuda")
    res = torch.rand(M, D, device="cuda")
    gy = r(M, D)
    _, gelu_aux = ops.linear_fwd(x, w1, b1, BF, ops.EPI_BIAS_GELU)
    cases = {
        "fc1+GELU": lambda: ops.linear_fwd(x, w1, b1, BF, ops.EPI_BIAS_GELU),
        "fc1 store": lambda: ops.linear_fwd(x, w1, b1, BF),
        "qkv store": lambda: ops.linear_fwd(x, wq, bq, BF),
        "fc2+resid": lambda: ops.linear_fwd(h, w2, b2, torch.float32, ops.EPI_RESIDUAL, res),
        "fc2 dgrad DGELU": lambda: ops.linear_dgrad(gy, w2, BF, ops.EPI_DGELU, aux=gelu_aux),
        "fc1 dgrad": lambda: ops.linear_dgrad(h, w1, BF),
    }
    settings = [(0, 0), (1, 0), (2, 0), (3, 0), (4, 1), (8, 1), (2, 2), (4, 2)]
    print("case".ljust(18) + "".join(f"{a}/{m}".rjust(9) for a, m in settings))
    for name, fn in cases.items():
        row = []
        for a, m in settings:
            lib.vitmi_gemm_experiment(a, m)
            row.append(t(fn))
        lib.vitmi_gemm_experiment(0, 0)
        print(name.ljust(18) + "".join(f"{v:9.1f}" for v in row), flush=True)


if __name__ == "__main__":
    main()
