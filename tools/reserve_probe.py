"""gemm256 time vs vitmi_gemm_set_reserved_cus (no side traffic): the ViT-B backward GEMMs and
qkv fwd with 0 / 8 / 16 / 32 CUs left out of the persistent grid.  usage: python tools/reserve_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import _lib, ops  # noqa: E402

BF = torch.bfloat16
M, D, F = 256 * 197, 768, 3072


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


g = torch.Generator(device="cuda").manual_seed(0)
r = lambda *s: (torch.rand(*s, device="cuda", generator=g) * 2 - 1).to(BF)  # noqa: E731
x, h, wq, w1 = r(M, D), r(M, F), r(3 * D, D) * 0.05, r(F, D) * 0.05
bq = torch.zeros(3 * D, device="cuda")
dw = torch.zeros(F, D, device="cuda")
cases = {"qkv fwd": lambda: ops.linear_fwd(x, wq, bq, BF),
         "fc1 dgrad": lambda: ops.linear_dgrad(h, w1, BF),
         "fc1 wgrad": lambda: ops.linear_wgrad(h, x, dw)}
for rnd in range(2):
    for res in (0, 8, 16, 32):
        _lib.lib().vitmi_gemm_set_reserved_cus(res)
        print(f"round {rnd} reserve {res:2d}: " + "  ".join(f"{k} {t(fn):7.1f} us" for k, fn in cases.items()),
              flush=True)
_lib.lib().vitmi_gemm_set_reserved_cus(0)
