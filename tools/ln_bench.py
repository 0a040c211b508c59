"""Time LayerNorm fwd/bwd at the ViT-B/16 bs=256 shape (M = 50432 rows, D = 768) with the
operands of the block backward (bf16 dy, fp32 residual gradient, bf16 copy of dx)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402

M, D = 256 * 197, 768
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(M, D, device="cuda", generator=g)
w = torch.rand(D, device="cuda", generator=g) + 0.5
b = torch.randn(D, device="cuda", generator=g) * 0.1
dy = torch.randn(M, D, device="cuda", generator=g).to(torch.bfloat16)
dres = torch.randn(M, D, device="cuda", generator=g)
dw, db, ds = torch.zeros(D, device="cuda"), torch.zeros(D, device="cuda"), torch.zeros(D, device="cuda")
y, mean, rstd = ops.layernorm_fwd(x, w, b, 1e-6, torch.bfloat16)


def t(fn, iters=50):
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


tf = t(lambda: ops.layernorm_fwd(x, w, b, 1e-6, torch.bfloat16))
tb = t(lambda: ops.layernorm_bwd(dy, x, mean, rstd, w, dw, db, dres=dres, lp_dtype=torch.bfloat16, dxsum=ds))
fb, bb = M * D * (4 + 2) + M * 8, M * D * (2 + 4 + 4 + 4 + 2)
print(f"ln fwd {tf:7.1f} us ({fb / tf / 1e3:6.0f} GB/s)   ln bwd {tb:7.1f} us ({bb / tb / 1e3:6.0f} GB/s)", flush=True)

# the fused Adam step over a ViT-B/16-sized arena (86.6 M fp32 parameters, bf16 shadow)
n = 86_567_656
p, gr = torch.randn(n, device="cuda", generator=g), torch.randn(n, device="cuda", generator=g)
m, v = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
sh = torch.empty(n, dtype=torch.bfloat16, device="cuda")
from vitmi._lib import lib  # noqa: E402
ta = t(lambda: lib().vitmi_adam_step(n, ops._p(p), ops._p(gr), ops._p(m), ops._p(v), ops._p(sh), 1e-3, 0.9, 0.999,
                                     1e-7, 1.0, ops._s()), 20)
print(f"adam {ta:7.1f} us ({n * 30 / ta / 1e3:6.0f} GB/s)", flush=True)
