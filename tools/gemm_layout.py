"""Run one GEMM layout a few times (for rocprofv3 PMC passes).
usage: python tools/gemm_layout.py {NT,NN,TN} [iters] [M N K]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402

mode = sys.argv[1]
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
M, N, K = (int(v) for v in sys.argv[3:6]) if len(sys.argv) > 5 else (8192, 8192, 8192)
g = torch.Generator(device="cuda").manual_seed(0)
ak, bk = {"NT": (True, True), "NN": (True, False), "TN": (False, False)}[mode]
a = (torch.rand(M, K, device="cuda", generator=g) if ak else torch.rand(K, M, device="cuda", generator=g)).to(torch.bfloat16)
b = (torch.rand(N, K, device="cuda", generator=g) if bk else torch.rand(K, N, device="cuda", generator=g)).to(torch.bfloat16)
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(iters):
    ops.gemm(a, b, ak, bk, M, N, K, c)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(iters):
    ops.gemm(a, b, ak, bk, M, N, K, c)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / iters
print(f"{mode} {M}x{N}x{K}: {ms:.3f} ms {2 * M * N * K / ms / 1e9:.0f} TFLOP/s")
