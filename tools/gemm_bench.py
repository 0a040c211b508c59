"""Time the ViT-B/16 bs=256 GEMM shapes through libvitmi (and torch/hipBLASLt as a
comparator).  usage: python tools/gemm_bench.py [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402

M, D, F = 256 * 197, 768, 3072
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
    return e0.elapsed_time(e1) / iters


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s: (torch.rand(*s, device="cuda", generator=g) * 2 - 1).to(BF)  # noqa: E731
    x, h = r(M, D), r(M, F)
    w1, w2, wq, wo = r(F, D) * 0.05, r(D, F) * 0.05, r(3 * D, D) * 0.05, r(D, D) * 0.05
    b1, b2, bq = torch.zeros(F, device="cuda"), torch.zeros(D, device="cuda"), torch.zeros(3 * D, device="cuda")
    res = torch.rand(M, D, device="cuda")
    gq = r(M, 3 * D)
    dw = torch.zeros(F, D, device="cuda")
    a8, b8 = r(8192, 8192), r(8192, 8192)
    c8 = torch.empty(8192, 8192, device="cuda", dtype=BF)
    cases = {
        "square bf16    [8192^3]": (lambda: ops.linear_fwd(a8, b8, None, BF), 2 * 8192 ** 3),
        "torch square   [8192^3]": (lambda: torch.mm(a8, b8.t()), 2 * 8192 ** 3),
        "square NN      [8192^3]": (lambda: ops.gemm(a8, b8, True, False, 8192, 8192, 8192, c8), 2 * 8192 ** 3),
        "square TN      [8192^3]": (lambda: ops.gemm(a8, b8, False, False, 8192, 8192, 8192, c8), 2 * 8192 ** 3),
        "fc1 fwd store  [M,3072,768]": (lambda: ops.linear_fwd(x, w1, b1, BF), 2 * M * F * D),
        "fc1 fwd f32out [M,3072,768]": (lambda: ops.linear_fwd(x, w1, b1, torch.float32), 2 * M * F * D),
        "fc1 fwd +GELU  [M,3072,768]": (lambda: ops.linear_fwd(x, w1, b1, BF, ops.EPI_BIAS_GELU, aux_tiled=True),
                                        2 * M * F * D),
        "fc1 +GELU rowmajor gelu'": (lambda: ops.linear_fwd(x, w1, b1, BF, ops.EPI_BIAS_GELU), 2 * M * F * D),
        "qkv fwd store  [M,2304,768]": (lambda: ops.linear_fwd(x, wq, bq, BF), 2 * M * 3 * D * D),
        "fc2 fwd +resid [M,768,3072]": (lambda: ops.linear_fwd(h, w2, b2, torch.float32, ops.EPI_RESIDUAL, res),
                                        2 * M * F * D),
        "proj fwd +res  [M,768,768]": (lambda: ops.linear_fwd(x, wo, b2, torch.float32, ops.EPI_RESIDUAL, res),
                                       2 * M * D * D),
        # (M x 3072 is a whole number of 256 x 256 tiles: h doubles as a tile-native gelu' buffer)
        "fc2 dgrad dGELU[M,3072,768]": (lambda: ops.linear_dgrad(x, w2, BF, ops.EPI_DGELU, aux=h, aux_tiled=True),
                                        2 * M * F * D),
        "fc2 dGELU rowmajor gelu'": (lambda: ops.linear_dgrad(x, w2, BF, ops.EPI_DGELU, aux=h), 2 * M * F * D),
        "fc1 dgrad f32  [M,768,3072]": (lambda: ops.linear_dgrad(h, w1, torch.float32), 2 * M * F * D),
        "fc1 dgrad bf16 [M,768,3072]": (lambda: ops.linear_dgrad(h, w1, BF), 2 * M * F * D),
        "qkv dgrad bf16 [M,768,2304]": (lambda: ops.linear_dgrad(gq, wq, BF), 2 * M * 3 * D * D),
        "proj dgrad bf16[M,768,768]": (lambda: ops.linear_dgrad(x, wo, BF), 2 * M * D * D),
        "qkv dgrad f32  [M,768,2304]": (lambda: ops.linear_dgrad(gq, wq, torch.float32), 2 * M * 3 * D * D),
        "fc1 wgrad      [3072,768]/M": (lambda: ops.linear_wgrad(h, x, dw), 2 * M * F * D),
        "torch mm       [M,3072,768]": (lambda: torch.mm(x, w1.t()), 2 * M * F * D),
    }
    only = os.environ.get("GEMM_BENCH_ONLY")
    for name, (fn, flops) in cases.items():
        if only and not any(k in name for k in only.split(",")):
            continue
        ms = t(fn, iters)
        print(f"{name}: {ms * 1e3:8.1f} us  {flops / ms / 1e9:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
