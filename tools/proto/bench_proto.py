"""A/B of the 2-blocks-per-CU GEMM prototype (tools/proto/gemm2b.hip -> libproto.so) against
gemm256 (libvitmi) on the ViT-B NT shapes and 8192^3, interleaved rounds in one process,
random [-1, 1) bf16 operands.  usage: python tools/proto/bench_proto.py [iters]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "tools", "proto", "libproto.so"))
P, I = ctypes.c_void_p, ctypes.c_int
lib.proto_gemm_nt.argtypes = [I, I, I, I, P, P, P, P, P, P]
BF = torch.bfloat16


def proto(ns, a, b, bias, gelu=False):
    M, K = a.shape
    N = b.shape[0]
    c = torch.empty(M, N, dtype=BF, device=a.device)
    u = torch.empty(M, N, dtype=BF, device=a.device) if gelu else None
    rc = lib.proto_gemm_nt(ns, M, N, K, a.data_ptr(), b.data_ptr(), c.data_ptr(), u.data_ptr() if gelu else None,
                           bias.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert rc == 0, rc
    return (c, u) if gelu else c


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
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s: (torch.rand(*s, device="cuda", generator=g) * 2 - 1).to(BF)  # noqa: E731
    # correctness
    a, b = r(512, 256), r(384, 256)
    bias = torch.randn(384, device="cuda")
    ref = a.float() @ b.float().t() + bias
    for ns in (2, 3, 4):
        err = (proto(ns, a, b, bias).float() - ref).abs().max().item()
        print(f"check nstage {ns}: max abs err {err:.3e}", flush=True)
        assert err < 0.1
    M = 256 * 197
    shapes = {"fc1 [M,3072,768]": (M, 3072, 768), "qkv [M,2304,768]": (M, 2304, 768),
              "proj [M,768,768]": (M, 768, 768), "fc2 [M,768,3072]": (M, 768, 3072), "sq [8192^3]": (8192, 8192, 8192)}
    for name, (m, n, k) in shapes.items():
        x, w = r(m, k), r(n, k) * 0.05
        bias = torch.zeros(n, device="cuda")
        c256 = ops.linear_fwd(x, w, bias, BF)
        cp = proto(3, x, w, bias)
        diff = (c256.float() - cp.float()).abs().max().item()
        res = {"gemm256": [], "p2": [], "p3": [], "p4": []}
        for _ in range(2):
            res["gemm256"].append(t(lambda: ops.linear_fwd(x, w, bias, BF), iters))
            for ns in (2, 3, 4):
                res[f"p{ns}"].append(t(lambda: proto(ns, x, w, bias), iters))
        fl = 2.0 * m * n * k
        print(f"{name}: diff {diff:.2e}  " + "  ".join(f"{kk} {min(v):7.1f} us {fl / min(v) / 1e6:6.0f} TF"
                                                       for kk, v in res.items()), flush=True)
        if name.startswith("fc1"):
            a256, u256 = ops.linear_fwd(x, w, bias, BF, ops.EPI_BIAS_GELU)
            ap, up = proto(3, x, w, bias, True)
            d1 = (a256.float() - ap.float()).abs().max().item()
            d2 = (u256.float() - up.float()).abs().max().item()
            rg = {"gemm256": [], "p2": [], "p3": [], "p4": []}
            for _ in range(2):
                rg["gemm256"].append(t(lambda: ops.linear_fwd(x, w, bias, BF, ops.EPI_BIAS_GELU), iters))
                for ns in (2, 3, 4):
                    rg[f"p{ns}"].append(t(lambda: proto(ns, x, w, bias, True), iters))
            print(f"fc1+GELU: diff {d1:.2e}/{d2:.2e}  " + "  ".join(
                f"{kk} {min(v):7.1f} us {fl / min(v) / 1e6:6.0f} TF" for kk, v in rg.items()), flush=True)
        del x, w


if __name__ == "__main__":
    main()
