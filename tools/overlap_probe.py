"""Can a memory-bound LayerNorm backward run UNDER a compute-bound weight-gradient GEMM?

ViT-B/16 bs 256 shapes (M = 50,432 tokens): the fc1 + fc2 weight gradients (the two TN GEMMs
the LN2 backward does not depend on, vitmi/modules.py _BlockFn.backward) and one LayerNorm
backward (D = 768, residual gradient + bf16 copy).  Times, per repetition:
  serial     both GEMMs then the LN backward on one stream (what the step does today);
  reserve    the GEMMs' persistent grid leaves R CUs free (vitmi_gemm_set_reserved_cus) and the
             LN backward runs on a second stream;
  cumask     as reserve, with CU-masked streams (hipExtStreamCreateWithCUMask): the LN stream
             gets R CUs, the GEMM stream the others.
usage: python tools/overlap_probe.py [R ...]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402
from vitmi._lib import lib  # noqa: E402

BF = torch.bfloat16


def hip():
    for name in ("libamdhip64.so.7", "libamdhip64.so"):
        try:
            return ctypes.CDLL(name, mode=os.RTLD_NOLOAD | os.RTLD_GLOBAL)
        except OSError:
            continue
    return ctypes.CDLL("libamdhip64.so")


def masked_stream(bits):
    """A HIP stream restricted to the CUs whose bits are set (list of CU indices)."""
    h = hip()
    n = 256
    words = (ctypes.c_uint32 * (n // 32))()
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    s = ctypes.c_void_p()
    rc = h.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(n // 32), words)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value)


def main():
    rs = [int(a) for a in sys.argv[1:]] or [16, 32, 64]
    g = torch.Generator(device="cuda").manual_seed(0)
    M, D, F = 50432, 768, 3072
    du = (torch.randn(M, F, device="cuda", generator=g) * 0.1).to(BF)
    h2 = torch.randn(M, D, device="cuda", generator=g).to(BF)
    g2 = (torch.randn(M, D, device="cuda", generator=g) * 0.1).to(BF)
    act = torch.randn(M, F, device="cuda", generator=g).to(BF)
    dw1 = torch.zeros(F, D, device="cuda")
    dw2 = torch.zeros(D, F, device="cuda")
    x = torch.randn(M, D, device="cuda", generator=g)
    w = torch.ones(D, device="cuda")
    _, mean, rstd = ops.layernorm_fwd(x, w, torch.zeros(D, device="cuda"), 1e-6, BF)
    dh = (torch.randn(M, D, device="cuda", generator=g) * 0.1).to(BF)
    dres = torch.randn(M, D, device="cuda", generator=g)
    dgm, dbt = torch.zeros(D, device="cuda"), torch.zeros(D, device="cuda")

    def gemms():
        ops.linear_wgrad(du, h2, dw1)
        ops.linear_wgrad(g2, act, dw2)

    def ln():
        ops.layernorm_bwd(dh, x, mean, rstd, w, dgm, dbt, dres=dres, lp_dtype=BF)

    def timed(fn, reps=10):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    t_g = timed(gemms)
    t_l = timed(ln)
    print(f"gemms alone {t_g:7.1f} us   ln alone {t_l:6.1f} us   serial sum {t_g + t_l:7.1f} us", flush=True)
    main_s = torch.cuda.current_stream()
    for R in rs:
        side = torch.cuda.Stream()

        def both_reserve():
            ev = torch.cuda.Event()
            ev.record(main_s)
            side.wait_event(ev)
            prev = lib().vitmi_gemm_set_reserved_cus(R)
            gemms()
            lib().vitmi_gemm_set_reserved_cus(prev)
            with torch.cuda.stream(side):
                ln()
            main_s.wait_stream(side)

        t_r = timed(both_reserve)
        ln_cus = [8 * i + j for j in range(R // 8) for i in range(32)] if R % 8 == 0 else list(range(R))
        ln_cus = sorted(set(c for c in ln_cus if c < 256))[:R]
        gm_cus = [c for c in range(256) if c not in set(ln_cus)]
        sg, sl = masked_stream(gm_cus), masked_stream(ln_cus)

        def both_mask():
            ev = torch.cuda.Event()
            ev.record(main_s)
            sg.wait_event(ev)
            sl.wait_event(ev)
            prev = lib().vitmi_gemm_set_reserved_cus(R)
            with torch.cuda.stream(sg):
                gemms()
            lib().vitmi_gemm_set_reserved_cus(prev)
            with torch.cuda.stream(sl):
                ln()
            main_s.wait_stream(sg)
            main_s.wait_stream(sl)

        t_m = timed(both_mask)
        with torch.cuda.stream(sl):
            t_lm = timed(ln)
        with torch.cuda.stream(sg):
            prev = lib().vitmi_gemm_set_reserved_cus(R)
            t_gm = timed(gemms)
            lib().vitmi_gemm_set_reserved_cus(prev)
        print(f"R={R:3d}: reserve+2 streams {t_r:7.1f} us   cu-masked {t_m:7.1f} us   "
              f"(ln on {R} CUs alone {t_lm:6.1f}, gemms on {256 - R} CUs alone {t_gm:7.1f})", flush=True)


if __name__ == "__main__":
    main()
