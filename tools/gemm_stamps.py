"""DIAGNOSTIC: per-tile timeline of the persistent GEMM from s_memtime stamps (variant built with
-DVITMI_GEMM_STAMPS, loaded through VITMI_LIB): K-loop and epilogue cycles per tile, per shape.
usage: VITMI_LIB=.../stamps.so python tools/gemm_stamps.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import _lib, ops  # noqa: E402

M, D, F = 256 * 197, 768, 3072
BF = torch.bfloat16


def main():
    lib = _lib.lib()
    lib.vitmi_gemm_set_stamps.argtypes = [ctypes.c_void_p]
    buf = torch.zeros(256 * 16 * 2 * 8, dtype=torch.int64, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s: (torch.rand(*s, device="cuda", generator=g) * 2 - 1).to(BF)  # noqa: E731
    x, h = r(M, D), r(M, F)
    w1, w2, wq = r(F, D) * 0.05, r(D, F) * 0.05, r(3 * D, D) * 0.05
    b1, b2, bq = torch.zeros(F, device="cuda"), torch.zeros(D, device="cuda"), torch.zeros(3 * D, device="cuda")
    res = torch.rand(M, D, device="cuda")
    gy = r(M, D)
    _, aux = ops.linear_fwd(x, w1, b1, BF, ops.EPI_BIAS_GELU)
    dw = torch.zeros(F, D, device="cuda")
    # the bf16f8 knob's operand rows (VITMI_BF16F8)
    x8, _ = ops.split_bf16f8(x.float(), 0)
    w18, _ = ops.split_bf16f8(w1.float(), 1)
    cases = {
        "fc1+GELU f8": lambda: ops.linear_fwd(x8, w18, b1, BF, ops.EPI_BIAS_GELU, aux_tiled=True, split_f8=True,
                                              f8=True),
        "fc1 store f8": lambda: ops.linear_fwd(x8, w18, b1, BF, f8=True),
        "fc1+GELU tiled": lambda: ops.linear_fwd(x, w1, b1, BF, ops.EPI_BIAS_GELU, aux_tiled=True),
        "fc1+GELU": lambda: ops.linear_fwd(x, w1, b1, BF, ops.EPI_BIAS_GELU),
        "fc1 store": lambda: ops.linear_fwd(x, w1, b1, BF),
        "qkv store": lambda: ops.linear_fwd(x, wq, bq, BF),
        "fc2+resid": lambda: ops.linear_fwd(h, w2, b2, torch.float32, ops.EPI_RESIDUAL, res),
        "DGELU": lambda: ops.linear_dgrad(gy, w2, BF, ops.EPI_DGELU, aux=aux),
        "fc1 dgrad": lambda: ops.linear_dgrad(h, w1, BF),
        "fc1 wgrad": lambda: ops.linear_wgrad(h, x, dw),
    }
    import time
    for name, fn in cases.items():
        # >= 2 s of back-to-back launches first, so the stamped launch runs at the clock the chip
        # holds under this load (DVFS)
        t_end = time.time() + 2.0
        while time.time() < t_end:
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
        lib.vitmi_gemm_set_stamps(buf.data_ptr())
        buf.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        lib.vitmi_gemm_set_stamps(None)
        us = e0.elapsed_time(e1) * 1e3
        st = buf.view(256, 16, 2, 8).cpu()
        valid = st[..., 2] > 0
        t0 = st[..., 0][valid].min().item()
        kl = (st[..., 1] - st[..., 0])[valid].double()
        ep = (st[..., 2] - st[..., 1])[valid].double()
        # gap: next tile's K-loop start minus this tile's epilogue end (same block, same wave)
        nxt = st[:, 1:, :, 0] - st[:, :-1, :, 2]
        gv = nxt[(st[:, 1:, :, 0] > 0) & valid[:, :-1]].double()
        end = (st[..., 2][valid].max().item() - t0)
        starts = st[:, 0, :, 0][st[:, 0, :, 0] > 0].double() - t0
        iters = valid[:, :, 0].sum(1).double()
        # per-iteration means of the K-loop (cold first tile vs later tiles) and per-XCD (block % 8)
        per_it = [(st[:, i, :, 1] - st[:, i, :, 0])[valid[:, i]].double().mean().item() for i in range(int(iters.max()))]
        per_x = [(st[x::8, :, :, 1] - st[x::8, :, :, 0])[valid[x::8]].double().mean().item() for x in range(8)]
        w0 = (st[:, :, 0, 1] - st[:, :, 0, 0])[valid[:, :, 0]].double().mean().item()
        w4 = (st[:, :, 1, 1] - st[:, :, 1, 0])[valid[:, :, 1]].double().mean().item()
        # in-kernel clock: s_memtime cycles per s_memrealtime tick (100 MHz) over each K-loop
        kv = valid & (st[..., 4] > st[..., 3])
        dcy = (st[..., 1] - st[..., 0])[kv].double()
        drt = (st[..., 4] - st[..., 3])[kv].double()
        clk = (dcy / drt * 0.1).median().item() if dcy.numel() else float("nan")   # GHz
        print(f"   in-kernel clock {clk:.2f} GHz (median over {dcy.numel()} K-loops)")
        print(f"   per-iter kloop: {' '.join(f'{v:6.0f}' for v in per_it)}")
        print(f"   per-XCD  kloop: {' '.join(f'{v:6.0f}' for v in per_x)}   wave0 {w0:6.0f} wave4 {w4:6.0f}")
        print(f"{name:10s} {us:7.1f} us | tiles/block {iters.min():.0f}-{iters.max():.0f} | cycles: kloop "
              f"{kl.mean():7.0f} (min {kl.min():6.0f} max {kl.max():6.0f}) epi {ep.mean():6.0f} (max {ep.max():6.0f}) "
              f"gap {gv.mean() if gv.numel() else 0:5.0f}",
              flush=True)


if __name__ == "__main__":
    main()
