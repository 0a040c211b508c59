"""DIAGNOSTIC: per-pair phase timeline of the single-pass attention backward (attn_bwd_fused_seq_bf16)
at the C3 shape from s_memrealtime stamps (variant built with -DVITMI_ATTN_STAMPS, loaded through
VITMI_LIB).  usage: VITMI_LIB=.../astamps.so python tools/attn_fused_stamps.py [B N H]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import _lib, ops  # noqa: E402

TICK_NS = 10.0   # s_memrealtime: 100 MHz


def main():
    B, N, H = (int(a) for a in (sys.argv[1:] + ["256", "197", "12"][len(sys.argv) - 1:]))
    D = 64 * H
    lib = _lib.lib()
    lib.vitmi_attn_set_stamps.argtypes = [ctypes.c_void_p]
    buf = torch.zeros(3 * 65536 * 8, dtype=torch.int64, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = (torch.randn(B * N, 3 * D, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    do = torch.randn(B * N, D, device="cuda", generator=g).to(torch.bfloat16)
    o, lse = ops.attention_fwd(qkv, B, N, H, 0.125)
    for _ in range(20):
        ops.attention_bwd(qkv, o, do, lse, B, N, H, 0.125)
    torch.cuda.synchronize()
    lib.vitmi_attn_set_stamps(buf.data_ptr())
    ops.attention_bwd(qkv, o, do, lse, B, N, H, 0.125)
    torch.cuda.synchronize()
    lib.vitmi_attn_set_stamps(None)
    st = buf.view(3, 65536, 8)[2, :B * H].cpu().numpy()
    st = st[st[:, 0] != 0]
    t0 = st[:, 0].min()
    s = (st[:, :5] - t0).astype(np.float64) * TICK_NS / 1000.0
    d = np.diff(s, axis=1)
    names = ["delta", "phase 1", "K image + phase 2", "epilogue"]
    print(f"{len(st)} pairs, span {s[:, 4].max():.1f} us; per pair (us, mean / p10 / p90):")
    for i, nm in enumerate(names):
        print(f"  {nm:<18} {d[:, i].mean():6.2f} {np.percentile(d[:, i], 10):6.2f} {np.percentile(d[:, i], 90):6.2f}")
    # gap between a CU's pairs: end of one epilogue to the next pair's start (its loads' wait)
    hw, xcc = st[:, 6], st[:, 7]
    cu = (xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15)
    gaps = []
    for c in np.unique(cu):
        a = s[cu == c]
        a = a[np.argsort(a[:, 0])]
        gaps += list(a[1:, 0] - a[:-1, 4])
    if gaps:
        print(f"  wait for the next pair's loads {np.mean(gaps):6.2f} {np.percentile(gaps, 10):6.2f} {np.percentile(gaps, 90):6.2f}")
    print(f"  first pair start spread {np.sort(s[:, 0])[255] - s[:, 0].min():.2f} us (first 256 pairs)")


if __name__ == "__main__":
    main()
