"""DIAGNOSTIC: per-workgroup timeline of the whole-sequence attention kernels (fwd, dQ) at the C3
shape from s_memrealtime stamps (variant built with -DVITMI_ATTN_STAMPS, loaded through VITMI_LIB):
phase durations (operand load, loop, store) and, per CU, how the resident workgroups' phases
overlap.  usage: VITMI_LIB=.../astamps.so python tools/attn_stamps.py [B N H]"""
import ctypes
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import _lib, ops  # noqa: E402

TICK_NS = 10.0   # s_memrealtime: 100 MHz


def analyse(name, st):
    st = st[st[:, 0] != 0]
    t0 = st[:, 0].min()
    s = (st[:, :4] - t0).astype(np.float64) * TICK_NS / 1000.0   # us
    hw, xcc = st[:, 4], st[:, 5]
    cu = (xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15)
    span = s[:, 3].max()
    load, loop, store = s[:, 1] - s[:, 0], s[:, 2] - s[:, 1], s[:, 3] - s[:, 2]
    print(f"{name}: {len(st)} workgroups on {len(np.unique(cu))} CUs, span {span:.1f} us; per workgroup "
          f"load {load.mean():.2f} (p10 {np.percentile(load, 10):.2f} p90 {np.percentile(load, 90):.2f}) "
          f"loop {loop.mean():.2f} (p10 {np.percentile(loop, 10):.2f} p90 {np.percentile(loop, 90):.2f}) "
          f"store-issue {store.mean():.2f} us; life {(s[:, 3] - s[:, 0]).mean():.2f} us")
    # per CU: time with n workgroups resident, and with k of them in their loop phase
    grid = np.linspace(0, span, 2000)
    dt = grid[1] - grid[0]
    res = defaultdict(float)
    inloop = defaultdict(float)
    byc = defaultdict(list)
    for i, c in enumerate(cu):
        byc[c].append(i)
    for c, idx in byc.items():
        a = s[idx]
        nres = ((grid[:, None] >= a[None, :, 0]) & (grid[:, None] < a[None, :, 3])).sum(1)
        nl = ((grid[:, None] >= a[None, :, 1]) & (grid[:, None] < a[None, :, 2])).sum(1)
        for n in range(4):
            res[n] += (nres == n).sum() * dt
            inloop[n] += (nl == n).sum() * dt
    tot = sum(res.values())
    print("  CU time with n workgroups resident: " + "  ".join(f"{n}: {res[n] / tot:.2f}" for n in range(4)))
    print("  CU time with n workgroups in their loop: " + "  ".join(f"{n}: {inloop[n] / tot:.2f}" for n in range(4)))
    first = np.sort(s[:, 0])
    print(f"  start times: first 512 within {first[511] - first[0]:.2f} us; per-CU workgroups "
          f"{np.mean([len(v) for v in byc.values()]):.1f}")


def main():
    B, N, H = (int(a) for a in (sys.argv[1:] + ["256", "197", "12"][len(sys.argv) - 1:]))
    D = 64 * H
    lib = _lib.lib()
    lib.vitmi_attn_set_stamps.argtypes = [ctypes.c_void_p]
    buf = torch.zeros(2 * 65536 * 8, dtype=torch.int64, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = (torch.randn(B * N, 3 * D, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    do = torch.randn(B * N, D, device="cuda", generator=g).to(torch.bfloat16)
    for _ in range(3):
        o, lse = ops.attention_fwd(qkv, B, N, H, 0.125)
        ops.attention_bwd(qkv, o, do, lse, B, N, H, 0.125)
    torch.cuda.synchronize()
    lib.vitmi_attn_set_stamps(buf.data_ptr())
    o, lse = ops.attention_fwd(qkv, B, N, H, 0.125)
    ops.attention_bwd(qkv, o, do, lse, B, N, H, 0.125)
    torch.cuda.synchronize()
    lib.vitmi_attn_set_stamps(None)
    st = buf.view(2, 65536, 8).cpu().numpy().view(np.uint64).astype(np.int64)
    analyse("fwd seq", st[0])
    analyse("dQ seq", st[1])


if __name__ == "__main__":
    main()
