"""CU contention of the overlapped gradient all-reduce on ONE GPU (verdict r02 item 3).

The ViT-B/16 bs-256 step runs with a GradReducer whose communicator is replaced by side-stream
traffic shaped like RCCL's ring all-reduce of each bucket on 8 ranks: per 64 MiB fp32 bucket
every rank reads and writes about 2 x 7/8 x 64 MiB, emulated by a copy out and an add back
(3 bucket-sized passes over HBM) on the reducer's side stream, launched from the same backward
hooks after the same hipEvent.  The persistent GEMM holds one block per CU, so those side
kernels queue until blocks drain unless `reserve_cus` CUs are kept free.  For each reserve value
this prints the step time and, per bucket, the side stream's wall time from the moment its
event gate opened to the end of its traffic (HIP events on the side stream).

With --emu B the side traffic is tools/proto/rccl_emu.hip instead: B persistent "channel"
blocks that must all be running before any streams (RCCL's co-residency requirement), so a
channel block that finds every CU held by the persistent GEMM delays the whole collective.

usage: python tools/contention.py [steps] [--emu B] [reserve values...]   -> JSON on stdout
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import dp, optim  # noqa: E402
from vitmi.config import config_c3  # noqa: E402
from vitmi.modules import VisionTransformer, cross_entropy  # noqa: E402


class RcclShapedTraffic:
    """Stands in for VitmiComm: allreduce_async = gate on the ready event, then 3 bucket-sized
    HBM passes on the side stream, bracketed by timing events."""

    world = 8

    def __init__(self, emu_blocks=0):
        self.spans = []
        self._tmp = None
        self.emu_blocks = emu_blocks
        self._gen = 0
        if emu_blocks:
            self._lib = ctypes.CDLL(os.path.join(ROOT, "tools", "proto", "librccl_emu.so"))
            self._lib.emu_allreduce_launch.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                                                       ctypes.c_uint, ctypes.c_void_p]
            self._counter = torch.zeros(1, dtype=torch.int32, device="cuda")

    def allreduce_async(self, buf, side, ready=None, op=None):
        if self.emu_blocks:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if ready is not None:
                side.wait_event(ready)
            e0.record(side)
            rc = self._lib.emu_allreduce_launch(buf.data_ptr(), buf.numel() // 4 * 4, self.emu_blocks,
                                                self._counter.data_ptr(), self._gen, side.cuda_stream)
            assert rc == 0, rc
            self._gen += 1
            e1.record(side)
            self.spans.append((e0, e1))
            return
        if self._tmp is None or self._tmp.numel() < buf.numel():
            self._tmp = torch.empty(buf.numel(), dtype=buf.dtype, device=buf.device)
        tmp = self._tmp[:buf.numel()]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if ready is not None:
            side.wait_event(ready)
        with torch.cuda.stream(side):
            e0.record(side)
            tmp.copy_(buf)
            buf.add_(tmp, alpha=0.0)         # values unchanged; the bytes move
            e1.record(side)
        self.spans.append((e0, e1))

    def check(self):
        pass

    @property
    def live(self):
        return True

    def destroy(self, abort=False):
        pass


def run(steps, reserve, traffic, emu=0):
    cfg = config_c3()
    dev = torch.device("cuda", 0)
    model = VisionTransformer(cfg).to(dev)
    model.reset_parameters(seed=0)
    comm = RcclShapedTraffic(emu) if traffic else None
    red = dp.GradReducer(model.arena().grad, 64.0, comm=comm, reserve_cus=reserve, timeout_s=0) if traffic else None
    if red is not None:
        arena = model.arena()

        def end_of(ps):
            return max(arena.offsets[id(p)] + p.numel() for p in ps)
        head_end = end_of(list(model.head.parameters()) + list(model.norm.parameters()))
        object.__setattr__(model, "_head_ready_hook", lambda: red.mark_ready(head_end))
        for blk in model.blocks:
            e = end_of(list(blk.parameters()))
            object.__setattr__(blk, "_grad_ready_hook", lambda _m, e=e: red.mark_ready(e))
        object.__setattr__(model.patch_embed, "_grad_ready_hook", lambda _m: red.mark_ready(arena.numel))
    opt = optim.Adam(model, learning_rate=1e-3)
    arena = model.arena()
    g = torch.Generator(device=dev).manual_seed(1234)
    img = torch.rand(256, 3, 224, 224, device=dev, generator=g)
    tgt = torch.randint(0, 2, (256,), device=dev, generator=g)

    def step():
        arena.grad.zero_()
        if red is not None:
            red.start()
        loss = cross_entropy(model(img), tgt)
        loss.backward()
        if red is not None:
            red.finish()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    if comm is not None:
        comm.spans.clear()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        step()
    e1.record()
    torch.cuda.synchronize()
    out = {"reserve_cus": reserve, "traffic": ("emu%d" % emu if emu else "torch") if traffic else None,
           "ms_per_step": round(e0.elapsed_time(e1) / steps, 3)}
    if comm is not None:
        sp = [a.elapsed_time(b) for a, b in comm.spans]
        nb = len(sp) // steps
        per = [sp[i::nb] for i in range(nb)]
        out["buckets_per_step"] = nb
        out["side_ms_per_bucket"] = [round(sum(p) / len(p), 3) for p in per]
        out["side_ms_per_step"] = round(sum(sp) / steps, 3)
    del model, opt, red
    torch.cuda.empty_cache()
    return out


def main():
    args = sys.argv[1:]
    steps = int(args.pop(0)) if args else 10
    emu = 0
    if args and args[0] == "--emu":
        emu = int(args[1])
        args = args[2:]
    reserves = [int(v) for v in args] or [0, 8, 16, 32]
    rows = [run(steps, 0, False)]
    print(json.dumps(rows[-1]), flush=True)
    for rnd in range(2):                                   # two alternating rounds (rule 24)
        for r in reserves:
            rows.append(dict(run(steps, r, True, emu), round=rnd))
            print(json.dumps(rows[-1]), flush=True)
    print(json.dumps({"rows": rows}))


if __name__ == "__main__":
    main()
