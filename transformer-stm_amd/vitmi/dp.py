"""Data-parallel gradient reduction for the MI355X ViT path.

Replaces the reference's only parallel construct, ``tf.distribute.MirroredStrategy()``
(``old_codes/BayConvT(Par)(Muti).py:16-19``): synchronous data parallelism with a
cross-replica mean of every gradient once per step.  MI355X design:

* one process per GPU (torchrun); ``torch.distributed`` bootstraps the job (rendezvous,
  TCPStore, barriers) and, with ``comm="vitmi"`` (the default on GPUs), the gradient
  exchange itself goes through the library's own RCCL communicator
  (``vitmi_comm_*`` in include/vitmi.h): the 128-byte RCCL id travels through the
  TCPStore, every bucket is all-reduced on a dedicated side HIP stream after a hipEvent
  recorded on the compute stream, and the compute stream waits on the side stream once,
  before the optimizer.  ``comm="torch"`` runs the same buckets through
  ``torch.distributed.all_reduce`` (RCCL via ProcessGroupNCCL on GPUs, gloo on CPU);
* all gradients live in ONE flat fp32 buffer (``ParamArena``) laid out in the order
  the backward finishes them (head, norm, block L-1 ... block 0, patch-embed), so
  fixed-size buckets (default 64 MiB: few, large collectives suit per-link-bound
  xGMI rings) become ready front to back;
* a post-accumulate-grad hook on every parameter (torch's own signal that ``.grad`` is final,
  the one DistributedDataParallel's reducer uses) advances the finished prefix of the arena;
  every bucket wholly inside it is all-reduced at once, overlapping the rest of the backward;
* ``grad_dtype="bf16"`` halves the bytes on the wire (ViT-L: 1.2 GB -> 607 MB per step):
  each bucket is cast to bf16 on the side stream, averaged, and cast back into the fp32
  arena (rounding each gradient to bf16 once, plus RCCL's bf16 partial sums);
* ``reserve_cus``: the persistent GEMM (one 512-thread block per CU, the whole register
  file) leaves that many CUs free while the backward runs, so RCCL's kernels find CUs
  instead of waiting for a GEMM to drain (``vitmi_gemm_set_reserved_cus``).
"""
from __future__ import annotations

import ctypes
import os
import threading
import time
from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

UID_BYTES = 128
_F32, _BF16, _F64 = 0, 1, 2
_DT = {torch.float32: _F32, torch.bfloat16: _BF16, torch.float64: _F64}
REDUCE_SUM, REDUCE_AVG = 0, 1


class VitmiComm:
    """The library's RCCL communicator (one per process, bound to the current HIP device).

    No Python lock is held across a library call: the CommWatchdog thread's abort must be able to
    run while the training thread waits inside an all-reduce (a dead peer), which the abort then
    ends with an error.  The library creates the communicator non-blocking, so its RCCL calls never
    wait on a peer and run serialised with the abort under the library's own lock; a wait is a poll
    that stops once the communicator is released (csrc/comm.cpp).  ``self._lock`` only makes
    ``destroy`` happen once."""

    def __init__(self, rank: int, world: int, uid: bytes):
        if len(uid) != UID_BYTES:
            raise ValueError(f"vitmi comm: the RCCL id must be {UID_BYTES} bytes")
        self.rank, self.world = rank, world
        self._lock = threading.Lock()
        self._uid = ctypes.create_string_buffer(uid, UID_BYTES)
        self._init(rank, world)
        self._live = True

    def _init(self, rank: int, world: int) -> None:
        from ._lib import check, lib
        check(lib().vitmi_comm_init(rank, world, self._uid), "comm_init")

    def _call(self, name: str, *args) -> int:
        from ._lib import lib
        return getattr(lib(), name)(*args)

    @staticmethod
    def unique_id() -> bytes:
        from ._lib import check, lib
        buf = ctypes.create_string_buffer(UID_BYTES)
        check(lib().vitmi_comm_get_unique_id(buf), "comm_get_unique_id")
        return buf.raw

    @classmethod
    def from_store(cls, rank: int, world: int, store=None, key: str = "vitmi_comm_uid") -> "VitmiComm":
        """Rank 0 creates the id and publishes it in the job's TCPStore; the others wait for it."""
        return cls(rank, world, exchange_unique_id(rank, world, store, key))

    def allreduce_async(self, buf: torch.Tensor, side: "torch.cuda.Stream", ready=None, op: int = REDUCE_AVG) -> None:
        from ._lib import check
        assert buf.is_cuda and buf.is_contiguous() and buf.dtype in _DT
        dt = _DT[buf.dtype]
        check(self._call("vitmi_comm_allreduce_async", buf.data_ptr(), buf.numel(), dt, op,
                         side.cuda_stream if side is not None else None,
                         ready.cuda_event if ready is not None else None), "comm_allreduce_async")

    def broadcast(self, buf: torch.Tensor, root: int = 0) -> None:
        from ._lib import check
        dt = _F32 if buf.dtype == torch.float32 else _BF16
        check(self._call("vitmi_comm_broadcast", buf.data_ptr(), buf.numel(), dt, root,
                         torch.cuda.current_stream().cuda_stream), "comm_broadcast")

    def check(self) -> None:
        from ._lib import check
        check(self._call("vitmi_comm_check"), "comm_check")

    def info(self) -> Tuple[int, int]:
        """(rank, world) as the library's communicator holds them (vitmi_comm_info)."""
        from ._lib import check
        r, w = ctypes.c_int(-1), ctypes.c_int(0)
        check(self._call("vitmi_comm_info", ctypes.byref(r), ctypes.byref(w)), "comm_info")
        return r.value, w.value

    @property
    def live(self) -> bool:
        return self._live

    @staticmethod
    def library() -> str:
        """File name of the RCCL the comm leg bound (the copy torch mapped, not a second one)."""
        from ._lib import check, lib
        buf = ctypes.create_string_buffer(4096)
        check(lib().vitmi_comm_library(buf, 4096), "comm_library")
        return buf.value.decode()

    def destroy(self, abort: bool = False) -> None:
        from ._lib import check, lib
        with self._lock:
            if not self._live:
                return
            self._live = False
        check(lib().vitmi_comm_destroy(int(abort)), "comm_destroy")


def exchange_unique_id(rank: int, world: int, store=None, key: str = "vitmi_comm_uid") -> bytes:
    """The RCCL id of a new communicator: created by rank 0 (vitmi_comm_get_unique_id) and passed
    to the other ranks through the job's TCPStore (the torch.distributed rendezvous)."""
    if world <= 1:
        return VitmiComm.unique_id()
    store = store if store is not None else dist.distributed_c10d._get_default_store()
    if rank == 0:
        try:
            uid = VitmiComm.unique_id()
        except Exception as e:
            store.set(key, b"ERR:" + str(e).encode()[:200])   # (the other ranks fail too, not wait)
            raise
        store.set(key, uid)
        return uid
    uid = bytes(store.get(key))
    if uid.startswith(b"ERR:"):
        raise RuntimeError(f"vitmi comm: rank 0 could not create the id ({uid[4:].decode(errors='replace')})")
    if len(uid) != UID_BYTES:
        raise RuntimeError(f"vitmi comm: id from the store has {len(uid)} bytes, not {UID_BYTES}")
    return uid


class CommWatchdog:
    """Abort-on-timeout for the RCCL leg ("an ncclCommAbort path on timeout").

    ``watch(event)`` hands over a HIP event recorded on the comm side stream behind a step's last
    all-reduce.  A daemon thread polls the events (``query()`` never blocks); if one is not done
    ``timeout_s`` after it was handed over -- a peer died or hangs, so RCCL's kernels never
    finish -- it calls ``on_timeout()`` (the reducer's abort: ``ncclCommAbort`` through
    ``vitmi_comm_destroy(1)``, which lets the stuck kernels exit and the streams drain) and
    records the failure; ``check()`` raises it in the training thread."""

    def __init__(self, timeout_s: float, on_timeout: Callable[[], None], poll_s: float = 0.05):
        self.timeout_s = float(timeout_s)
        self.poll_s = poll_s
        self._on_timeout = on_timeout
        self._pending: List[Tuple[object, float]] = []
        self._lock = threading.Lock()
        self._wake = threading.Event()
        self._stop = False
        self.error: Optional[str] = None
        self._thread = threading.Thread(target=self._run, name="vitmi-comm-watchdog", daemon=True)
        self._thread.start()

    def watch(self, event) -> None:
        with self._lock:
            self._pending.append((event, time.monotonic() + self.timeout_s))
        self._wake.set()

    def check(self) -> None:
        if self.error is not None:
            raise RuntimeError(self.error)

    def close(self) -> None:
        self._stop = True
        self._wake.set()
        self._thread.join(timeout=5)

    def _run(self) -> None:
        while not self._stop and self.error is None:
            with self._lock:
                pend = list(self._pending)
            if not pend:
                self._wake.wait(1.0)
                self._wake.clear()
                continue
            done = 0
            for ev, deadline in pend:
                if ev.query():
                    done += 1
                    continue
                if time.monotonic() > deadline:
                    self.error = (f"vitmi comm: gradient all-reduce not finished after {self.timeout_s:g} s "
                                  "(peer failure or hang); communicator aborted")
                    try:
                        self._on_timeout()
                    finally:
                        return
                break                      # events complete in order: wait for this one
            with self._lock:
                del self._pending[:done]
            time.sleep(self.poll_s)


def plan_buckets(n: int, per: int, cuts: Optional[Sequence[int]] = None, solo_tail: int = 2) -> List[Tuple[int, int]]:
    """Bucket bounds over a flat buffer of n elements, at most ``per`` elements each.

    Without ``cuts``: fixed-size buckets.  With ``cuts`` (the offsets at which the backward's
    finished prefix can end: one per block, head and embedding, in order), buckets end on cuts,
    packed greedily up to ``per``, except that the last ``solo_tail`` segments get buckets of
    their own.  A bucket's all-reduce can only start when the backward has passed its end, so
    whatever the last bucket holds is exchanged after the backward, exposed: with the ViT-B
    arena in 64 MiB fixed buckets that is 64 MiB launched at block 0's end plus 7.3 MiB at
    finish(); with solo tail segments it is block 0's 28 MB, overlapped with the patch
    embedding's backward, plus the embedding's 3 MB."""
    if not cuts:
        return [(s, min(n, s + per)) for s in range(0, n, per)]
    cuts = sorted({c for c in cuts if 0 < c < n} | {n})
    segs, prev = [], 0
    for c in cuts:
        segs.append((prev, c))
        prev = c
    tail = segs[len(segs) - solo_tail:] if solo_tail > 0 else []
    head = segs[:len(segs) - len(tail)]
    out: List[Tuple[int, int]] = []
    start = 0
    for a, b in head:
        if b - start > per and a > start:           # close the bucket before this segment
            out.append((start, a))
            start = a
        while b - start > per:                      # a segment larger than a bucket: split it
            out.append((start, start + per))
            start += per
    if head and head[-1][1] > start:
        out.append((start, head[-1][1]))
    for a, b in tail:
        for s0 in range(a, b, per):
            out.append((s0, min(b, s0 + per)))
    return out


class GradReducer:
    """Bucketed, overlapped all-reduce (mean) over one flat gradient buffer.

    ``timeout_s`` (vitmi RCCL leg): a step whose exchange has not finished that long after
    ``finish()`` aborts the communicator (CommWatchdog) and the next ``start()``/``finish()``
    raises; 0 disables the watchdog."""

    def __init__(self, flat_grad: torch.Tensor, bucket_mb: float = 64.0, group=None,
                 comm: Optional[VitmiComm] = None, grad_dtype: str = "fp32", reserve_cus: int = 0,
                 timeout_s: float = 600.0, cuts: Optional[Sequence[int]] = None):
        self.flat = flat_grad
        self.group = group
        self.comm = comm
        if comm is not None:
            self.world = comm.world
            self.backend = "vitmi"
        else:
            self.world = dist.get_world_size(group) if dist.is_initialized() else 1
            self.backend = dist.get_backend(group) if dist.is_initialized() else None
        if grad_dtype not in ("fp32", "bf16"):
            raise ValueError("grad_dtype must be 'fp32' or 'bf16'")
        if grad_dtype == "bf16" and comm is None:
            raise ValueError("grad_dtype='bf16' needs the vitmi RCCL communicator")
        self.grad_dtype = grad_dtype
        self.reserve_cus = int(reserve_cus)
        n = flat_grad.numel()
        per = max(64, int(bucket_mb * (1 << 20) / flat_grad.element_size()) // 64 * 64)
        self.bounds: List[Tuple[int, int]] = plan_buckets(n, per, cuts)
        self._next = 0
        self._ready = 0
        self._handles: list = []
        self._active = comm is not None or self.world > 1
        self._side = torch.cuda.Stream(device=flat_grad.device) if comm is not None and flat_grad.is_cuda else None
        self._lp = (torch.empty(n, dtype=torch.bfloat16, device=flat_grad.device)
                    if comm is not None and grad_dtype == "bf16" else None)
        self._prev_reserve: Optional[int] = None
        self.launch_log: List[Tuple[int, int]] = []   # (ready prefix, bucket index) for tests
        self.readiness: Optional["ArenaReadiness"] = None   # set by attach()
        # the watchdog thread only aborts the communicator (which releases a blocked enqueue); the CU
        # reservation is a training-thread global, restored by finish()/start()/abort()
        self.watchdog = (CommWatchdog(timeout_s, self._abort_comm)
                         if comm is not None and timeout_s and timeout_s > 0 else None)
        # the step's tail: the buckets launched by the last readiness event of the backward (the
        # embedding's parameters) and by finish(): exchanged after the backward's compute
        self.tail_launched: List[int] = []
        self._burst: List[int] = []
        # called as f(start, end, stream) when bucket [start, end) holds its final (reduced)
        # gradient, ready on `stream` (None: the current stream): world 1, or the vitmi comm leg
        # with its side stream (vitmi.optim.Adam.overlap_with)
        self.listeners: List[Callable[[int, int, Optional["torch.cuda.Stream"]], None]] = []

    def _restore_reserve(self) -> None:
        if self._prev_reserve is not None:
            from ._lib import lib
            lib().vitmi_gemm_set_reserved_cus(self._prev_reserve)
            self._prev_reserve = None

    def _abort_comm(self) -> None:
        """Abort the RCCL communicator without waiting for peers (vitmi_comm_destroy(1) ->
        ncclCommAbort), so its stuck kernels exit.  Safe from the watchdog thread."""
        if self.comm is not None and self.comm.live:
            self.comm.destroy(abort=True)

    def abort(self) -> None:
        """Tear down after a failure (training thread): give the persistent GEMM its CUs back and
        abort the communicator."""
        self._restore_reserve()
        self._abort_comm()

    def close(self) -> None:
        if self.watchdog is not None:
            self.watchdog.close()

    def start(self) -> None:
        """Call before the backward of every step."""
        if self.watchdog is not None:
            try:
                self.watchdog.check()
            except RuntimeError:
                self._restore_reserve()
                raise
        self._next, self._ready, self._handles = 0, 0, []
        self._burst = []
        self.launch_log = []
        if self.readiness is not None:
            self.readiness.reset()
        if self._active and self.reserve_cus > 0 and self._prev_reserve is None:
            from ._lib import lib
            self._prev_reserve = lib().vitmi_gemm_set_reserved_cus(self.reserve_cus)

    def _launch(self) -> None:
        s, e = self.bounds[self._next]
        buf = self.flat[s:e]
        if self.comm is not None and self._side is None:
            self.comm.allreduce_async(buf, None, None, REDUCE_AVG)      # a host-side comm (tests)
        elif self.comm is not None:
            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream(buf.device))
            if self._lp is None:
                self.comm.allreduce_async(buf, self._side, ready, REDUCE_AVG)
            else:
                from . import ops
                lp = self._lp[s:e]
                self._side.wait_event(ready)
                with torch.cuda.stream(self._side):
                    ops.cast_bf16(buf, lp)
                    self.comm.allreduce_async(lp, self._side, None, REDUCE_AVG)
                    ops.cast_f32(lp, buf)
        else:
            op = dist.ReduceOp.AVG if self.backend == "nccl" else dist.ReduceOp.SUM
            h = dist.all_reduce(buf, op=op, group=self.group, async_op=True)
            self._handles.append((h, buf))
        self.launch_log.append((self._ready, self._next))
        self._next += 1

    def _notify(self, i: int, stream) -> None:
        s, e = self.bounds[i]
        for f in self.listeners:
            f(s, e, stream)

    def mark_ready(self, end: int) -> None:
        """Gradients in flat[0:end] are final: launch every bucket inside that prefix."""
        self._ready = max(self._ready, end)
        if not self._active:
            # nothing to exchange: the buckets are final as they are (listeners only)
            while self.listeners and self._next < len(self.bounds) and self.bounds[self._next][1] <= self._ready:
                self._notify(self._next, None)
                self._next += 1
            return
        burst = []
        while self._next < len(self.bounds) and self.bounds[self._next][1] <= self._ready:
            burst.append(self._next)
            self._launch()
            if self.comm is not None and self._side is not None:
                self._notify(self._next - 1, self._side)
        if burst:
            self._burst = burst

    def finish(self) -> None:
        if not self._active:
            return
        try:
            if self.watchdog is not None:
                self.watchdog.check()
            rest = list(range(self._next, len(self.bounds)))
            self.tail_launched = (self._burst if self._ready >= self.flat.numel() else []) + rest
            while self._next < len(self.bounds):
                self._launch()
            if self._side is not None:
                # the optimizer (on the compute stream) runs after every bucket's exchange
                torch.cuda.current_stream(self.flat.device).wait_stream(self._side)
                if self.watchdog is not None:
                    done = torch.cuda.Event()
                    done.record(self._side)
                    self.watchdog.watch(done)
                self.comm.check()          # asynchronous RCCL errors surface here, not as a hang
            for h, buf in self._handles:
                h.wait()   # nccl: the current (compute) stream waits on the RCCL stream
                if self.backend != "nccl":
                    buf.div_(self.world)
            self._handles = []
        finally:
            self._restore_reserve()


class ParamGradReducer:
    """Data parallelism for a model without a parameter arena (the CvT / SLS regressors of
    models/CvT(Par).py, trained by vitmi.train.fit): after the backward, the parameters'
    gradients are packed into one persistent flat fp32 buffer (one multi-tensor copy), averaged
    by the same bucketed GradReducer (RCCL through the vitmi communicator, or the process
    group), and unpacked.  These models are a few MB of parameters, so the exchange is not
    overlapped with the backward; the ViT's arena path (attach) is."""

    def __init__(self, params: Sequence[torch.nn.Parameter], bucket_mb: float = 64.0, group=None,
                 comm: Optional[VitmiComm] = None):
        self.params = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("ParamGradReducer: no trainable parameters")
        n = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(n, dtype=torch.float32, device=self.params[0].device)
        self.views: List[torch.Tensor] = []
        off = 0
        for p in self.params:
            self.views.append(self.flat[off:off + p.numel()].view(p.shape))
            off += p.numel()
        self.red = GradReducer(self.flat, bucket_mb, group, comm=comm)

    @property
    def active(self) -> bool:
        return self.red._active

    def start(self) -> None:
        """Before the backward (nothing to do: the exchange runs after it)."""

    def finish(self) -> None:
        self.reduce()

    @torch.no_grad()
    def reduce(self) -> None:
        """Replace every parameter's .grad by its mean over ranks (a missing grad counts as 0)."""
        if not self.active:
            return
        for p in self.params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        torch._foreach_copy_(self.views, [p.grad for p in self.params])
        self.red.start()
        self.red.mark_ready(self.flat.numel())
        self.red.finish()
        torch._foreach_copy_([p.grad for p in self.params], self.views)


def broadcast_module(model: torch.nn.Module, src: int = 0, group=None, comm: Optional[VitmiComm] = None) -> None:
    """Rank ``src``'s parameters and buffers (BatchNorm moving statistics) to every rank, for a
    model without a parameter arena."""
    if comm is not None:
        if comm.world <= 1:
            return
    elif not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return
    with torch.no_grad():
        for t in list(model.parameters()) + list(model.buffers()):
            if not t.is_floating_point():
                continue
            if comm is not None:
                buf = t.detach().contiguous().float()
                comm.broadcast(buf, src)
                t.copy_(buf)
            else:
                dist.broadcast(t.data, src, group=group)


class ArenaReadiness:
    """Tracks which parameters of a ParamArena hold their final gradient in this backward and
    feeds the finished prefix (arena order = backward order) to the reducer.

    One ``register_post_accumulate_grad_hook`` per parameter fires once AccumulateGrad has
    written ``.grad`` (after the Function that produced it, and after every other Function
    contributing to that parameter).  If ``.grad`` is not the parameter's arena view (a gradient
    accumulated into a tensor of its own), the hook copies it into the view and rebinds it, so
    the bucket that all-reduces the flat buffer sees it.  Frozen parameters count as done."""

    def __init__(self, arena, red: GradReducer):
        self.arena, self.red = arena, red
        ps = arena.params
        self.index = {id(p): i for i, p in enumerate(ps)}
        self.starts = [arena.offsets[id(p)] for p in ps] + [arena.numel]
        self.done = [False] * len(ps)
        self.k = 0
        self.handles = [p.register_post_accumulate_grad_hook(self._hook) for p in ps]

    def reset(self) -> None:
        self.done = [not p.requires_grad for p in self.arena.params]
        self.k = 0
        self._advance()

    def _hook(self, p: torch.Tensor) -> None:
        i = self.index[id(p)]
        v = self.arena.view(self.arena.grad, p)
        if p.grad is not None and p.grad.data_ptr() != v.data_ptr():
            with torch.no_grad():
                v.copy_(p.grad)
            p.grad = v
        self.done[i] = True
        self._advance()

    def _advance(self) -> None:
        k, n = self.k, len(self.done)
        while k < n and self.done[k]:
            k += 1
        if k != self.k:
            self.k = k
            self.red.mark_ready(self.starts[k])

    def remove(self) -> None:
        for h in self.handles:
            h.remove()
        self.handles = []


def attach(model, bucket_mb: float = 64.0, group=None, comm: Optional[VitmiComm] = None,
           grad_dtype: str = "fp32", reserve_cus: int = 0, timeout_s: float = 600.0) -> GradReducer:
    """Wire a GradReducer to a vitmi VisionTransformer's arena: buckets launch from the
    parameters' post-accumulate-grad hooks (ArenaReadiness) as the backward finishes them."""
    arena = model.arena()

    def end_of(params) -> int:
        return max(arena.offsets[id(p)] + p.numel() for p in params) if params else 0

    # bucket ends on the prefixes the backward finishes (head, each block, the embedding)
    cuts = [end_of(list(model.head.parameters()) + list(model.norm.parameters()))]
    cuts += [end_of(list(blk.parameters())) for blk in reversed(model.blocks)]
    cuts += [arena.numel]
    red = GradReducer(arena.grad, bucket_mb, group, comm=comm, grad_dtype=grad_dtype, reserve_cus=reserve_cus,
                      timeout_s=timeout_s, cuts=cuts)
    red.readiness = ArenaReadiness(arena, red)
    return red


def param_checksum(flat: torch.Tensor) -> Tuple[float, int]:
    """(fp64 sum, exact bit checksum) of a flat fp32 buffer.  The bit checksum is
    sum_i bits_i * (i mod 65521 + 1) over the int32 bit patterns in wrapping int64 arithmetic:
    independent of the summation order, so equal on two replicas exactly when (barring a
    collision) their bytes are."""
    with torch.no_grad():
        f = flat.detach().reshape(-1)
        s64 = float(f.double().sum().item())
        bits = f.view(torch.int32).to(torch.int64)
        w = torch.arange(bits.numel(), device=f.device, dtype=torch.int64).remainder_(65521).add_(1)
        exact = int(bits.mul_(w).sum().item())
    return s64, exact


def replica_report(flat: torch.Tensor, group=None) -> dict:
    """Whether every rank holds the same parameters after the timed steps: MAX and MIN over the
    ranks of the checksums must agree (synchronous data parallelism keeps the replicas
    bit-identical, as MirroredStrategy does: old_codes/BayConvT(Par)(Muti).py:16-19)."""
    s64, exact = param_checksum(flat)
    out = {"param_checksum_fp64": s64, "param_checksum_bits": exact}
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        out["replicas_identical"] = True
        return out
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    vals = {}
    for name, v, dt in (("bits", exact, torch.int64), ("fp64", s64, torch.float64)):
        mx = torch.tensor([v], dtype=dt, device=dev)
        mn = mx.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
        dist.all_reduce(mn, op=dist.ReduceOp.MIN, group=group)
        vals[name] = (mx.item(), mn.item())
    out["replicas_identical"] = all(a == b for a, b in vals.values())
    out["param_checksum_fp64_minmax"] = list(vals["fp64"])
    return out


def comm_report(red: GradReducer) -> dict:
    """The exchange the reducer ran: communicator ranks and library (asked of the communicator
    itself), the bucket plan and the tail the last finish() launched after the backward."""
    es = red.flat.element_size()
    mib = [(e - s) * es / 2 ** 20 for s, e in red.bounds]
    out = {"buckets_mib": [round(m, 2) for m in mib], "bucket_count": len(mib),
           "tail_buckets": list(red.tail_launched),
           "tail_bucket_mib": round(sum(mib[i] for i in red.tail_launched), 2),
           "grad_dtype": red.grad_dtype, "reserve_cus": red.reserve_cus}
    if red.comm is not None:
        rank, world = red.comm.info()
        out.update(backend="vitmi RCCL communicator", ranks=world, rank=rank, library=type(red.comm).library())
    else:
        out.update(backend=f"torch.distributed {red.backend}", ranks=red.world,
                   library=f"ProcessGroup {red.backend}" if red.backend else None)
    return out


def comm_or_fallback(rank: int, world: int, make_group=None):
    """The library's RCCL communicator for the job, or -- when creating it fails on ANY rank (the
    ranks agree over the default, bootstrap process group) -- a torch.distributed process group
    from ``make_group`` (default: a new ``nccl`` group, i.e. torch's RCCL) for the same exchange.
    Returns (comm or None, group or None, this rank's error text or None).  The library's init is
    non-blocking and bounded (VITMI_COMM_INIT_TIMEOUT_S, default 600 s; csrc/comm.cpp): a rank
    whose peer failed inside the collective init times out there and reaches the agreement below
    instead of blocking for ever; a communicator that did come up is aborted, not destroyed
    gracefully (its peers may be gone)."""
    err = None
    comm = None
    try:
        comm = VitmiComm.from_store(rank, world)
    except Exception as e:   # noqa: BLE001 -- any init failure of the comm leg
        err = f"{type(e).__name__}: {e}"
    ok = torch.tensor([0 if err else 1], dtype=torch.int32)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if ok.item() == 1:
        return comm, None, None
    if comm is not None:
        comm.destroy(abort=True)
    group = make_group() if make_group is not None else dist.new_group(backend="nccl")
    return None, group, err


def broadcast_parameters(model, src: int = 0, group=None, comm: Optional[VitmiComm] = None) -> None:
    flat = model.arena().flat
    if comm is not None:
        if comm.world > 1:
            comm.broadcast(flat, src)
    elif dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(flat, src, group=group)


def init_from_env(backend: Optional[str] = None) -> Tuple[int, int, int]:
    """torchrun-style bootstrap: returns (rank, world, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend or ("nccl" if torch.cuda.is_available() else "gloo"),
                                rank=rank, world_size=world)
    return rank, world, local
