"""Data-parallel gradient reduction for the MI355X ViT path.

Replaces the reference's only parallel construct, ``tf.distribute.MirroredStrategy()``
(``old_codes/BayConvT(Par)(Muti).py:16-19``): synchronous data parallelism with a
cross-replica mean of every gradient once per step.  MI355X design:

* one process per GPU (torchrun), ``torch.distributed`` with backend ``nccl`` = RCCL
  over xGMI (``gloo`` on CPU for the tests);
* all gradients live in ONE flat fp32 buffer (``ParamArena``) laid out in the order
  the backward finishes them (head, norm, block L-1 ... block 0, patch-embed), so
  fixed-size buckets (default 64 MiB: few, large collectives suit per-link-bound
  xGMI rings) become ready front to back;
* each block's backward calls its ``_grad_ready_hook`` when its grads are final;
  every bucket wholly inside the finished prefix is all-reduced at once with
  ``async_op=True``: RCCL runs it on the process group's own HIP stream, ordered
  after the compute stream's work so far, so it overlaps the rest of the backward;
* ``finish()`` launches the tail buckets and makes the compute stream wait for them,
  so the optimizer sees averaged gradients.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


class GradReducer:
    """Bucketed, overlapped all-reduce over one flat gradient buffer."""

    def __init__(self, flat_grad: torch.Tensor, bucket_mb: float = 64.0, group=None):
        self.flat = flat_grad
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.backend = dist.get_backend(group) if dist.is_initialized() else None
        n = flat_grad.numel()
        per = max(64, int(bucket_mb * (1 << 20) / flat_grad.element_size()) // 64 * 64)
        self.bounds: List[Tuple[int, int]] = [(s, min(n, s + per)) for s in range(0, n, per)]
        self._next = 0
        self._ready = 0
        self._handles: list = []
        self.launch_log: List[Tuple[int, int]] = []   # (ready prefix, bucket index) for tests

    def start(self) -> None:
        """Call before the backward of every step."""
        self._next, self._ready, self._handles = 0, 0, []
        self.launch_log = []

    def _launch(self) -> None:
        s, e = self.bounds[self._next]
        buf = self.flat[s:e]
        op = dist.ReduceOp.AVG if self.backend == "nccl" else dist.ReduceOp.SUM
        h = dist.all_reduce(buf, op=op, group=self.group, async_op=True)
        self._handles.append((h, buf))
        self.launch_log.append((self._ready, self._next))
        self._next += 1

    def mark_ready(self, end: int) -> None:
        """Gradients in flat[0:end] are final: launch every bucket inside that prefix."""
        if self.world <= 1:
            return
        self._ready = max(self._ready, end)
        while self._next < len(self.bounds) and self.bounds[self._next][1] <= self._ready:
            self._launch()

    def finish(self) -> None:
        if self.world <= 1:
            return
        while self._next < len(self.bounds):
            self._launch()
        for h, buf in self._handles:
            h.wait()   # nccl: the current (compute) stream waits on the RCCL stream
            if self.backend != "nccl":
                buf.div_(self.world)
        self._handles = []


def attach(model, bucket_mb: float = 64.0, group=None) -> GradReducer:
    """Wire a GradReducer to a vitmi VisionTransformer's arena and backward hooks."""
    arena = model.arena()
    red = GradReducer(arena.grad, bucket_mb, group)

    def end_of(params: Sequence[torch.nn.Parameter]) -> int:
        return max(arena.offsets[id(p)] + p.numel() for p in params)

    head_end = end_of(list(model.head.parameters()) + list(model.norm.parameters()))
    object.__setattr__(model, "_head_ready_hook", lambda: red.mark_ready(head_end))
    for blk in model.blocks:
        e = end_of(list(blk.parameters()))
        object.__setattr__(blk, "_grad_ready_hook", _hook(red, e))
    object.__setattr__(model.patch_embed, "_grad_ready_hook", _hook(red, arena.numel))
    return red


def _hook(red: GradReducer, end: int) -> Callable:
    return lambda _mod: red.mark_ready(end)


def broadcast_parameters(model, src: int = 0, group=None) -> None:
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(model.arena().flat, src, group=group)


def init_from_env(backend: Optional[str] = None) -> Tuple[int, int, int]:
    """torchrun-style bootstrap: returns (rank, world, local_rank)."""
    import os
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
