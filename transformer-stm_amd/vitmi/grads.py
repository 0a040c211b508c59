"""Parameter gradients of the fused autograd Functions.

The nn.Module surface keeps torch's contract for parameters ("Parameters are
plain nn.Parameters, so torch.optim, state_dict, and DDP-style hooks work unchanged"; the
reference's PyTorch twin accumulates them through autograd, ``old_codes/MS_CvT.py:289-333``).
So every vitmi Function RETURNS its parameters' gradients: AccumulateGrad, parameter hooks
(``register_hook`` / ``register_post_accumulate_grad_hook``), DistributedDataParallel's reducer
and ``torch.autograd.grad`` see them exactly as for a torch op, and a frozen parameter
(``requires_grad=False``) gets no gradient and costs no kernel.

The kernels still write each gradient where it will live, with no extra pass: a GradSink hands
out one fp32 destination per parameter, which the kernels accumulate into (+=):
  * a model with a ParamArena (VisionTransformer) whose ``.grad`` is None: the parameter's view
    of the arena's flat gradient buffer, zeroed once at the forward (``ParamArena.begin_step``).
    AccumulateGrad keeps ("steals") that exact tensor as ``.grad``, so ``.grad`` IS the arena
    view and the DP buckets and the fused Adam read the flat buffer directly;
  * otherwise a fresh zero tensor, which AccumulateGrad adds into an existing ``.grad``
    (gradient accumulation across backwards) or keeps as the new ``.grad``.
"""
from __future__ import annotations

from typing import Dict, Iterable, Optional, Sequence, Tuple

import torch

Tensor = torch.Tensor
_UNSET = object()


class GradSink:
    """Destinations of one backward's parameter gradients.

    ``slots``: (input index of the Function, parameter) pairs; ``ctx.needs_input_grad`` at those
    indices says which parameters take a gradient in this backward.  ``arena``: the owning model's
    ParamArena, or None."""

    def __init__(self, ctx, slots: Iterable[Tuple[int, Tensor]], arena=None):
        need = ctx.needs_input_grad
        self._need: Dict[int, bool] = {}
        for i, p in slots:
            if p is not None:
                self._need[id(p)] = self._need.get(id(p), False) or bool(need[i])
        self._arena = arena
        self._dst: Dict[int, Optional[Tensor]] = {}

    def __call__(self, p: Optional[Tensor]) -> Optional[Tensor]:
        """The fp32 buffer the kernels add p's gradient into, or None (no gradient wanted)."""
        if p is None:
            return None
        d = self._dst.get(id(p), _UNSET)
        if d is not _UNSET:
            return d
        d = None
        if self._need.get(id(p), False):
            if self._arena is not None:
                d = self._arena.take(p)
            if d is None:
                d = torch.zeros_like(p, memory_format=torch.contiguous_format)
        self._dst[id(p)] = d
        return d

    def wants(self, p: Optional[Tensor]) -> bool:
        return p is not None and self._need.get(id(p), False)

    def grads(self, params: Sequence[Optional[Tensor]]) -> Tuple[Optional[Tensor], ...]:
        """What the Function returns for ``params``: the destinations handed out (None for a
        parameter whose gradient another Function of the graph supplies, or none wants)."""
        return tuple(None if p is None else self._dst.get(id(p)) for p in params)


__all__ = ["GradSink"]
