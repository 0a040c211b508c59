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
  * otherwise a zeroed buffer, which AccumulateGrad adds into an existing ``.grad`` (gradient
    accumulation across backwards) or keeps as the new ``.grad``.  The buffers of one backward
    are views of ONE flat allocation, zeroed by one fill (a model without an arena, e.g. the CvT,
    otherwise paid a fill launch per parameter per step: CvT step 7.32-7.33 -> 7.23-7.27 ms).
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
        self._params: Dict[int, Tensor] = {}
        for i, p in slots:
            if p is not None:
                self._need[id(p)] = self._need.get(id(p), False) or bool(need[i])
                self._params[id(p)] = p
        self._arena = arena
        self._dst: Dict[int, Optional[Tensor]] = {}
        self._flat: Optional[Tensor] = None
        self._off: Dict[int, int] = {}

    def _fresh(self, p: Tensor) -> Tensor:
        """p's zeroed destination: a view of the flat buffer laid out, on the first call, for every
        parameter of this backward that takes a gradient (the call only comes when the arena,
        if any, has no fresh view to offer, i.e. for all of them but in a mixed case)."""
        if self._flat is None:
            n = 0
            for k, q in self._params.items():
                if self._need[k]:
                    self._off[k] = n
                    n += (q.numel() + 3) // 4 * 4     # 16-B aligned views
            self._flat = torch.zeros(max(n, 4), dtype=torch.float32, device=p.device)
        o = self._off.get(id(p))
        if o is None or p.dtype != torch.float32 or p.device != self._flat.device:
            return torch.zeros_like(p, memory_format=torch.contiguous_format)
        return self._flat[o:o + p.numel()].view(p.shape)

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
                d = self._fresh(p)
        self._dst[id(p)] = d
        return d

    def wants(self, p: Optional[Tensor]) -> bool:
        return p is not None and self._need.get(id(p), False)

    def grads(self, params: Sequence[Optional[Tensor]]) -> Tuple[Optional[Tensor], ...]:
        """What the Function returns for ``params``: the destinations handed out (None for a
        parameter whose gradient another Function of the graph supplies, or none wants)."""
        return tuple(None if p is None else self._dst.get(id(p)) for p in params)


__all__ = ["GradSink"]
