"""The reference's optimizer and learning-rate schedule on the fused vitmi kernel.

``model.compile(optimizer=keras.optimizers.Adam(learning_rate=1e-3), loss='mean_squared_error')``
(``models/CvT(Par).py:458-460``) and ``lr_scheduler`` (``:357-360``: x0.8 every 50 epochs).

``Adam`` runs Keras' update (include/vitmi.h ``vitmi_adam_step``): ONE launch over a model's
ParamArena (every parameter, gradient and moment at the same flat offsets), which also writes
the bf16 operand shadow the next forward's GEMMs read; models without an arena (the CvT) get
one launch per parameter tensor.
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np
import torch

from . import ops
from ._lib import check, lib

Tensor = torch.Tensor


def keras_alpha(lr: float, beta_1: float, beta_2: float, step: int) -> float:
    """alpha = lr sqrt(1 - b2^t) / (1 - b1^t), in float32 like Keras' update_step."""
    f = np.float32
    b1p = np.power(f(beta_1), f(step), dtype=np.float32)
    b2p = np.power(f(beta_2), f(step), dtype=np.float32)
    return float(f(lr) * np.sqrt(f(1) - b2p, dtype=np.float32) / (f(1) - b1p))


class Adam:
    """keras.optimizers.Adam(learning_rate, beta_1=0.9, beta_2=0.999, epsilon=1e-7).

    ``target``: a model with ``arena()`` (VisionTransformer: single fused launch + bf16 shadow
    refresh) or an iterable of parameters.  ``grad_scale`` multiplies the gradients as they are
    read (e.g. 1/world for a sum all-reduce)."""

    def __init__(self, target, learning_rate: float = 1e-3, beta_1: float = 0.9, beta_2: float = 0.999,
                 epsilon: float = 1e-7, grad_scale: float = 1.0):
        self.learning_rate = float(learning_rate)
        self.beta_1, self.beta_2, self.epsilon = float(beta_1), float(beta_2), float(epsilon)
        self.grad_scale = float(grad_scale)
        self.iterations = 0
        self._model = target if hasattr(target, "arena") else None
        if self._model is not None:
            arena = self._model.arena()
            self._arena = arena
            self.params: List[Tensor] = list(arena.params)
            self._m = torch.zeros_like(arena.flat)
            self._v = torch.zeros_like(arena.flat)
        else:
            self._arena = None
            self.params = [p for p in target if p.requires_grad]
            self._m = [torch.zeros_like(p) for p in self.params]
            self._v = [torch.zeros_like(p) for p in self.params]
        self._ov = None   # overlap_with state

    def overlap_with(self, red) -> None:
        """Step each gradient bucket of ``red`` (``vitmi.dp.attach``'s reducer) as soon as the
        backward has finished it (world 1) or its all-reduce has (the vitmi comm leg): the update
        of the blocks behind the backward runs on a side stream beside it, and ``step()`` only
        launches the rest and joins.  The update is the same launch over the same elements, in
        another order of ranges (elementwise, so bitwise the same result).  Needs one backward per
        ``step()`` (no gradient accumulation across backwards) and every arena parameter
        trainable; otherwise that step runs the plain single launch.  The learning rate is read
        when the backward finishes its first bucket."""
        if self._arena is None:
            raise ValueError("vitmi Adam.overlap_with: needs a model with a parameter arena")
        if red.flat.data_ptr() != self._arena.grad.data_ptr() or red.flat.numel() != self._arena.grad.numel():
            raise ValueError("vitmi Adam.overlap_with: the reducer is not over this model's gradient arena")
        self._ov = {"stream": torch.cuda.Stream(device=self._arena.flat.device), "done": 0, "alpha": None,
                    "skip": False}
        red.listeners.append(self._on_bucket)

    def _launch(self, s0: int, e0: int, alpha: float) -> None:
        arena, lp = self._arena, self._arena.flat_lp
        check(lib().vitmi_adam_step(e0 - s0, ops._p(arena.flat[s0:]), ops._p(arena.grad[s0:]), ops._p(self._m[s0:]),
                                    ops._p(self._v[s0:]), ops._p(lp[s0:]) if lp is not None else None, alpha,
                                    self.beta_1, self.beta_2, self.epsilon, self.grad_scale, ops._s()),
              "adam_step")

    @torch.no_grad()
    def _on_bucket(self, s0: int, e0: int, stream) -> None:
        ov = self._ov
        if ov["skip"]:
            return
        if ov["alpha"] is None:
            # the first bucket of this backward
            if not all(p.requires_grad for p in self._arena.params) or s0 != 0:
                ov["skip"] = True
                return
            ov["alpha"] = keras_alpha(self.learning_rate, self.beta_1, self.beta_2, self.iterations + 1)
        if s0 != ov["done"]:
            raise RuntimeError("vitmi Adam: gradient buckets finished out of order")
        side = ov["stream"]
        ready = torch.cuda.Event()
        ready.record(stream if stream is not None else torch.cuda.current_stream(self._arena.flat.device))
        side.wait_event(ready)
        with torch.cuda.stream(side):
            self._launch(s0, e0, ov["alpha"])
        ov["done"] = e0

    # -- keras-style schedule hook
    @property
    def lr(self) -> float:
        return self.learning_rate

    @lr.setter
    def lr(self, v: float) -> None:
        self.learning_rate = float(v)

    def zero_grad(self, set_to_none: bool = True) -> None:
        """torch's convention: drop the gradients (the next forward of an arena model zeroes the
        flat buffer once and the backward writes into it again), or zero them in place."""
        for p in self.params:
            if p.grad is None:
                continue
            if set_to_none:
                p.grad = None
            else:
                p.grad.zero_()

    @torch.no_grad()
    def step(self) -> None:
        self.iterations += 1
        alpha = keras_alpha(self.learning_rate, self.beta_1, self.beta_2, self.iterations)
        if self._arena is not None:
            arena = self._model.arena()
            if arena is not self._arena:
                raise RuntimeError("vitmi Adam: the model's parameter arena was rebuilt after the optimizer "
                                   "was created (model moved?); create the optimizer after placing the model")
            # the launch reads the flat gradient buffer: every .grad must be its arena view (they
            # are after a backward from an arena forward; a gradient set elsewhere is copied in).
            # Parameters with no gradient (frozen, or zero_grad(set_to_none) and no backward) are
            # not stepped, as in torch / Keras: the launch covers the runs of the arena between them
            stepping = [p.requires_grad and p.grad is not None for p in arena.params]
            ov, done = self._ov, 0
            if ov is not None:
                done, ov_alpha = ov["done"], ov["alpha"]
                ov["done"], ov["alpha"], ov["skip"] = 0, None, False
                if done:
                    # the buckets the backward finished were stepped on the side stream
                    torch.cuda.current_stream(arena.flat.device).wait_stream(ov["stream"])
                    alpha = ov_alpha
            if not any(stepping):
                return
            lp = arena.flat_lp
            if not all(stepping):
                arena.refresh_lp()          # the skipped parameters' shadow must be current too
            arena.bind_grads(fill_missing=all(stepping))
            for s0, e0 in arena.runs(stepping):
                s0 = max(s0, done)
                if e0 > s0:
                    self._launch(s0, e0, alpha)
            arena.mark_lp_fresh()
            return
        for p, m, v in zip(self.params, self._m, self._v):
            if p.grad is None:
                continue
            if not (p.is_contiguous() and p.grad.is_contiguous()):
                raise RuntimeError("vitmi Adam: parameters and gradients must be contiguous")
            check(lib().vitmi_adam_step(p.numel(), ops._p(p), ops._p(p.grad), ops._p(m), ops._p(v), None, alpha,
                                        self.beta_1, self.beta_2, self.epsilon, self.grad_scale, ops._s()),
                  "adam_step")
            # the kernel wrote through a raw pointer: bump the version counter, so a ParamArena
            # that owns p (its bf16 operand shadow is keyed on these counters) re-casts it
            torch.autograd.graph.increment_version(p)

    # -- checkpointing (Keras saves the optimizer variables with the model weights)
    def state_dict(self) -> Dict:
        if self._arena is not None:
            return {"iterations": self.iterations, "learning_rate": self.learning_rate, "m": self._m.clone(),
                    "v": self._v.clone()}
        return {"iterations": self.iterations, "learning_rate": self.learning_rate,
                "m": [t.clone() for t in self._m], "v": [t.clone() for t in self._v]}

    def load_state_dict(self, sd: Dict) -> None:
        self.iterations = int(sd["iterations"])
        self.learning_rate = float(sd["learning_rate"])
        with torch.no_grad():
            if self._arena is not None:
                self._m.copy_(sd["m"])
                self._v.copy_(sd["v"])
            else:
                for dst, src in zip(self._m, sd["m"]):
                    dst.copy_(src)
                for dst, src in zip(self._v, sd["v"]):
                    dst.copy_(src)


def keras_step_decay(epoch: int, lr: float, every: int = 50, factor: float = 0.8) -> float:
    """lr_scheduler (models/CvT(Par).py:357-360): x0.8 at every 50th epoch (epoch > 0)."""
    if epoch > 0 and epoch % every == 0:
        return lr * factor
    return lr


__all__ = ["Adam", "keras_alpha", "keras_step_decay"]

