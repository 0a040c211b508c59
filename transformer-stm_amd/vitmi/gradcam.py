"""Grad-CAM heatmaps on the vitmi CvT.

``make_gradcam_heatmap`` (``tools/grad_cam_CvT.py:422-481``): for each batch (default one
image), the gradient of ``predictions[:, 0]`` with respect to a stage's spatial output
activation A [b, H, W, C] (``stage3_transformer`` by default, ``:48``), channel weights
``pooled = mean(grads, axis=(0, 1, 2))``, ``heatmap = sum_c pooled[c] * A[0, :, :, c]``, then
``max(heatmap, 0) / max(heatmap)``.

The activation gradients come out of the hand-written backward kernels (head, LayerNorm, the
fused CvT blocks); the model runs in inference mode (BatchNorm on its moving statistics), as
the Keras model call inside the reference's GradientTape does.  Batches of ``chunk`` images are
processed together; the reference's per-``batch_size`` pooling is applied within each chunk.
"""
from __future__ import annotations

from typing import Optional

import torch

Tensor = torch.Tensor


def gradcam_heatmaps(model, images: Tensor, proc: Optional[Tensor] = None, stage: int = -1, batch_size: int = 1,
                     chunk: int = 64) -> Tensor:
    """images [N, C, S, S] (device) -> heatmaps [N // batch_size, H, W] fp32 of ``stage``."""
    if chunk % batch_size:
        raise ValueError("chunk must be a multiple of batch_size")
    was = model.training
    model.eval()
    out = []
    try:
        model._capture_stage = stage
        for lo in range(0, images.shape[0], chunk):
            img = images[lo:lo + chunk]
            pr = None if proc is None else proc[lo:lo + chunk]
            with torch.enable_grad():
                for p in model.parameters():
                    p.grad = None
                pred = model(img, pr) if pr is not None else model(img)
                t, H, has_cls = model._captured
                pred[:, 0].sum().backward()
            A = t.detach()
            G = t.grad
            if has_cls:
                A, G = A[:, 1:], G[:, 1:]
            n, _, C = A.shape
            A = A.reshape(n, H, H, C)
            G = G.reshape(n // batch_size, batch_size, H, H, C)
            pooled = G.mean(dim=(1, 2, 3))                                  # [groups, C]
            first = A.reshape(n // batch_size, batch_size, H, H, C)[:, 0]   # A[0] of each batch
            hm = (first * pooled[:, None, None, :]).sum(-1)
            mx = hm.flatten(1).max(dim=1).values
            out.append(torch.clamp(hm, min=0) / mx[:, None, None])
    finally:
        model._capture_stage = None
        model._captured = None
        for p in model.parameters():
            p.grad = None
        model.train(was)
    return torch.cat(out, 0)
