"""ORACLE — CPU restatement of the reference's optimizer (TEST INFRASTRUCTURE ONLY).

Only ``tests/`` use this module; the product package never imports it.

``keras.optimizers.Adam(learning_rate=1e-3)`` (``models/CvT(Par).py:458-460``; beta_1 0.9,
beta_2 0.999, epsilon 1e-7).  The algorithm lives in the third-party Keras package, absent
here and unpinned by the reference (``from tensorflow import keras``); restated from Keras'
published ``Adam.update_step`` (TF >= 2.11 / Keras 3, ``keras/optimizers/adam.py``):

    alpha = lr * sqrt(1 - beta_2 ** t) / (1 - beta_1 ** t)        (float32 tensors)
    m += (g - m) * (1 - beta_1);  v += (g**2 - v) * (1 - beta_2)   ((1 - beta) a Python float)
    p -= (m * alpha) / (sqrt(v) + epsilon)

in numpy float32, one IEEE-rounded operation at a time (the GPU kernel does the same ops in the
same order, so the comparison is bit-exact).  ``lr_scheduler`` (``:357-360``) is restated too.
Parity: unpinned against Keras itself (not importable here); pinned by the formula above.
"""
from __future__ import annotations

import numpy as np

f32 = np.float32


def keras_alpha(lr: float, beta_1: float, beta_2: float, t: int) -> np.float32:
    b1p = np.power(f32(beta_1), f32(t), dtype=np.float32)
    b2p = np.power(f32(beta_2), f32(t), dtype=np.float32)
    return f32(lr) * np.sqrt(f32(1) - b2p, dtype=np.float32) / (f32(1) - b1p)


def adam_step(p, g, m, v, lr, t, beta_1=0.9, beta_2=0.999, epsilon=1e-7, grad_scale=1.0):
    """One Keras Adam step on float32 numpy arrays; returns new (p, m, v)."""
    p, g, m, v = (np.asarray(a, dtype=np.float32) for a in (p, g, m, v))
    if grad_scale != 1.0:
        g = g * f32(grad_scale)
    alpha = keras_alpha(lr, beta_1, beta_2, t)
    m = m + (g - m) * f32(1.0 - beta_1)
    v = v + (g * g - v) * f32(1.0 - beta_2)
    p = p - (m * alpha) / (np.sqrt(v) + f32(epsilon))
    return p, m, v


def lr_scheduler(epoch: int, lr: float) -> float:
    """models/CvT(Par).py:357-360."""
    if epoch > 0 and epoch % 50 == 0:
        return lr * 0.8
    return lr
