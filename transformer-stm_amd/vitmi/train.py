"""The reference's training objective and loop on the vitmi path.

``train_and_save_model`` (``models/CvT(Par).py:430-489``): ``model.compile(Adam(1e-3),
loss='mean_squared_error', metrics=['mae'])``, ``model.fit([x, proc], y, epochs, batch_size=128,
validation_data=..., callbacks=[LearningRateScheduler(lr_scheduler)])`` (x0.8 every 50 epochs),
then ``save_weights`` and the per-epoch history written out.

``fit`` keeps Keras' semantics: the scheduler runs at the start of every epoch, the training
rows are re-shuffled every epoch (``shuffle=True``), the last batch may be partial, ``loss`` /
``mae`` are batch-size-weighted means over the epoch's steps, ``val_loss`` / ``val_mae`` are
computed in inference mode (BatchNorm with its moving statistics) at the epoch's end.  All
tensors stay on the GPU: batches are gathered from the HBM-resident ``SLSDataset``, and the
epoch's metric sums are read back once per epoch.
"""
from __future__ import annotations

import csv
import time
from typing import Callable, Dict, List, Optional

import torch

from .modules import mse_loss
from .optim import Adam, keras_step_decay
from .sls import SLSDataset

Tensor = torch.Tensor


def _predict(model, img: Tensor, proc: Tensor) -> Tensor:
    return model(img, proc) if getattr(model.cfg, "proc_dim", 0) else model(img)


@torch.no_grad()
def evaluate(model, ds: SLSDataset, rows: Tensor, batch_size: int = 128) -> Dict[str, float]:
    """Inference-mode MSE and MAE over ``rows`` (Keras ``evaluate`` / validation)."""
    was = model.training
    model.eval()
    se = torch.zeros((), dtype=torch.float64, device=ds.images.device)
    ae = torch.zeros((), dtype=torch.float64, device=ds.images.device)
    n = 0
    for img, proc, y in ds.batches(rows, batch_size, shuffle=False):
        pred = _predict(model, img, proc)[:, 0]
        d = (pred - y).double()
        se += (d * d).sum()
        ae += d.abs().sum()
        n += y.numel()
    model.train(was)
    n = max(n, 1)
    return {"loss": se.item() / n, "mae": ae.item() / n}


def fit(model, ds: SLSDataset, epochs: int, batch_size: int = 128, optimizer: Optional[Adam] = None,
        learning_rate: float = 1e-3, lr_schedule: Optional[Callable[[int, float], float]] = keras_step_decay,
        shuffle: bool = True, seed: int = 0, validate: bool = True,
        log: Optional[Callable[[str], None]] = None) -> Dict[str, List[float]]:
    """models/CvT(Par).py:458-476.  Returns the Keras-style history (one entry per epoch)."""
    dev = ds.images.device
    # a model with a parameter arena gets the single fused launch (which also refreshes its bf16 shadow)
    target = model if hasattr(model, "arena") else list(model.parameters())
    opt = optimizer if optimizer is not None else Adam(target, learning_rate=learning_rate)
    gen = torch.Generator(device=dev).manual_seed(seed)
    hist: Dict[str, List[float]] = {"epoch": [], "loss": [], "mae": [], "lr": [], "seconds": []}
    if validate:
        hist["val_loss"], hist["val_mae"] = [], []
    model.train()
    for epoch in range(epochs):
        if lr_schedule is not None:
            opt.lr = lr_schedule(epoch, opt.lr)
        t0 = time.perf_counter()
        se = torch.zeros((), dtype=torch.float64, device=dev)
        ae = torch.zeros((), dtype=torch.float64, device=dev)
        n = 0
        for img, proc, y in ds.batches(ds.train_rows, batch_size, shuffle=shuffle, generator=gen):
            opt.zero_grad()
            pred = _predict(model, img, proc)
            loss = mse_loss(pred, y)
            loss.backward()
            opt.step()
            with torch.no_grad():
                d = (pred.detach()[:, 0] - y).double()
                se += (d * d).sum()
                ae += d.abs().sum()
            n += y.numel()
        n = max(n, 1)
        hist["epoch"].append(epoch + 1)
        hist["loss"].append(se.item() / n)
        hist["mae"].append(ae.item() / n)
        hist["lr"].append(opt.lr)
        if validate and ds.val_rows.numel():
            v = evaluate(model, ds, ds.val_rows, batch_size)
            hist["val_loss"].append(v["loss"])
            hist["val_mae"].append(v["mae"])
        hist["seconds"].append(time.perf_counter() - t0)
        if log is not None:
            log(" ".join(f"{k}={hist[k][-1]:.6g}" for k in hist if hist[k]))
    return hist


def write_history(hist: Dict[str, List[float]], path: str) -> None:
    """The per-epoch records (the reference writes them with DataFrame.to_excel, :484-486)."""
    keys = [k for k in hist if hist[k]]
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(keys)
        for i in range(len(hist["epoch"])):
            w.writerow([hist[k][i] for k in keys])
