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
        log: Optional[Callable[[str], None]] = None, group=None, comm=None,
        dp_bucket_mb: float = 64.0) -> Dict[str, List[float]]:
    """models/CvT(Par).py:458-476.  Returns the Keras-style history (one entry per epoch).

    Data parallel when the process group (``group``) or the vitmi RCCL communicator (``comm``)
    spans more than one rank — the reference's MirroredStrategy (models/CvT(Par).py:20-21,
    old_codes/BayConvT(Par)(Muti).py:16-19): ``batch_size`` stays the GLOBAL batch, every rank
    takes the rows ``[rank::world]`` of each global batch (same shuffle on every rank), rank 0's
    weights are broadcast first, and the gradients are averaged before every optimizer step with
    each rank's loss weighted by its share of the batch, so a ragged last batch still gives the
    global-batch-mean gradient.  BatchNorm normalises over each rank's rows (per-replica, as
    under MirroredStrategy).  The epoch metrics are summed over ranks."""
    from . import dp
    dev = ds.images.device
    if comm is not None:
        rank, world = comm.rank, comm.world
    elif torch.distributed.is_initialized():
        rank, world = torch.distributed.get_rank(group), torch.distributed.get_world_size(group)
    else:
        rank, world = 0, 1
    red = None
    if world > 1:
        if hasattr(model, "arena"):     # the ViT: bucketed exchange overlapped with its backward
            dp.broadcast_parameters(model, 0, group, comm)
            red = dp.attach(model, dp_bucket_mb, group, comm)
        else:
            dp.broadcast_module(model, 0, group, comm)
            red = dp.ParamGradReducer(list(model.parameters()), dp_bucket_mb, group, comm)
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
        n_train = ds.train_rows.numel()
        for i, (img, proc, y) in enumerate(ds.batches(ds.train_rows, batch_size, shuffle=shuffle,
                                                        generator=gen, shard=(rank, world))):
            opt.zero_grad()
            if red is not None:
                red.start()
            if y.numel():
                pred = _predict(model, img, proc)
                loss = mse_loss(pred, y)
                if red is not None:     # this rank's share of the global batch, x world (averaged below)
                    loss = loss * (y.numel() * world / min(batch_size, n_train - i * batch_size))
                loss.backward()
            if red is not None:
                red.finish()
            opt.step()
            if not y.numel():
                continue
            with torch.no_grad():
                d = (pred.detach()[:, 0] - y).double()
                se += (d * d).sum()
                ae += d.abs().sum()
            n += y.numel()
        if red is not None:
            sums = torch.stack([se, ae, torch.tensor(float(n), dtype=torch.float64, device=dev)])
            sums = _sum_over_ranks(sums, group, comm)
            se, ae, n = sums[0], sums[1], int(round(sums[2].item()))
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


def _sum_over_ranks(v: Tensor, group, comm) -> Tensor:
    if comm is not None:
        from .dp import REDUCE_SUM
        buf = v.double().contiguous()       # float64 on the wire, as the process-group path
        side = torch.cuda.current_stream(buf.device)
        comm.allreduce_async(buf, side, None, REDUCE_SUM)
        return buf
    v = v.clone()
    torch.distributed.all_reduce(v, group=group)
    return v


def write_history(hist: Dict[str, List[float]], path: str) -> None:
    """The per-epoch records (the reference writes them with DataFrame.to_excel, :484-486)."""
    keys = [k for k in hist if hist[k]]
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(keys)
        for i in range(len(hist["epoch"])):
            w.writerow([hist[k][i] for k in keys])
