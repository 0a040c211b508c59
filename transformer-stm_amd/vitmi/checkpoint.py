"""Weight save / load: ``model.save_weights(...h5)`` after training
(``models/CvT(Par).py:489``) and ``model.load_weights(...)`` before testing
(``models/CvT_test(Par).py:513``).

One safetensors file (no pickling; h5py is not in this image): every parameter and buffer
(BatchNorm moving statistics included) under its module path, plus optionally the optimizer's
moments and step count under ``optimizer/...``.  Loading checks names and shapes strictly.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
from safetensors.torch import load_file, save_file

Tensor = torch.Tensor


def state_tensors(model) -> Dict[str, Tensor]:
    out = {k: v.detach() for k, v in model.named_parameters()}
    out.update({k: v.detach() for k, v in model.named_buffers()})
    return out


def save_weights(model, path: str, optimizer=None, metadata: Optional[Dict[str, str]] = None) -> None:
    t = {k: v.contiguous().cpu() for k, v in state_tensors(model).items()}
    meta = dict(metadata or {})
    if optimizer is not None:
        sd = optimizer.state_dict()
        meta["optimizer.iterations"] = str(sd["iterations"])
        meta["optimizer.learning_rate"] = repr(sd["learning_rate"])
        if isinstance(sd["m"], list):
            for i, (m, v) in enumerate(zip(sd["m"], sd["v"])):
                t[f"optimizer/m/{i}"] = m.contiguous().cpu()
                t[f"optimizer/v/{i}"] = v.contiguous().cpu()
        else:
            t["optimizer/m"] = sd["m"].contiguous().cpu()
            t["optimizer/v"] = sd["v"].contiguous().cpu()
    save_file(t, path, metadata=meta)


def load_weights(model, path: str, optimizer=None, strict: bool = True) -> None:
    from safetensors import safe_open
    t = load_file(path)
    mine = state_tensors(model)
    missing = [k for k in mine if k not in t]
    extra = [k for k in t if k not in mine and not k.startswith("optimizer/")]
    if strict and (missing or extra):
        raise KeyError(f"checkpoint mismatch: missing {missing[:5]}, unexpected {extra[:5]}")
    with torch.no_grad():
        for k, dst in mine.items():
            if k not in t:
                continue
            src = t[k]
            if tuple(src.shape) != tuple(dst.shape):
                raise ValueError(f"{k}: checkpoint shape {tuple(src.shape)} != model {tuple(dst.shape)}")
            dst.copy_(src.to(dst.device, dst.dtype))
    if optimizer is not None:
        with safe_open(path, framework="pt") as f:
            meta = f.metadata() or {}
        if "optimizer.iterations" not in meta:
            raise KeyError("checkpoint holds no optimizer state")
        if "optimizer/m" in t:
            m, v = t["optimizer/m"], t["optimizer/v"]
        else:
            n = sum(1 for k in t if k.startswith("optimizer/m/"))
            m = [t[f"optimizer/m/{i}"] for i in range(n)]
            v = [t[f"optimizer/v/{i}"] for i in range(n)]
        optimizer.load_state_dict({"iterations": int(meta["optimizer.iterations"]),
                                   "learning_rate": float(meta["optimizer.learning_rate"]), "m": m, "v": v})
