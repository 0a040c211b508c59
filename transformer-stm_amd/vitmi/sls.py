"""SLS data pipeline: the reference's dataset, resident in HBM.

``preprocess_data`` / ``train_and_save_model`` (``models/CvT(Par).py:363-453``) rebuilt for one
process per GPU:

* labels / process parameters from the two workbooks (``vitmi.xlsx``, no openpyxl needed),
  the reference's valid-piece logic, ``StandardScaler`` on the repeated process rows, and its
  train / validation split (first valid piece of every block of 5 -> validation);
* images: JPEG decode on the host (PIL, a thread pool; libjpeg releases the GIL), uint8 frames
  staged through pinned memory in chunks, H2D on a side stream, and ONE ``vitmi_sls_preprocess``
  launch per chunk (cv2 INTER_LINEAR resize + BGR2GRAY + /255 in OpenCV's 8-bit fixed point)
  writing the fp32 model inputs into a tensor that stays in HBM for the whole run (40,000
  layers x 64 KiB = 2.6 GB of the 288 GB);
* batches: ``vitmi_gather_rows`` from device index tensors -- no per-step host->device copy
  (the reference feeds numpy arrays to ``model.fit`` every step, §3.1).
"""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import ops
from ._lib import check, lib
from .xlsx import read_xlsx

Tensor = torch.Tensor

# models/CvT(Par).py:22 and :392
FREQUENCIES = ['50HZ_Bm', '50HZ_Hc', '50HZ_μa', '50HZ_Br', '50HZ_Pcv', '200HZ_Bm', '200HZ_Hc', '200HZ_μa',
               '200HZ_Br', '200HZ_Pcv', '400HZ_Bm', '400HZ_Hc', '400HZ_μa', '400HZ_Br', '400HZ_Pcv', '800HZ_Bm',
               '800HZ_Hc', '800HZ_μa', '800HZ_Br', '800HZ_Pcv']
PROCESS_PARAMETERS = ["氧濃度", "雷射掃描速度", "雷射功率", "線間距", "能量密度"]


@dataclass
class SLSSpec:
    """The reference's constants (models/CvT(Par).py:31-46, :60-64, :421)."""
    labels_xlsx: str = ""                 # Excel/Processed_Circle_test.xlsx
    process_xlsx: str = ""                # Excel/Process_parameters.xlsx
    data_root: str = ""                   # data/  (holds circle(340x345)/trail{g}_{pp}/layer_{i:02d}.jpg)
    freq: str = "50HZ_Bm"
    group_start: int = 1
    group_end: int = 40
    piece_start: int = 1
    piece_end: int = 5
    image_layers: int = 200
    height: int = 128
    width: int = 128

    @property
    def pieces_per_group(self) -> int:
        return self.piece_end - self.piece_start + 1


# ---------------------------------------------------------------- labels / params / split
def standard_scaler(x: np.ndarray) -> np.ndarray:
    """sklearn StandardScaler().fit_transform: population std, (near-)constant columns -> 1."""
    mean = x.mean(axis=0)
    std = x.std(axis=0)
    std = np.where(std < 10 * np.finfo(np.float64).eps * np.maximum(1.0, np.abs(mean)), 1.0, std)
    return (x - mean) / std


def build_index(spec: SLSSpec, label_col: Optional[Sequence[float]] = None,
                process_rows: Optional[Sequence[Sequence[float]]] = None):
    """(labels [n_valid*layers], proc_scaled [n_valid*layers, 5], valid piece indices, count):
    models/CvT(Par).py:363-412.  The tables come from the workbooks unless given."""
    per = spec.pieces_per_group
    n_pieces = spec.group_end * per
    if label_col is None:
        sheet = read_xlsx(spec.labels_xlsx)
        label_col = [sheet.cell(i, spec.freq) for i in range(n_pieces)]
    if process_rows is None:
        ps = read_xlsx(spec.process_xlsx)
        process_rows = [[ps.cell(g, name) for name in PROCESS_PARAMETERS] for g in range(spec.group_end)]
    lab = np.array([np.nan if v is None or isinstance(v, str) else float(v) for v in label_col[:n_pieces]],
                   dtype=np.float64)
    start, end = (spec.group_start - 1) * per, spec.group_end * per
    idx = np.arange(n_pieces)
    valid = idx[~np.isnan(lab) & (idx >= start) & (idx < end)]
    L = spec.image_layers
    labels = np.repeat(lab[valid], L)
    proc = np.asarray(process_rows, dtype=np.float64)[valid // per]
    proc = np.repeat(proc, L, axis=0)
    return labels, standard_scaler(proc), valid, n_pieces


def split_rows(valid: np.ndarray, count: int, image_layers: int) -> Tuple[np.ndarray, np.ndarray]:
    """models/CvT(Par).py:437-453: layer rows of the training and validation sets."""
    valid = np.asarray(valid)
    blocks = valid // 5
    first = np.zeros(len(valid), dtype=bool)
    if len(valid):
        _, first_pos = np.unique(blocks, return_index=True)   # valid is increasing
        first[first_pos] = True
    rows = np.arange(len(valid) * image_layers).reshape(len(valid), image_layers)
    return rows[~first].reshape(-1), rows[first].reshape(-1)


def layer_paths(spec: SLSSpec, valid: Sequence[int]) -> List[str]:
    """models/CvT(Par).py:415-423 (folder trail{g}_{pp}, files layer_{i:02d}.jpg)."""
    per = spec.pieces_per_group
    out = []
    for index in valid:
        g, p = int(index) // per + 1, int(index) % per + 1
        folder = os.path.join(spec.data_root, f"circle(340x345)/trail{g:01d}_{p:02d}")
        out += [os.path.join(folder, f"layer_{i + 1:02d}.jpg") for i in range(spec.image_layers)]
    return out


# ---------------------------------------------------------------- images
def resize_table(ssize: int, dsize: int) -> Tuple[np.ndarray, np.ndarray]:
    ofs = np.zeros(dsize, dtype=np.int32)
    w = np.zeros(2 * dsize, dtype=np.int16)
    check(lib().vitmi_sls_resize_table(ssize, dsize, ofs.ctypes.data, w.ctypes.data), "sls_resize_table")
    return ofs, w


class _Tables:
    def __init__(self, H: int, W: int, Ho: int, Wo: int, device):
        xo, xw = resize_table(W, Wo)
        yo, yw = resize_table(H, Ho)
        self.key = (H, W, Ho, Wo)
        self.xo, self.xw = torch.from_numpy(xo).to(device), torch.from_numpy(xw).to(device)
        self.yo, self.yw = torch.from_numpy(yo).to(device), torch.from_numpy(yw).to(device)


def preprocess_frames(frames: Tensor, Ho: int, Wo: int, out: Optional[Tensor] = None, bgr: bool = False,
                      tables: Optional[_Tables] = None) -> Tensor:
    """uint8 frames [n, H, W, 3] on the device -> fp32 [n, 1, Ho, Wo] (resize, gray, /255)."""
    assert frames.dtype == torch.uint8 and frames.dim() == 4 and frames.shape[-1] == 3 and frames.is_contiguous()
    n, H, W, _ = frames.shape
    if tables is None or tables.key != (H, W, Ho, Wo):
        tables = _Tables(H, W, Ho, Wo, frames.device)
    if out is None:
        out = torch.empty(n, 1, Ho, Wo, dtype=torch.float32, device=frames.device)
    assert out.is_contiguous() and out.numel() == n * Ho * Wo
    check(lib().vitmi_sls_preprocess(n, H, W, ops._p(frames), H * W * 3, W * 3, int(bgr), Ho, Wo, ops._p(tables.xo),
                                     ops._p(tables.xw), ops._p(tables.yo), ops._p(tables.yw), ops._p(out), ops._s()),
          "sls_preprocess")
    return out


def decode_jpeg_rgb(path: str) -> np.ndarray:
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("RGB"))


def load_images(paths: Sequence[str], Ho: int, Wo: int, device, chunk: int = 256, workers: int = 16,
                decode=decode_jpeg_rgb) -> Tensor:
    """Decode on the host (thread pool) -> pinned chunks -> side-stream H2D -> preprocess
    launch per chunk; the next chunk decodes while the GPU converts the current one."""
    n = len(paths)
    if n == 0:
        return torch.empty(0, 1, Ho, Wo, dtype=torch.float32, device=device)
    first = decode(paths[0])
    H, W, _ = first.shape
    out = torch.empty(n, 1, Ho, Wo, dtype=torch.float32, device=device)
    tables = _Tables(H, W, Ho, Wo, device)
    pinned = [torch.empty(chunk, H, W, 3, dtype=torch.uint8).pin_memory() for _ in range(2)]
    dev_buf = [torch.empty(chunk, H, W, 3, dtype=torch.uint8, device=device) for _ in range(2)]
    done = [None, None]
    copy_stream = torch.cuda.Stream(device=device)
    compute = torch.cuda.current_stream(device)

    def fill(slot: int, lo: int, hi: int, pool) -> None:
        imgs = list(pool.map(decode, paths[lo:hi]))
        for i, a in enumerate(imgs):
            if a.shape != (H, W, 3):
                raise ValueError(f"{paths[lo + i]}: frame {a.shape} differs from the first frame {(H, W, 3)}")
            pinned[slot][i].numpy()[...] = a

    with ThreadPoolExecutor(max_workers=workers) as pool:
        for k, lo in enumerate(range(0, n, chunk)):
            hi = min(n, lo + chunk)
            slot = k % 2
            if done[slot] is not None:
                done[slot].synchronize()          # the pinned slot's previous upload has landed
            fill(slot, lo, hi, pool)
            with torch.cuda.stream(copy_stream):
                copy_stream.wait_stream(compute)   # dev_buf[slot] free (its last preprocess done)
                dev_buf[slot][:hi - lo].copy_(pinned[slot][:hi - lo], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(copy_stream)
            compute.wait_event(ev)
            preprocess_frames(dev_buf[slot][:hi - lo], Ho, Wo, out[lo:hi], tables=tables)
            done[slot] = ev
    torch.cuda.synchronize(device)
    return out


def gather_rows(src: Tensor, idx: Tensor, out: Optional[Tensor] = None) -> Tensor:
    """out[i] = src[idx[i]] (device idx int64) on the vitmi gather kernel."""
    assert src.is_contiguous() and idx.dtype == torch.int64 and idx.is_cuda
    rows = src.shape[0]
    row_bytes = src[0].numel() * src.element_size() if rows else src.element_size()
    if out is None:
        out = torch.empty((idx.numel(),) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    check(lib().vitmi_gather_rows(idx.numel(), row_bytes, ops._p(src), rows, ops._p(idx.contiguous()), ops._p(out),
                                  ops._s()), "gather_rows")
    return out


# ---------------------------------------------------------------- dataset
class SLSDataset:
    """HBM-resident (images [N,1,H,W], proc [N,5], labels [N]) + train / val row indices."""

    def __init__(self, images: Tensor, proc: Tensor, labels: Tensor, train_rows: np.ndarray, val_rows: np.ndarray):
        self.images, self.proc, self.labels = images, proc, labels
        dev = images.device
        self.train_rows = torch.as_tensor(np.asarray(train_rows, dtype=np.int64), device=dev)
        self.val_rows = torch.as_tensor(np.asarray(val_rows, dtype=np.int64), device=dev)

    @classmethod
    def from_reference_layout(cls, spec: SLSSpec, device="cuda", max_pieces: Optional[int] = None,
                              workers: int = 16, label_col=None, process_rows=None) -> "SLSDataset":
        """The reference's files (workbooks + data/circle(340x345)/...), or explicit tables."""
        labels, proc, valid, count = build_index(spec, label_col, process_rows)
        train, val = split_rows(valid, count, spec.image_layers)
        if max_pieces is not None:                      # bounded subsets (tests / smoke runs)
            keep = max_pieces * spec.image_layers
            labels, proc, valid = labels[:keep], proc[:keep], valid[:max_pieces]
            train, val = train[train < keep], val[val < keep]
        images = load_images(layer_paths(spec, valid), spec.height, spec.width, device, workers=workers)
        return cls(images, torch.as_tensor(proc, dtype=torch.float32, device=device),
                   torch.as_tensor(labels, dtype=torch.float32, device=device), train, val)

    @classmethod
    def synthetic(cls, n_pieces: int = 200, image_layers: int = 200, height: int = 128, width: int = 128,
                  proc_dim: int = 5, device="cuda", seed: int = 0, frame_hw=(345, 340)) -> "SLSDataset":
        """Same shapes and flow as the reference data (random uint8 frames through the same
        preprocessing kernel), for benchmarks on a box without the dataset."""
        g = torch.Generator(device=device).manual_seed(seed)
        N = n_pieces * image_layers
        images = torch.empty(N, 1, height, width, dtype=torch.float32, device=device)
        tables = _Tables(frame_hw[0], frame_hw[1], height, width, device)
        for lo in range(0, N, 1024):
            hi = min(N, lo + 1024)
            fr = torch.randint(0, 256, (hi - lo, frame_hw[0], frame_hw[1], 3), dtype=torch.uint8, device=device,
                               generator=g)
            preprocess_frames(fr, height, width, images[lo:hi], tables=tables)
        proc = torch.randn(n_pieces, proc_dim, device=device, generator=g).repeat_interleave(image_layers, 0)
        labels = torch.randn(n_pieces, device=device, generator=g).repeat_interleave(image_layers, 0)
        valid = np.arange(n_pieces)
        train, val = split_rows(valid, n_pieces, image_layers)
        return cls(images, proc.contiguous(), labels.contiguous(), train, val)

    def __len__(self) -> int:
        return self.images.shape[0]

    def batches(self, rows: Tensor, batch_size: int, shuffle: bool = True,
                generator: Optional[torch.Generator] = None,
                shard: Tuple[int, int] = (0, 1)) -> Iterator[Tuple[Tensor, Tensor, Tensor]]:
        """Keras fit order: a fresh permutation per epoch (shuffle=True), the last batch partial.
        ``shard=(rank, world)`` yields only this rank's rows ``[rank::world]`` of every global
        batch (the generator must be seeded alike on every rank, so the permutation agrees)."""
        if shuffle:
            rows = rows[torch.randperm(rows.numel(), device=rows.device, generator=generator)]
        rank, world = shard
        for lo in range(0, rows.numel(), batch_size):
            idx = rows[lo:lo + batch_size][rank::world]
            yield gather_rows(self.images, idx), gather_rows(self.proc, idx), gather_rows(self.labels, idx)


__all__ = ["SLSSpec", "SLSDataset", "FREQUENCIES", "PROCESS_PARAMETERS", "build_index", "split_rows",
           "layer_paths", "standard_scaler", "resize_table", "preprocess_frames", "load_images", "gather_rows"]

