#!/usr/bin/env python
"""Measure the SLS rows of SURVEY §8f on one GPU (prints one JSON line):

* row 3, data pipeline: JPEG frames (340x345 RGB, the reference's layer images; synthetic
  content written to a temp dir since the dataset is not on the GPU box) -> host decode
  (thread pool) -> pinned chunks -> H2D -> cv2-fixed-point resize + gray + /255 kernel ->
  HBM-resident fp32 dataset.  Reported: frames/s end to end, and the GPU conversion alone;
  beside it the reference's per-image host loop with PIL standing in for cv2 (1 thread, a
  bounded sample) as the CPU baseline.
* row 2, the reference's training objective: CvT (Keras spec, dw_bn, cls, process-parameter
  head) fwd + MSE + bwd + Keras Adam at batch 128 (models/CvT(Par).py:46,458-476) over
  batches gathered from the HBM-resident dataset: images/s of `vitmi.train.fit`.

    python tools/sls_bench.py [--frames 2048 --epochs 2 --workers 16]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vitmi import cvt, optim, sls, train  # noqa: E402


def write_frames(d: str, n: int, seed: int = 0):
    from PIL import Image
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:345, 0:340]
    paths = []
    for i in range(n):
        # a bright ring on a noisy background, roughly like an SLS layer photograph
        r = np.hypot(yy - 172 + rng.normal(0, 3), xx - 170 + rng.normal(0, 3))
        base = np.clip(200 * np.exp(-((r - 110) / 25) ** 2) + rng.normal(40, 12, r.shape), 0, 255)
        img = np.stack([base, base * 0.95, base * 0.9], -1).astype(np.uint8)
        p = os.path.join(d, f"layer_{i:05d}.jpg")
        Image.fromarray(img).save(p, quality=92)
        paths.append(p)
    return paths


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=2048)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--cpu-frames", type=int, default=64)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    out = {}
    with tempfile.TemporaryDirectory() as d:
        paths = write_frames(d, args.frames)
        sls.load_images(paths[:64], 128, 128, dev, chunk=64, workers=args.workers)   # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        images = sls.load_images(paths, 128, 128, dev, chunk=256, workers=args.workers)
        torch.cuda.synchronize()
        t_load = time.perf_counter() - t0
        # the GPU conversion alone, on frames already in HBM
        frames = torch.from_numpy(np.stack([sls.decode_jpeg_rgb(p) for p in paths[:512]])).to(dev)
        sls.preprocess_frames(frames, 128, 128)
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(10):
            sls.preprocess_frames(frames, 128, 128)
        ev1.record()
        torch.cuda.synchronize()
        t_kern = ev0.elapsed_time(ev1) / 10 / 1e3
        # the reference's per-image host work (imread -> resize -> gray -> /255, :419-423) with
        # PIL standing in for cv2 (absent here), one thread, bounded sample
        from PIL import Image
        t0 = time.perf_counter()
        for p in paths[:args.cpu_frames]:
            with Image.open(p) as im:
                g8 = im.convert("RGB").resize((128, 128), Image.BILINEAR).convert("L")
                np.asarray(g8, dtype=np.float32) / 255.0
        t_cpu = (time.perf_counter() - t0) / args.cpu_frames
    out["pipeline"] = {"frames": args.frames, "frame": "340x345 RGB JPEG -> 128x128 fp32",
                       "end_to_end_frames_per_sec": round(args.frames / t_load, 1),
                       "gpu_convert_frames_per_sec": round(512 / t_kern, 1),
                       "gpu_convert_frame_GBps_mall_resident": round(512 * (345 * 340 * 3 + 128 * 128 * 4) / t_kern / 1e9, 1),
                       "host_decode_workers": args.workers,
                       "cpu_baseline_frames_per_sec": round(1 / t_cpu, 1),
                       "cpu_baseline": "PIL decode + bilinear resize + gray + /255 per image (cv2 absent), 1 thread"}
    # training objective on the resident dataset
    layers = 200 if images.shape[0] >= 2000 else max(1, images.shape[0] // 10)
    n_pieces = images.shape[0] // layers                 # 200 layers per piece, as the reference
    n = n_pieces * layers
    g = torch.Generator(device=dev).manual_seed(0)
    proc = torch.randn(n_pieces, 5, device=dev, generator=g).repeat_interleave(layers, 0)
    labels = torch.randn(n_pieces, device=dev, generator=g).repeat_interleave(layers, 0)
    tr, va = sls.split_rows(np.arange(n_pieces), n_pieces, layers)
    ds = sls.SLSDataset(images[:n].contiguous(), proc.contiguous(), labels.contiguous(), tr, va)
    model = cvt.CvT(cvt.CvTConfig(proc_dim=5, dtype="bf16", drop_rate=0.1)).to(dev)
    model.reset_parameters(0)
    opt = optim.Adam(list(model.parameters()), learning_rate=1e-3)
    train.fit(model, ds, epochs=1, batch_size=args.batch, optimizer=opt, validate=False)   # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hist = train.fit(model, ds, epochs=args.epochs, batch_size=args.batch, optimizer=opt)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n_train = ds.train_rows.numel() * args.epochs
    out["training"] = {"model": "CvT Keras spec 128x128x1 dw_bn cls + process MLP, dropout 0.1", "batch": args.batch,
                       "train_images_per_sec": round(n_train / dt, 1), "epochs": args.epochs,
                       "includes": "batch gather + fwd + MSE + bwd + Keras Adam + per-epoch validation",
                       "last_loss": hist["loss"][-1]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
