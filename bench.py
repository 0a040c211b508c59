#!/usr/bin/env python
"""Benchmark: images/sec of the ViT-B/16 fwd+bwd training step on MI355X.

BASELINE.json metric: "images/sec fwd+bwd ViT-B/16 224px bs=256/GPU at 1/2/4/8 MI355X;
% MFMA roofline".  One step = forward + CE loss + full backward (hand-written gfx950
kernels) + RCCL gradient all-reduce (N>1) + Keras Adam update (one fused vitmi launch), on a synthetic
batch of 256 images/GPU already resident in HBM, random-init ViT-B/16 weights.

Launch:  python bench.py [--gpus 1 --steps 10 --warmup 3]
         python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
             --master-port P bench.py --gpus N ...
Rank 0 prints ONE JSON line.  Extra fields: `roofline` (dominant kernel: the fc1 GEMM
[M x 3072 x 768], timed live with HIP events on its stream inside the timed region) and
`cpu_baseline` (the CPU oracle's fwd+bwd on the host cores, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from vitmi import dp, ops, optim  # noqa: E402
from vitmi.config import config_c3, config_c5  # noqa: E402
from vitmi.modules import VisionTransformer, cross_entropy  # noqa: E402

METRIC = "images/sec fwd+bwd ViT-B/16 224px bs=256/GPU at 1/2/4/8 MI355X; % MFMA roofline"
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip-level table)
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic_fc1_fwd.json")


def cpu_baseline(cfg, batch: int, steps: int):
    """The CPU oracle (oracle/vit_ref.py) timed on this host's cores: a bounded sample."""
    from oracle import vit_ref
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)), 16))
    torch.set_num_threads(cores)
    params = vit_ref.init_params(cfg, seed=0, randomize_all=False)
    img, tgt = vit_ref.synthetic_batch(cfg, batch)
    vit_ref.forward_backward(img, tgt, params, cfg)          # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        vit_ref.forward_backward(img, tgt, params, cfg)
    dt_ = time.perf_counter() - t0
    return {"value": round(batch * steps / dt_, 3), "unit": "images/sec", "cores": cores, "kind": "port",
            "sample": f"oracle/vit_ref.py fp32 fwd+bwd ViT-B/16 224px, bs={batch}, {steps} steps after 1 warm-up "
                      f"({dt_:.1f} s), torch CPU threads={cores}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=["c3", "c5"], default="c3",
                    help="c3: ViT-B/16 224px bs 256/GPU (the headline metric); c5: ViT-L/16 384px bs 64/GPU "
                         "(BASELINE config 5, N = 577 tokens: a secondary line, not the headline)")
    ap.add_argument("--batch", type=int, default=None, help="images per GPU (default 256 for c3, 64 for c5)")
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=16)
    ap.add_argument("--cpu-steps", type=int, default=8)
    ap.add_argument("--no-optimizer", action="store_true", help="diagnostic only: skip Adam")
    ap.add_argument("--optimizer", choices=["vitmi", "torch"], default="vitmi",
                    help="vitmi: Keras Adam, one fused launch over the arena (+ bf16 shadow); torch: fused torch Adam")
    args = ap.parse_args()

    rank, world, local = dp.init_from_env("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cfg = config_c3() if args.config == "c3" else config_c5()
    B = args.batch or (256 if args.config == "c3" else 64)
    model_name = "vit_base_16" if args.config == "c3" else "vit_large_16"
    metric = METRIC if args.config == "c3" else \
        "images/sec fwd+bwd ViT-L/16 384px bs=64/GPU MI355X; % MFMA roofline (BASELINE config 5)"

    torch.manual_seed(0)
    model = VisionTransformer(cfg).to(dev)
    model.reset_parameters(seed=0)
    red = dp.attach(model, bucket_mb=args.bucket_mb)
    dp.broadcast_parameters(model)
    if args.optimizer == "vitmi":
        opt = optim.Adam(model, learning_rate=1e-3)     # keras.optimizers.Adam(1e-3), models/CvT(Par).py:458
    else:
        try:
            opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)
        except (RuntimeError, TypeError):
            opt = torch.optim.Adam(model.parameters(), lr=1e-3, foreach=True)
    arena = model.arena()

    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    img = torch.rand(B, cfg.in_chans, cfg.img_size, cfg.img_size, device=dev, generator=g)
    tgt = torch.randint(0, cfg.num_classes, (B,), device=dev, generator=g)

    opt_events = []   # (start, end) around each timed optimizer step (reported separately)

    def step(timed=False):
        arena.grad.zero_()
        red.start()
        logits = model(img)
        loss = cross_entropy(logits, tgt)
        loss.backward()
        red.finish()
        if not args.no_optimizer:
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            opt.step()
            if timed:
                e1.record()
                opt_events.append((e0, e1))
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    M, F_, D = B * cfg.seq_len, cfg.mlp_dim, cfg.embed_dim
    events = ops.set_probe((M, F_, D))        # fc1 forward GEMM launches
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step(timed=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ops.set_probe(None)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = t.item()

    ms_step = elapsed / args.steps * 1e3
    imgs = B * world * args.steps / elapsed
    kern_ms = sum(a.elapsed_time(b) for a, b in events) / max(1, len(events))
    kflop = 2.0 * M * F_ * D
    achieved = kflop / (kern_ms * 1e-3) / 1e12
    traffic = None
    if os.path.exists(TRAFFIC_FILE):
        try:
            tr = json.load(open(TRAFFIC_FILE))
            if tr.get("M") == M:
                traffic = tr.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None
    step_flops = cfg.flops_per_image_fwd_bwd() * B * world
    out = {
        "metric": metric,
        "value": round(imgs, 2),
        "unit": "images/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (torch.rand images in [0,1), randint labels; random-init trunc_normal(.02) weights)",
        "config": {"workload": f"{'ViT-B/16 224' if args.config == 'c3' else 'ViT-L/16 384'}x"
                               f"{cfg.img_size}x3 fwd + CE loss + bwd + RCCL grad all-reduce + Adam step",
                   "optimizer": "keras Adam (vitmi fused)" if args.optimizer == "vitmi" else "torch fused Adam",
                   "model": model_name, "global_batch": B * world, "seq_len": cfg.seq_len,
                   "parallelism": f"dp{world}"},
        "roofline": {"bound": "mfma", "kernel": f"gemm fc1 fwd bf16 [{M}x{F_}x{D}] +bias+GELU",
                     "achieved": round(achieved, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": traffic,
                     "launches_timed": len(events), "avg_launch_ms": round(kern_ms, 4)},
        "optimizer_ms": (round(sum(a.elapsed_time(b) for a, b in opt_events) / len(opt_events), 3)
                         if opt_events else None),
        "step_mfma_frac": round(step_flops / (elapsed / args.steps) / 1e12 / (PEAK_BF16_TFLOPS * world), 4),
        "loss": round(float(loss.item()), 5),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "c3":
        out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_batch, args.cpu_steps)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
