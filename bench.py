#!/usr/bin/env python
"""Benchmark: images/sec of the ViT-B/16 fwd+bwd training step on MI355X.

BASELINE.json metric: "images/sec fwd+bwd ViT-B/16 224px bs=256/GPU at 1/2/4/8 MI355X;
% MFMA roofline".  One step = forward + CE loss + full backward (hand-written gfx950
kernels) + RCCL gradient all-reduce (N>1, the library's vitmi_comm_* leg on a side stream,
overlapped with the backward) + Keras Adam update (one fused vitmi launch), on a synthetic
batch of 256 images/GPU already resident in HBM, random-init ViT-B/16 weights.

Launch:  python bench.py [--gpus 1 --steps 10 --warmup 3]
         python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
             --master-port P bench.py --gpus N ...
Rank 0 prints ONE JSON line.  Besides the contract fields it carries, measured in this run:
  roofline      the dominant kernel (fc1 GEMM [M x 3072 x 768] + bias + GELU) timed with HIP
                events on its stream inside the timed region; `traffic` = its HBM bytes per
                launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over the same
                GEMM run as a child process;
  per_kernel    a rocprofv3 --kernel-trace --stats child run of this bench (3 steps), joined
                with the library's own per-kernel algorithmic work (vitmi_stats_*): ms/step,
                TFLOP/s, GB/s and MFMA fraction per kernel;
  cpu_baseline  the CPU oracle's fwd+bwd on the host cores (rank 0 at N=1 only);
  parity        this line's own arithmetic (dtype, knobs) against the north star's 1e-3: logits
                max-abs of the line's full-depth model with randomised parameters on 2 images
                vs the fp32 CPU oracle (every line, secondary ones included).
The evidence legs run after the timed region (N=1, rank 0) and never change `value`.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil
import signal
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from vitmi import _lib, dp, ops, optim, trace  # noqa: E402
from vitmi.config import config_c2, config_c3, config_c5  # noqa: E402
from vitmi.modules import VisionTransformer, cross_entropy  # noqa: E402

METRIC = "images/sec fwd+bwd ViT-B/16 224px bs=256/GPU at 1/2/4/8 MI355X; % MFMA roofline"
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip-level table)
PEAK_HBM_GBPS = 8000.0      # MI355X HBM3E peak (MI355X_MICROARCH.md)
PEAK_FP32_TFLOPS = 157.3    # MI355X fp32 matrix


def _knob_qkv(cfg) -> str:
    """How the precision knob's qkv GEMM runs (vitmi/modules.py Block.split_qkv's default)."""
    sq = cfg.split_qkv
    if sq is None:
        sq = True if cfg.dtype == "bf16x3" else ("weight" if cfg.embed_dim % 128 == 0 else False)
    if sq is True:
        return "split"
    return "weight-side e4m3 correction" if sq == "weight" and cfg.dtype == "bf16f8" else "bf16"


# ------------------------------------------------------------------ CPU baseline (oracle)

def _lscpu_model() -> str:
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                return line.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    return "unknown"


def cpu_baseline(cfg, batch: int, steps: int):
    """The CPU oracle (oracle/vit_ref.py, fp32) timed on this host's cores: 1 warm-up step and
    `steps` timed steps at `batch` images (BASELINE.md §2 protocol).  Threads: every core of the
    affinity mask, capped by the pool's per-GPU CPU share (OMP_NUM_THREADS, set to 16 on the
    GPU boxes, whose affinity mask spans the whole multi-tenant host)."""
    from oracle import vit_ref
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", affinity) or affinity)
    cores = max(1, min(affinity, share))
    torch.set_num_threads(cores)
    params = vit_ref.init_params(cfg, seed=0, randomize_all=False)
    img, tgt = vit_ref.synthetic_batch(cfg, batch)
    vit_ref.forward_backward(img, tgt, params, cfg)          # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        vit_ref.forward_backward(img, tgt, params, cfg)
    dt_ = time.perf_counter() - t0
    out = {"value": round(batch * steps / dt_, 3), "unit": "images/sec", "cores": cores, "kind": "port",
           "affinity_cores": affinity, "cpu_model": _lscpu_model(),
           "sample": f"oracle/vit_ref.py fp32 fwd+bwd ViT-B/16 224px, bs={batch}, 1 warm-up + {steps} timed "
                     f"steps ({dt_:.1f} s), torch CPU threads={cores} (affinity {affinity}, pool share "
                     f"OMP_NUM_THREADS={share})"}
    return out


NORTH_STAR_LOGITS = 1e-3    # BASELINE.json north_star: logits within 1e-3 of the fp32 CPU reference


def parity_check(cfg, dev, n_img: int = 2):
    """The north-star logits check of THIS line's arithmetic, after the timed region: the line's
    model (its config, compute dtype and knob settings) at full depth with randomised parameters
    (every weight, bias, LayerNorm gamma/beta drawn: vit_ref.init_params(randomize_all=True), the
    stress case of tests/test_gpu_model.py) on `n_img` synthetic images, GPU logits against the
    fp32 CPU oracle (oracle/vit_ref.py) on the same parameters and inputs."""
    from oracle import vit_ref
    t0 = time.perf_counter()
    params = vit_ref.init_params(cfg, seed=0, randomize_all=True)
    x, _ = vit_ref.synthetic_batch(cfg, n_img)
    with torch.no_grad():
        ref = vit_ref.forward(x, params, cfg)
        model = VisionTransformer(cfg).to(dev)
        model.load_param_dict(params)
        got = model(x.to(dev)).float().cpu()
    del model
    err = float((got - ref).abs().max().item())
    return {"logits_max_abs": err, "bound": NORTH_STAR_LOGITS, "within_bound": err <= NORTH_STAR_LOGITS,
            "logits_max_abs_ref": float(ref.abs().max().item()),
            "sample": f"{n_img} synthetic images, this line's model ({cfg.depth} blocks, D={cfg.embed_dim}, "
                      f"{cfg.img_size}px, dtype {cfg.dtype}) with randomised parameters (init_params seed 0, "
                      f"randomize_all), GPU logits vs the fp32 CPU oracle ({time.perf_counter() - t0:.1f} s)"}


# ------------------------------------------------------------------ evidence legs (child runs)
def _run(cmd, timeout, cwd=ROOT, log=None):
    """Run a child in its own process group; kill the group on timeout.  -> returncode or None."""
    with open(log or os.devnull, "w") as f:
        p = subprocess.Popen(cmd, cwd=cwd, stdout=f, stderr=subprocess.STDOUT, start_new_session=True,
                             env=dict(os.environ, PYTHONUNBUFFERED="1"))
        try:
            return p.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
            return None


def _demangle(names):
    """__cxa_demangle of mangled names (the demangler rocprofv3 applies to kernel names)."""
    import ctypes
    try:
        cxx = ctypes.CDLL("libstdc++.so.6")
        fn = cxx.__cxa_demangle
        fn.restype = ctypes.c_void_p
        free = ctypes.CDLL("libc.so.6").free
    except OSError:
        return {n: n for n in names}
    out = {}
    for n in names:
        st = ctypes.c_int(0)
        # libstdc++'s demangler predates the DF16b (__bf16) mangling: retry it as a vendor type
        for m in (n, n.replace("DF16b", "u6__bf16")):
            r = fn(m.encode(), None, None, ctypes.byref(st))
            if r and st.value == 0:
                out[n] = ctypes.string_at(r).decode()
                free(ctypes.c_void_p(r))
                break
        else:
            out[n] = n
    return out


def _short(name: str) -> str:
    s = name[5:] if name.startswith("void ") else name
    return s.split("(")[0]


def per_kernel_evidence(args, tmp):
    """rocprofv3 --kernel-trace --stats over a 3-step child run of this bench, joined per kernel
    with the library's algorithmic work table of the same run."""
    rp = shutil.which("rocprofv3")
    if rp is None:
        return {"error": "rocprofv3 not found"}
    steps = 3
    stats_json = os.path.join(tmp, "stats.json")
    cmd = [rp, "--kernel-trace", "--marker-trace", "--stats", "-d", os.path.join(tmp, "kt"), "-o", "run",
           "--output-format", "csv",
           "--", sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(steps), "--warmup", "2",
           "--config", args.config, "--no-cpu-baseline", "--no-evidence", "--no-secondary", "--roctx",
           "--stats-out", stats_json]
    if args.batch:
        cmd += ["--batch", str(args.batch)]
    rc = _run(cmd, 300, log=os.path.join(tmp, "kt.log"))
    if rc != 0 or not os.path.exists(stats_json):
        return {"error": f"rocprofv3 kernel-trace child failed (rc={rc})"}
    work = json.load(open(stats_json))
    lib_names = _demangle([w["name"] for w in work["kernels"]])
    by_name = {}
    for w in work["kernels"]:
        for key in (w["name"], lib_names[w["name"]]):
            by_name[_short(key)] = w
    traces = glob.glob(os.path.join(tmp, "kt", "**", "run_kernel_trace.csv"), recursive=True)
    if not traces:
        return {"error": "no kernel trace"}
    # the timed steps are the dispatches between the two marker kernels (torch.cuda._sleep ->
    # spin_kernel) the child launches around its timed region
    disp = sorted(csv.DictReader(open(traces[0])), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(disp) if "spin_kernel" in r["Kernel_Name"]]
    if len(marks) < 2:
        return {"error": "timed-region markers not found in the kernel trace"}
    agg = {}
    for r in disp[marks[0] + 1:marks[-1]]:
        k = _short(r["Kernel_Name"])
        a = agg.setdefault(k, [0, 0.0])
        a[0] += 1
        a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    tot = sum(a[1] for a in agg.values()) * 1e3 / steps
    out = []
    pretty = _demangle([k for k in agg if k.startswith("_Z")])   # names rocprofv3 left mangled
    for k, (calls, sec) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        ms = sec * 1e3 / steps
        if ms < 0.02:
            continue
        e = {"name": _short(pretty.get(k, k))[:120], "ms": round(ms, 3), "calls": round(calls / steps, 2),
             "avg_us": round(sec / calls * 1e6, 1)}
        w = by_name.get(k)
        if w is not None and w["calls"] == calls:       # the same launches the work table counted
            fl, by = w["flops"], w["bytes"]
            e["tflops"] = round(fl / sec / 1e12, 1) if fl else None
            e["mfma_util"] = round(fl / sec / 1e12 / PEAK_BF16_TFLOPS, 4) if fl else None
            e["gbps"] = round(by / sec / 1e9, 1) if by else None
        out.append(e)
    return {"source": "rocprofv3 --kernel-trace of a child run of this bench (3 timed steps after 2 warm-up, "
                      "bracketed by marker kernels); flops/bytes = the library's algorithmic work "
                      "(vitmi_stats_*) of the same launches; mfma_util vs the 2.5 PF bf16 dense peak",
            "kernel_ms_per_step": round(tot, 3), "kernels": out,
            "roctx_ranges": _roctx_ranges(tmp, steps)}


def _roctx_ranges(tmp, steps):
    """The child's ROCTx ranges (vitmi_trace_push/pop around forward / backward / all-reduce /
    optimizer, recorded by rocprofv3 --marker-trace): count per step and mean HOST duration of
    each (the enqueue time of the phase; its GPU time is the parent's phases_ms)."""
    files = glob.glob(os.path.join(tmp, "kt", "**", "*marker_api_trace.csv"), recursive=True)
    if not files:
        return {"error": "no marker trace"}
    agg = {}
    for r in csv.DictReader(open(files[0])):
        name = r.get("Function") or r.get("Operation") or r.get("Name") or "?"
        if not name.startswith("vitmi:"):
            continue
        try:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
        except (KeyError, ValueError):
            continue
        a = agg.setdefault(name, [0, 0.0])
        a[0] += 1
        a[1] += d
    return {k: {"per_step": round(c / (steps + 2), 2), "host_ms_mean": round(t / c, 3)} for k, (c, t) in agg.items()}


def traffic_evidence(tmp, M):
    """HBM bytes per launch of the fc1 GEMM (+bias+GELU) from two rocprofv3 --pmc passes, with the
    gfx950 corrections of MI355X_MICROARCH.md §HBM (FETCH_SIZE KiB x2 for wide streaming reads;
    WRITE_SIZE KiB exact for 16-B stores)."""
    rp = shutil.which("rocprofv3")
    if rp is None:
        return None, "rocprofv3 not found"
    vals = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(tmp, ctr)
        cmd = [rp, "--pmc", ctr, "-d", d, "-o", "run", "--output-format", "csv", "--",
               sys.executable, os.path.join(ROOT, "tools", "gemm_one.py"), "fc1_gelu", "5"]
        rc = _run(cmd, 120, log=os.path.join(tmp, ctr + ".log"))
        files = glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True)
        if rc != 0 or not files:
            return None, f"rocprofv3 --pmc {ctr} failed (rc={rc})"
        per = {}
        for r in csv.DictReader(open(files[0])):
            name = r.get("Kernel_Name", "")
            if "gemm256_kernel" not in name or r.get("Counter_Name") != ctr:
                continue
            per[r.get("Dispatch_Id")] = per.get(r.get("Dispatch_Id"), 0.0) + float(r["Counter_Value"])
        v = list(per.values())
        if not v:
            return None, f"no gemm256 dispatch in the {ctr} pass"
        v = v[1:] or v                                   # skip the cold first launch
        vals[ctr] = sum(v) / len(v)
    fetch = vals["FETCH_SIZE"] * 1024 * 2
    write = vals["WRITE_SIZE"] * 1024
    return {"fetch": fetch, "write": write, "total": fetch + write}, None


# ------------------------------------------------------------------ the benchmark
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=["c2", "c3", "c5"], default="c3",
                    help="c3: ViT-B/16 224px bs 256/GPU (the headline metric); c5: ViT-L/16 384px bs 64/GPU "
                         "(BASELINE config 5, N = 577 tokens); c2: ViT-S/16 224px bs 128 fp32 (BASELINE config "
                         "2). c2 and c5 are secondary lines, not the headline")
    ap.add_argument("--dtype", choices=["bf16", "bf16x3", "bf16f8", "fp32"], default=None,
                    help="override the config's compute dtype (the precision knob: bf16x3 = split-bf16 forward "
                         "GEMM operands, bf16f8 = the same with the correction products in block-scaled e4m3, "
                         "fp32 = exact-fp32 MFMA everywhere; all keep the logits within 1e-3 of the CPU oracle "
                         "at ViT-B depth 12)")
    ap.add_argument("--split-qkv", choices=["auto", "yes", "no", "weight"], default="auto",
                    help="the precision knobs' qkv GEMM on split operands, plain bf16 or (bf16f8) with the "
                         "weight-side correction alone (auto: split for bf16x3, weight for bf16f8; "
                         "ViTConfig.split_qkv)")
    ap.add_argument("--batch", type=int, default=None, help="images per GPU (default 256 for c3, 64 for c5, "
                                                             "128 for c2)")
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--comm", choices=["vitmi", "torch", "gloo"], default="vitmi",
                    help="vitmi: the library's RCCL communicator (vitmi_comm_*, side stream + hipEvent gating); "
                         "torch: torch.distributed all_reduce (ProcessGroupNCCL); gloo: DIAGNOSTIC leg that runs "
                         "every multi-rank code path (bootstrap, broadcast, per-rank seeds, barriers, the "
                         "max-over-ranks time, teardown) with ranks sharing GPUs and gradients averaged through "
                         "gloo on the host (its timing means nothing)")
    ap.add_argument("--grad-dtype", choices=["fp32", "bf16"], default="fp32",
                    help="dtype of the gradient all-reduce (bf16 halves the bytes; vitmi comm only)")
    ap.add_argument("--reserve-cus", type=int, default=0,
                    help="CUs the persistent GEMM leaves to RCCL while buckets are in flight (N>1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the line's logits check against the fp32 CPU oracle (after the timed region)")
    ap.add_argument("--no-evidence", action="store_true", help="skip the rocprofv3 per-kernel / traffic legs")
    ap.add_argument("--cpu-batch", type=int, default=32)
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--no-optimizer", action="store_true", help="diagnostic only: skip Adam")
    ap.add_argument("--adam-overlap", type=int, choices=[0, 1], default=int(os.environ.get("VITMI_ADAM_OVERLAP", "0")),
                    help="vitmi Adam steps each gradient bucket on a side stream as the backward (or, on the "
                         "vitmi comm leg, its all-reduce) finishes it (optim.Adam.overlap_with)")
    ap.add_argument("--optimizer", choices=["vitmi", "torch"], default="vitmi",
                    help="vitmi: Keras Adam, one fused launch over the arena (+ bf16 shadow); torch: fused torch Adam")
    ap.add_argument("--attn-policy", type=int, default=0,
                    help="diagnostic: vitmi_attention_set_policy (0 auto: single-pass backward for N <= 224; "
                         "3: the two-kernel backward)")
    ap.add_argument("--stats-out", default=None, help=argparse.SUPPRESS)   # evidence child: work table
    ap.add_argument("--roctx", action="store_true", help="ROCTx ranges around the step's phases (vitmi.trace)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary C5 / C2 lines (child runs after the headline, N=1 only)")
    ap.add_argument("--comm-timeout", type=float, default=600.0,
                    help="seconds before a hung gradient exchange aborts the RCCL communicator (0: off)")
    args = ap.parse_args()

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    # with the vitmi communicator the process group only bootstraps (rendezvous, TCPStore,
    # barriers, the max-over-ranks time): gloo, so the job holds ONE RCCL communicator
    backend = "nccl" if args.comm == "torch" else "gloo"
    local_env = int(os.environ.get("LOCAL_RANK", "0"))
    # the gloo diagnostic leg may put several ranks on one GPU (device_count does not init HIP)
    gpu = local_env % max(1, torch.cuda.device_count()) if args.comm == "gloo" else local_env
    if world_env > 1:
        torch.cuda.set_device(gpu)
    rank, world, local = dp.init_from_env(backend)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if args.roctx:
        trace.enable()
    if args.attn_policy:
        ops.attention_set_policy(args.attn_policy)
    cfg = {"c2": config_c2, "c3": config_c3, "c5": config_c5}[args.config]()
    if args.dtype is not None:
        cfg = cfg.replace(dtype=args.dtype)
    if args.split_qkv != "auto":
        cfg = cfg.replace(split_qkv="weight" if args.split_qkv == "weight" else args.split_qkv == "yes")
    B = args.batch or {"c2": 128, "c3": 256, "c5": 64}[args.config]
    model_name = {"c2": "vit_small_16", "c3": "vit_base_16", "c5": "vit_large_16"}[args.config]
    metric = {"c3": METRIC,
              "c5": "images/sec fwd+bwd ViT-L/16 384px bs=64/GPU MI355X; % MFMA roofline (BASELINE config 5)",
              "c2": "images/sec fwd+bwd ViT-S/16 224px bs=128 fp32 MI355X; % fp32 MFMA roofline (BASELINE "
                    "config 2)"}[args.config]
    fp32 = cfg.dtype == "fp32"
    peak = PEAK_FP32_TFLOPS if fp32 else PEAK_BF16_TFLOPS

    torch.manual_seed(0)
    model = VisionTransformer(cfg).to(dev)
    model.reset_parameters(seed=0)
    comm, group, comm_leg = None, None, args.comm
    if world > 1 and args.comm == "vitmi":
        # the library's own RCCL communicator, or (RCCL refused it on some rank) torch.distributed's
        # RCCL process group: the line then says so instead of the multi-GPU run ending without one
        os.environ.setdefault("VITMI_COMM_INIT_TIMEOUT_S", "180")   # a peer that never joins: fall back
        comm, group, err = dp.comm_or_fallback(rank, world)
        if comm is None:
            comm_leg = "torch (fallback: vitmi comm init failed)"
            print(f"[bench] rank {rank}: vitmi comm init failed ({err or 'on another rank'}); "
                  f"gradients go through torch.distributed nccl (RCCL)", file=sys.stderr, flush=True)
    if world > 1 and args.grad_dtype != "fp32" and comm is None:
        raise SystemExit("bench: --grad-dtype bf16 needs the vitmi comm leg")
    red = dp.attach(model, bucket_mb=args.bucket_mb, group=group, comm=comm, grad_dtype=args.grad_dtype,
                    reserve_cus=args.reserve_cus if world > 1 else 0, timeout_s=args.comm_timeout)
    dp.broadcast_parameters(model, group=group, comm=comm)
    if args.optimizer == "vitmi":
        opt = optim.Adam(model, learning_rate=1e-3)     # keras.optimizers.Adam(1e-3), models/CvT(Par).py:458
        if args.adam_overlap:
            opt.overlap_with(red)
    else:
        try:
            opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)
        except (RuntimeError, TypeError):
            opt = torch.optim.Adam(model.parameters(), lr=1e-3, foreach=True)
    arena = model.arena()
    params = list(arena.params)

    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    img = torch.rand(B, cfg.in_chans, cfg.img_size, cfg.img_size, device=dev, generator=g)
    tgt = torch.randint(0, cfg.num_classes, (B,), device=dev, generator=g)

    phase_events = []   # per timed step: events between the phases (GPU time of each, compute stream)
    phases = ("forward", "backward", "allreduce_wait", "optimizer")

    def step(timed=False):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)] if timed else None
        if timed:
            ev[0].record()
        for p in params:                      # zero_grad(set_to_none=True): the forward zeroes the
            p.grad = None                     # arena once and AccumulateGrad keeps its views as .grad
        red.start()
        with trace.range("vitmi:forward"):
            logits = model(img)
            loss = cross_entropy(logits, tgt)
        if timed:
            ev[1].record()
        with trace.range("vitmi:backward"):
            loss.backward()
        if timed:
            ev[2].record()
        with trace.range("vitmi:allreduce"):
            red.finish()
        if timed:
            ev[3].record()
        if not args.no_optimizer:
            with trace.range("vitmi:optimizer"):
                opt.step()
        if timed:
            ev[4].record()
            phase_events.append(ev)
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    M, F_, D = B * cfg.seq_len, cfg.mlp_dim, cfg.embed_dim
    # the bf16x3 knob's fc1 GEMM runs over K' = 3D ([hi|hi|lo] x [hi|lo|hi] operand rows); the
    # bf16f8 one over D bf16 + 2D e4m3 k (2D bf16-equivalent MFMA work; its launch is keyed by D)
    KD = 3 * D if cfg.dtype == "bf16x3" else D
    KW = 2 * D if cfg.dtype == "bf16f8" else KD
    events = ops.set_probe((M, F_, KD))       # fc1 forward GEMM launches
    if args.stats_out:
        _lib.lib().vitmi_stats_enable(1)
        torch.cuda._sleep(1000)               # marker kernel: the timed region starts
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
    if args.stats_out:
        torch.cuda._sleep(1000)               # marker kernel: the timed region ended
    ops.set_probe(None)
    if args.stats_out:
        _dump_stats(args.stats_out)
    if comm is not None:
        comm.check()
    t = torch.tensor([elapsed], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = t.item()

    phases_ms = {p: round(sum(e[i].elapsed_time(e[i + 1]) for e in phase_events) / max(1, len(phase_events)), 3)
                 for i, p in enumerate(phases)}
    ms_step = elapsed / args.steps * 1e3
    imgs = B * world * args.steps / elapsed
    kern_ms = sum(a.elapsed_time(b) for a, b in events) / max(1, len(events))
    kflop = 2.0 * M * F_ * KW                 # MFMA work of the launch (3x / 2x the product's for bf16x3 / bf16f8)
    achieved = kflop / (kern_ms * 1e-3) / 1e12 if events else 0.0
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
        "dtype": cfg.dtype,
        "data": "synthetic (torch.rand images in [0,1), randint labels; random-init trunc_normal(.02) weights)",
        "config": {"workload": f"{ {'c2': 'ViT-S/16 224', 'c3': 'ViT-B/16 224', 'c5': 'ViT-L/16 384'}[args.config]}x"
                               f"{cfg.img_size}x3 fwd + CE loss + bwd"
                               + (f" + {args.grad_dtype} grad all-reduce ({comm_leg} RCCL, "
                                  f"{args.bucket_mb:g} MiB buckets)" if world > 1 else "")
                               + " + Adam step",
                   "optimizer": (("keras Adam (vitmi fused, per bucket beside the backward)" if args.adam_overlap
                                  else "keras Adam (vitmi fused)") if args.optimizer == "vitmi" else "torch fused Adam"),
                   "model": model_name, "global_batch": B * world, "seq_len": cfg.seq_len,
                   "parallelism": f"dp{world}",
                   **({"knob_qkv": _knob_qkv(cfg)} if cfg.dtype in ("bf16x3", "bf16f8") else {})},
        "roofline": {"bound": "mfma", "kernel": f"gemm fc1 fwd {'fp32' if fp32 else 'bf16'} [{M}x{F_}x{KW}] +bias+GELU"
                               + (" (bf16x3 split operands)" if KD != D else "")
                               + (" (bf16f8: bf16 hi.hi + e4m3 corrections, bf16-equivalent K)" if KW != KD else ""),
                     "achieved": round(achieved, 1), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(achieved / peak, 4), "traffic": None,
                     "launches_timed": len(events), "avg_launch_ms": round(kern_ms, 4),
                     "algorithmic_bytes": (4 if fp32 else 2) * (M * KW + F_ * KW
                                                                + (4 if KD != D else 3 if KW != KD else 2) * M * F_)},
        "optimizer_ms": phases_ms.get("optimizer"),
        "phases_ms": phases_ms,
        "step_mfma_frac": round(step_flops / (elapsed / args.steps) / 1e12 / (peak * world), 4),
        "loss": round(float(loss.item()), 5),
        "build_id": _lib.lib().vitmi_build_id().decode(),
    }
    if world > 1:
        # the multi-rank run verifies itself: what the exchange ran on (ranks and library as the
        # communicator reports them, the bucket plan, the tail launched after the backward), the
        # compute-stream time the step waited for it, and whether every rank ends with the same
        # parameters (MAX == MIN over ranks of the arena checksums)
        out["rccl"] = dp.comm_report(red)
        out["allreduce_exposed_ms"] = phases_ms.get("allreduce_wait")
        out.update(dp.replica_report(arena.flat, group))
    red.close()                               # the comm watchdog thread (the step loop is over)
    if rank == 0 and not args.no_parity and not args.stats_out:
        out["parity"] = parity_check(cfg, dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "c3":
        out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_batch, args.cpu_steps)
    if rank == 0 and world == 1 and not args.no_evidence and args.config == "c3" and not args.stats_out:
        del model, opt, arena, red, params
        torch.cuda.empty_cache()
        tmp = tempfile.mkdtemp(prefix="vitmi_bench_")
        tr, err = traffic_evidence(tmp, M)
        if tr is not None:
            out["roofline"]["traffic"] = round(tr["total"])
            out["roofline"]["traffic_detail"] = {
                "fetch_bytes": round(tr["fetch"]), "write_bytes": round(tr["write"]),
                "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over tools/gemm_one.py fc1_gelu "
                          "(this run); FETCH_SIZE KiB x2 (gfx950 wide-read half count), WRITE_SIZE KiB"}
        else:
            out["roofline"]["traffic_error"] = err
        out["per_kernel"] = per_kernel_evidence(args, tmp)
        keep = os.path.join(ROOT, "gpurun_out")
        if os.path.isdir(keep):
            shutil.copytree(tmp, os.path.join(keep, "bench_evidence"), dirs_exist_ok=True)
        shutil.rmtree(tmp, ignore_errors=True)
    if rank == 0 and world == 1 and not args.no_secondary and args.config == "c3" and not args.stats_out:
        out["secondary"] = secondary_lines()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.destroy()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def secondary_lines():
    """The precision knob's C3 lines and BASELINE configs 5 (ViT-L/16 384px bs 64, N = 577) and 2
    (ViT-S/16 224px bs 128 fp32) on the driver's clock: child runs of this bench after the headline;
    the headline `value` stays C3."""
    out = {}
    # the precision knob first (ViT-B/16 C3 with logits within 1e-3 of the fp32 reference: split-bf16
    # forward operands with the corrections in e4m3 (bf16f8) or bf16 (bf16x3)), then C5 and C2, then
    # exact-fp32 arithmetic throughout
    # (bf16f8's qkv GEMM: by default with the weight-side correction alone; the plain-qkv line beside it
    # is the faster setting with 4-5x less logits margin)
    runs = {"c3_bf16f8": ["--config", "c3", "--dtype", "bf16f8", "--steps", "10", "--warmup", "3"],
            "c3_bf16f8_qkv_plain": ["--config", "c3", "--dtype", "bf16f8", "--split-qkv", "no", "--steps", "10",
                                    "--warmup", "3"],
            "c3_bf16x3": ["--config", "c3", "--dtype", "bf16x3", "--steps", "10", "--warmup", "3"],
            # the north star's host-side optimizer: torch's fused Adam on the parameters (the
            # headline runs the reference's Keras Adam as one vitmi launch)
            "c3_torch_adam": ["--config", "c3", "--optimizer", "torch", "--steps", "10", "--warmup", "3"],
            "c5": ["--config", "c5", "--steps", "10", "--warmup", "3"],
            "c2": ["--config", "c2", "--steps", "10", "--warmup", "3"],
            "c3_fp32": ["--config", "c3", "--dtype", "fp32", "--steps", "3", "--warmup", "1"]}
    for cfg, extra in runs.items():
        log = os.path.join(tempfile.gettempdir(), f"vitmi_secondary_{cfg}.log")
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), *extra, "--no-evidence", "--no-cpu-baseline",
               "--no-secondary"]
        rc = _run(cmd, 300, log=log)
        line = None
        if rc == 0:
            for ln in open(log):
                if ln.startswith("{"):
                    line = json.loads(ln)
        if line is None:
            out[cfg] = {"error": f"child rc={rc}"}
            continue
        out[cfg] = {k: line[k] for k in ("metric", "value", "unit", "ms_per_step", "step_mfma_frac", "dtype",
                                         "phases_ms", "optimizer_ms") if k in line}
        if "parity" in line:
            out[cfg]["parity"] = line["parity"]
        out[cfg]["config"] = line["config"]
        r = line["roofline"]
        out[cfg]["dominant_kernel"] = {"kernel": r["kernel"], "avg_launch_ms": r["avg_launch_ms"],
                                       "achieved_tflops": r["achieved"], "peak": r["peak"], "frac": r["frac"]}
    return out


def _dump_stats(path):
    lib = _lib.lib()
    import ctypes
    n = lib.vitmi_stats_count()
    ks = []
    for i in range(n):
        name = ctypes.create_string_buffer(1024)
        calls, fl, by = ctypes.c_int64(0), ctypes.c_double(0), ctypes.c_double(0)
        lib.vitmi_stats_get(i, name, 1024, ctypes.byref(calls), ctypes.byref(fl), ctypes.byref(by))
        ks.append({"name": name.value.decode(), "calls": calls.value, "flops": fl.value, "bytes": by.value})
    lib.vitmi_stats_enable(0)
    with open(path, "w") as f:
        json.dump({"kernels": ks}, f)


if __name__ == "__main__":
    main()
