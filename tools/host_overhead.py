"""Host enqueue cost of one bench step (ViT-B/16 bs 256, vitmi Adam): the GPU is parked behind a
long sleep kernel, so the host's time to issue the step's ~700 launches is measured alone, then
compared with the step's GPU time.  usage: python tools/host_overhead.py [B]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402

from vitmi import optim  # noqa: E402
from vitmi.config import preset  # noqa: E402
from vitmi.modules import VisionTransformer, cross_entropy  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    cfg = preset("vit_base_16", img_size=224, num_classes=1000, dtype="bf16")
    model = VisionTransformer(cfg).cuda()
    model.reset_parameters(seed=0)
    opt = optim.Adam(model, learning_rate=1e-3)
    params = list(model.arena().params)
    img = torch.rand(B, 3, 224, 224, device="cuda")
    tgt = torch.randint(0, 1000, (B,), device="cuda")

    def step():
        for p in params:
            p.grad = None
        cross_entropy(model(img), tgt).backward()
        opt.step()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        step()
    e1.record()
    torch.cuda.synchronize()
    gpu_ms = e0.elapsed_time(e1) / 5
    for i in range(3):
        torch.cuda._sleep(2_000_000_000)     # ~1 s of GPU time: the queue holds everything issued below
        t0 = time.perf_counter()
        step()
        host_ms = (time.perf_counter() - t0) * 1e3
        torch.cuda.synchronize()
        print(f"round {i}: host enqueue {host_ms:.2f} ms per step, GPU {gpu_ms:.2f} ms per step", flush=True)


if __name__ == "__main__":
    main()
