"""torch.profiler view of the bench step (ViT-B/16, bs from argv): which host call sites
launch the non-vitmi kernels (fills, copies).  usage: python tools/torch_prof.py [batch] [dtype] [dp]
("dp": the step as bench.py runs it, with vitmi.dp.attach's reducer and readiness hooks at N = 1)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from vitmi import dp, optim  # noqa: E402
from vitmi.config import config_c3  # noqa: E402
from vitmi.modules import VisionTransformer, cross_entropy  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    cfg = config_c3(dtype=sys.argv[2]) if len(sys.argv) > 2 else config_c3()
    model = VisionTransformer(cfg).cuda()
    model.reset_parameters(seed=0)
    opt = optim.Adam(model, learning_rate=1e-3)
    red = dp.attach(model) if len(sys.argv) > 3 and sys.argv[3] == "dp" else None
    params = list(model.arena().params)
    img = torch.rand(B, 3, 224, 224, device="cuda")
    tgt = torch.randint(0, cfg.num_classes, (B,), device="cuda")

    def step():
        if red is None:
            opt.zero_grad()
        else:                     # as bench.py's step
            for p in params:
                p.grad = None
            red.start()
        loss = cross_entropy(model(img), tgt)
        loss.backward()
        if red is not None:
            red.finish()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(2):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=25), flush=True)
    for ev in prof.key_averages(group_by_stack_n=8):
        if any(t in ev.key for t in ("fill", "copy", "Fill", "Copy", "zero")):
            print(f"== {ev.key}  count {ev.count}  cuda {ev.device_time_total:.0f} us")
            for fr in ev.stack[:8]:
                print("     ", fr)


if __name__ == "__main__":
    main()
