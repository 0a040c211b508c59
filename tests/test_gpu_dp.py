"""Data parallelism through the HIP path: two ranks on the one GPU of the test box.

Each rank runs the vitmi forward+backward on half of the batch, and the gradient reducer's
hooks fire from inside the fused block backward. The bucketed all-reduce then averages the flat
gradient buffer on the GPU. The result must equal the oracle's full-batch gradient (mean loss ⇒
mean of the two half-batch gradients). This is the reference's MirroredStrategy semantics
(old_codes/BayConvT(Par)(Muti).py:16-19).

Two ranks cannot share one GPU under RCCL, so these ranks use gloo, which moves the CUDA
tensors through host memory. The hook/bucket/stream-ordering logic under test is identical
to the RCCL path. RCCL itself is exercised by the driver's multi-GPU bench."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg():
    from vitmi.config import ViTConfig
    return ViTConfig(img_size=32, patch_size=8, embed_dim=128, depth=3, num_heads=2, num_classes=3,
                     dtype="fp32")


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import vit_ref
        from vitmi import dp
        from vitmi.modules import VisionTransformer, cross_entropy
        cfg = _cfg()
        params = vit_ref.init_params(cfg, seed=3)
        img, tgt = vit_ref.synthetic_batch(cfg, 8, seed=11)
        per = img.shape[0] // world
        model = VisionTransformer(cfg).cuda()
        model.load_param_dict(params)
        if rank == 1:                     # broadcast must overwrite rank 1's params
            with torch.no_grad():
                model.arena().flat.mul_(0.5)
        dp.broadcast_parameters(model)
        red = dp.attach(model, bucket_mb=0.25)          # several buckets -> overlapped launches
        model.arena().grad.zero_()
        red.start()
        lo = rank * per
        loss = cross_entropy(model(img[lo:lo + per].cuda()), tgt[lo:lo + per].cuda())
        loss.backward()
        early = sum(1 for r, _ in red.launch_log if r < model.arena().numel)
        red.finish()
        torch.cuda.synchronize()
        # numpy arrays pickle by value (torch tensors would travel as fds that vanish with
        # this process)
        grads = {k: p.grad.detach().cpu().numpy() for k, p in model.named_parameters()}
        q.put((rank, dict(grads=grads, early=early, nb=len(red.bounds))))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dp_two_ranks_match_full_batch_oracle():
    from oracle import vit_ref
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cfg = _cfg()
    params = vit_ref.init_params(cfg, seed=3)
    img, tgt = vit_ref.synthetic_batch(cfg, 8, seed=11)
    _, _, g_ref = vit_ref.forward_backward(img, tgt, params, cfg)
    for r in range(world):
        o = res[r]
        assert o["nb"] > 2
        assert o["early"] >= 1, "no bucket was launched during the backward (no overlap)"
        for k, ref in g_ref.items():
            assert vit_ref.rel_err(torch.from_numpy(o["grads"][k]), ref) <= 1e-4, (r, k)
    for k in g_ref:
        assert (res[0]["grads"][k] == res[1]["grads"][k]).all(), k
