"""The nn.Module surface's parameter-gradient contract on the GPU.

SURVEY.md §8(b): "Parameters are plain nn.Parameters, so torch.optim, state_dict, and DDP-style
hooks work unchanged"; the reference's PyTorch twin accumulates its parameter gradients through
autograd (old_codes/MS_CvT.py:289-333).  vitmi's fused Functions return every parameter's
gradient to autograd (vitmi/grads.py), so:
  * a user model of two vitmi Blocks wrapped in torch.nn.parallel.DistributedDataParallel
    (gloo, two ranks on one GPU) gets the oracle's full-batch gradients;
  * register_post_accumulate_grad_hook fires once per parameter and backward;
  * torch.autograd.grad(loss, params) returns the oracle's gradients and leaves .grad alone;
  * a frozen parameter (requires_grad=False) gets no .grad, the others are unchanged;
  * a second backward without zero_grad accumulates;
  * inside VisionTransformer the gradients still land in the parameter arena with no copy
    (AccumulateGrad keeps the arena view as .grad).

Tolerances: fp32 grads ||d||/||g|| <= 1e-4 (SURVEY.md §8d fp32 bound), bf16 <= 2e-2."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

from oracle import vit_ref
from vitmi.config import ViTConfig
from vitmi.modules import Block, VisionTransformer, cross_entropy

pytestmark = pytest.mark.gpu

D, H, N, B = 128, 2, 17, 4
GTOL = {"fp32": 1e-4, "bf16": 2e-2}


def _cfg(dtype="fp32", depth=2):
    return ViTConfig(img_size=32, patch_size=8, embed_dim=D, depth=depth, num_heads=H, num_classes=2, dtype=dtype)


class _Stack(nn.Module):
    def __init__(self, dtype):
        super().__init__()
        self.b0 = Block(D, H, dtype=dtype)
        self.b1 = Block(D, H, dtype=dtype)

    def forward(self, x):
        return self.b1(self.b0(x, 4, 4) * 1.5 - 0.25, 4, 4)


def _ref_stack(x, lv, cfg):
    return vit_ref.block(vit_ref.block(x, lv, 0, cfg) * 1.5 - 0.25, lv, 1, cfg)


def _stack_model(dtype, params):
    m = _Stack(dtype).cuda()
    with torch.no_grad():
        for i, b in enumerate((m.b0, m.b1)):
            for k, p in b.named_parameters():
                p.copy_(params[f"blocks.{i}.{k}"].reshape(p.shape))
    return m


def _names(m):
    return {p: f"blocks.{0 if k.startswith('b0.') else 1}.{k[3:]}" for k, p in m.named_parameters()}


def _ref_grads(x, tgt, params, cfg):
    lv = {k: v.detach().clone().requires_grad_(True) for k, v in params.items() if k.startswith("blocks.")}
    ((_ref_stack(x, lv, cfg) - tgt) ** 2).mean().backward()
    return {k: v.grad for k, v in lv.items()}


def _data(seed=3):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(B, N, D, generator=g), torch.randn(B, N, D, generator=g)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_hooks_fire_once_and_autograd_grad_matches_oracle(dtype):
    cfg = _cfg(dtype)
    params = vit_ref.init_params(cfg, seed=4)
    x, tgt = _data()
    ref = _ref_grads(x, tgt, params, cfg)
    m = _stack_model(dtype, params)
    names = _names(m)
    fired = {n: 0 for n in names.values()}
    handles = [p.register_post_accumulate_grad_hook(lambda t, n=names[p]: fired.__setitem__(n, fired[n] + 1))
               for p in m.parameters()]
    seen = {}
    handles += [p.register_hook(lambda g, n=names[p]: seen.__setitem__(n, g.detach().clone())) for p in m.parameters()]
    ((m(x.cuda()) - tgt.cuda()) ** 2).mean().backward()
    assert all(v == 1 for v in fired.values()), fired
    for p, n in names.items():
        assert vit_ref.rel_err(p.grad.cpu(), ref[n]) <= GTOL[dtype], n
        assert torch.equal(seen[n], p.grad), n            # the tensor hook saw the gradient
    for h in handles:
        h.remove()
    # torch.autograd.grad: the same gradients, .grad untouched
    for p in m.parameters():
        p.grad = None
    ps = list(m.parameters())
    gs = torch.autograd.grad(((m(x.cuda()) - tgt.cuda()) ** 2).mean(), ps)
    for p, gr in zip(ps, gs):
        assert p.grad is None
        assert vit_ref.rel_err(gr.cpu(), ref[names[p]]) <= GTOL[dtype], names[p]


def test_frozen_parameter_gets_no_grad_and_second_backward_accumulates():
    cfg = _cfg("fp32")
    params = vit_ref.init_params(cfg, seed=5)
    x, tgt = _data(6)
    ref = _ref_grads(x, tgt, params, cfg)
    m = _stack_model("fp32", params)
    m.b0.norm1.requires_grad_(False)
    m.b1.attn.qkv.bias.requires_grad_(False)
    ((m(x.cuda()) - tgt.cuda()) ** 2).mean().backward()
    names = _names(m)
    for p, n in names.items():
        if not p.requires_grad:
            assert p.grad is None, n
        else:
            assert vit_ref.rel_err(p.grad.cpu(), ref[n]) <= 1e-4, n
    first = {n: p.grad.clone() for p, n in names.items() if p.grad is not None}
    ((m(x.cuda()) - tgt.cuda()) ** 2).mean().backward()       # no zero_grad: accumulate
    for p, n in names.items():
        if p.grad is not None:
            assert vit_ref.rel_err(p.grad, 2 * first[n]) <= 1e-6, n


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_vit_arena_grads_are_returned_without_copies(dtype):
    """VisionTransformer: every .grad is its parameter's view of the arena (AccumulateGrad kept
    the returned view), hooks fire once, the gradients are the oracle's; autograd.grad and a
    frozen norm1 behave as for any torch model; a second backward accumulates into the arena."""
    cfg = _cfg(dtype, depth=3)
    params = vit_ref.init_params(cfg, seed=1)
    img, tgt = vit_ref.synthetic_batch(cfg, 4)
    _, _, ref = vit_ref.forward_backward(img, tgt, params, cfg)
    model = VisionTransformer(cfg).cuda()
    model.load_param_dict(params)
    arena = model.arena()
    names = {p: k for k, p in model.named_parameters()}
    fired = {k: 0 for k in names.values()}
    hs = [p.register_post_accumulate_grad_hook(lambda t, k=names[p]: fired.__setitem__(k, fired[k] + 1))
          for p in model.parameters()]
    cross_entropy(model(img.cuda()), tgt.cuda()).backward()
    assert all(v == 1 for v in fired.values()), fired
    for p, k in names.items():
        assert p.grad.data_ptr() == arena.view(arena.grad, p).data_ptr(), k
        assert vit_ref.rel_err(p.grad.cpu(), ref[k]) <= GTOL[dtype], k
    for h in hs:
        h.remove()
    first = arena.grad.clone()
    cross_entropy(model(img.cuda()), tgt.cuda()).backward()     # accumulate
    assert vit_ref.rel_err(arena.grad, 2 * first) <= 1e-6
    for p, k in names.items():
        assert p.grad.data_ptr() == arena.view(arena.grad, p).data_ptr(), k
    # autograd.grad leaves .grad alone
    for p in model.parameters():
        p.grad = None
    ps = list(model.parameters())
    gs = torch.autograd.grad(cross_entropy(model(img.cuda()), tgt.cuda()), ps)
    for p, gr in zip(ps, gs):
        assert p.grad is None
        assert vit_ref.rel_err(gr.cpu(), ref[names[p]]) <= GTOL[dtype], names[p]
    # a frozen LayerNorm
    frozen = model.blocks[1].norm1
    frozen.requires_grad_(False)
    cross_entropy(model(img.cuda()), tgt.cuda()).backward()
    assert frozen.weight.grad is None and frozen.bias.grad is None
    for p, k in names.items():
        if p.requires_grad:
            assert vit_ref.rel_err(p.grad.cpu(), ref[k]) <= GTOL[dtype], k


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ddp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        cfg = _cfg("fp32")
        params = vit_ref.init_params(cfg, seed=7)
        x, tgt = _data(8)
        m = _stack_model("fp32", params)
        ddp = torch.nn.parallel.DistributedDataParallel(m, device_ids=None, bucket_cap_mb=0.1)
        half = B // world
        lo = rank * half
        y = ddp(x[lo:lo + half].cuda())
        ((y - tgt[lo:lo + half].cuda()) ** 2).mean().backward()
        torch.cuda.synchronize()
        names = _names(m)
        q.put((rank, {names[p]: p.grad.cpu().numpy() for p in m.parameters()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_ddp_two_ranks_matches_oracle_full_batch():
    """torch.nn.parallel.DistributedDataParallel over a model of two vitmi Blocks: DDP's reducer
    hooks see the returned gradients and average them; each rank ends with the oracle's
    full-batch gradient (two equal halves, mean losses)."""
    cfg = _cfg("fp32")
    params = vit_ref.init_params(cfg, seed=7)
    x, tgt = _data(8)
    ref = _ref_grads(x, tgt, params, cfg)
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ddp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=200) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for r in range(world):
        for n, g in res[r].items():
            assert vit_ref.rel_err(torch.from_numpy(g), ref[n]) <= 1e-4, (r, n)
