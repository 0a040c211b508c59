"""The reference's optimizer (keras Adam, models/CvT(Par).py:458-460) and LR schedule
(:357-360) on the fused vitmi kernel vs oracle/optim_ref.py: bit-exact fp32 (the kernel and
the oracle do the same IEEE-rounded ops in the same order)."""
import numpy as np
import pytest
import torch

from oracle import optim_ref
from vitmi import optim

DEV = "cuda"


def test_alpha_and_schedule_host():
    for t in (1, 2, 10, 1000):
        assert optim.keras_alpha(1e-3, 0.9, 0.999, t) == float(optim_ref.keras_alpha(1e-3, 0.9, 0.999, t))
    lr = 1e-3
    for e in range(0, 201):
        lr_ref = optim_ref.lr_scheduler(e, lr)
        lr = optim.keras_step_decay(e, lr)
        assert lr == lr_ref
    assert abs(lr - 1e-3 * 0.8 ** 4) < 1e-15


@pytest.mark.gpu
@pytest.mark.parametrize("n,scale", [(1, 1.0), (7, 1.0), (1_000_003, 1.0), (4096, 0.25)])
def test_adam_per_tensor_bit_exact(n, scale):
    g = torch.Generator().manual_seed(n)
    p = torch.randn(n, generator=g)
    ref = (p.numpy().copy(), np.zeros(n, np.float32), np.zeros(n, np.float32))
    pd = p.to(DEV).requires_grad_(True)
    opt = optim.Adam([pd], learning_rate=1e-3, grad_scale=scale)
    for t in range(1, 4):
        gr = torch.randn(n, generator=g) * (10.0 ** (t - 2))
        pd.grad = gr.to(DEV)
        opt.step()
        ref = optim_ref.adam_step(ref[0], gr.numpy(), ref[1], ref[2], 1e-3, t, grad_scale=scale)
        torch.cuda.synchronize()
        assert np.array_equal(pd.detach().cpu().numpy(), ref[0]), t
        assert np.array_equal(opt._m[0].cpu().numpy(), ref[1])
        assert np.array_equal(opt._v[0].cpu().numpy(), ref[2])


@pytest.mark.gpu
def test_adam_arena_single_launch_and_bf16_shadow():
    from vitmi.config import ViTConfig
    from vitmi.modules import VisionTransformer, cross_entropy
    cfg = ViTConfig(img_size=32, patch_size=8, in_chans=3, num_classes=3, embed_dim=128, depth=2, num_heads=2,
                    dtype="bf16")
    model = VisionTransformer(cfg).to(DEV)
    model.reset_parameters(seed=1)
    opt = optim.Adam(model, learning_rate=1e-3)
    arena = model.arena()
    p0 = arena.flat.cpu().numpy().copy()
    m0 = np.zeros_like(p0)
    v0 = np.zeros_like(p0)
    g = torch.Generator().manual_seed(2)
    img = torch.rand(4, 3, 32, 32, generator=g).to(DEV)
    tgt = torch.randint(0, 3, (4,), generator=g).to(DEV)
    for t in (1, 2):
        opt.zero_grad()
        cross_entropy(model(img), tgt).backward()
        grad = arena.grad.cpu().numpy().copy()
        opt.step()
        torch.cuda.synchronize()
        p0, m0, v0 = optim_ref.adam_step(p0, grad, m0, v0, 1e-3, t)
        assert np.array_equal(arena.flat.cpu().numpy(), p0)
        # the shadow the next forward's GEMMs read == bf16(updated params), without a cast pass
        assert torch.equal(arena.flat_lp, arena.flat.to(torch.bfloat16))
        v_before = arena._lp_version
        arena.refresh_lp()
        assert arena._lp_version == v_before
    # an in-place torch update of a parameter invalidates the shadow
    with torch.no_grad():
        model.head.weight.add_(1.0)
    arena.refresh_lp()
    assert torch.equal(arena.flat_lp, arena.flat.to(torch.bfloat16))


@pytest.mark.gpu
def test_adam_per_tensor_on_arena_params_refreshes_bf16_shadow():
    """Adam built from a parameter LIST of an arena-backed bf16 ViT (the per-tensor
    path, raw-pointer writes) must still invalidate the arena's bf16 operand shadow, so the
    next forward's GEMMs read the updated weights."""
    from vitmi.config import ViTConfig
    from vitmi.modules import VisionTransformer, cross_entropy
    cfg = ViTConfig(img_size=32, patch_size=8, in_chans=3, num_classes=2, embed_dim=128, depth=1, num_heads=2,
                    dtype="bf16")
    model = VisionTransformer(cfg).to(DEV)
    model.reset_parameters(seed=3)
    g = torch.Generator().manual_seed(4)
    img = torch.rand(4, 3, 32, 32, generator=g).to(DEV)
    tgt = torch.randint(0, 2, (4,), generator=g).to(DEV)
    cross_entropy(model(img), tgt).backward()          # builds the arena and its shadow
    arena = model.arena()
    opt = optim.Adam(list(model.parameters()), learning_rate=1e-2)
    assert opt._arena is None                           # the per-tensor path
    opt.step()
    model(img)                                          # the forward refreshes the shadow if stale
    torch.cuda.synchronize()
    assert torch.equal(arena.flat_lp, arena.flat.to(torch.bfloat16))


@pytest.mark.gpu
def test_adam_arena_skips_frozen_parameters():
    """a parameter frozen after it has been trained (stale m / v) and a parameter whose
    gradient is None after zero_grad(set_to_none) stay bit-identical through the fused arena
    step, as with torch / Keras; the others still follow the float32 oracle bit for bit, and the
    bf16 shadow stays equal to bf16(params)."""
    from vitmi.config import ViTConfig
    from vitmi.modules import VisionTransformer, cross_entropy
    cfg = ViTConfig(img_size=32, patch_size=8, in_chans=3, num_classes=2, embed_dim=128, depth=2, num_heads=2,
                    dtype="bf16")
    model = VisionTransformer(cfg).to(DEV)
    model.reset_parameters(seed=5)
    opt = optim.Adam(model, learning_rate=1e-3)
    arena = model.arena()
    g = torch.Generator().manual_seed(6)
    img = torch.rand(4, 3, 32, 32, generator=g).to(DEV)
    tgt = torch.randint(0, 2, (4,), generator=g).to(DEV)
    opt.zero_grad()
    cross_entropy(model(img), tgt).backward()
    opt.step()                                           # every parameter trained once: m, v != 0
    frozen = model.blocks[0].mlp.fc1.weight
    frozen.requires_grad_(False)
    before = {k: p.detach().clone() for k, p in model.named_parameters()}
    m0, v0 = opt._m.cpu().numpy().copy(), opt._v.cpu().numpy().copy()
    p0 = arena.flat.cpu().numpy().copy()
    opt.zero_grad()
    cross_entropy(model(img), tgt).backward()
    head_b = model.head.bias
    head_b.grad = None                                   # a parameter without a gradient this step
    grad = arena.grad.cpu().numpy().copy()
    opt.step()
    torch.cuda.synchronize()
    assert torch.equal(frozen.detach(), before["blocks.0.mlp.fc1.weight"])
    assert torch.equal(head_b.detach(), before["head.bias"])
    ref, _, _ = optim_ref.adam_step(p0, grad, m0, v0, 1e-3, 2)
    keep = np.ones(arena.numel, dtype=bool)
    for p in (frozen, head_b):
        o = arena.offsets[id(p)]
        keep[o:o + p.numel()] = False
    assert np.array_equal(arena.flat.cpu().numpy()[keep], ref[keep])
    assert torch.equal(arena.flat_lp, arena.flat.to(torch.bfloat16))


@pytest.mark.gpu
def test_adam_overlap_matches_single_launch_bitwise():
    """Adam.overlap_with (world 1): the buckets the backward finishes are stepped on a side
    stream during it, the rest in step(); parameters, moments and the bf16 shadow equal the plain
    single launch bit for bit over three steps.  A frozen parameter turns the overlap off for the
    step (the plain path's skip rule)."""
    from vitmi import dp
    from vitmi.config import ViTConfig
    from vitmi.modules import VisionTransformer, cross_entropy
    cfg = ViTConfig(img_size=32, patch_size=8, in_chans=3, num_classes=3, embed_dim=128, depth=3, num_heads=2,
                    dtype="bf16")
    g = torch.Generator().manual_seed(7)
    img = torch.rand(4, 3, 32, 32, generator=g).to(DEV)
    tgt = torch.randint(0, 3, (4,), generator=g).to(DEV)
    runs = []
    for overlap in (False, True):
        model = VisionTransformer(cfg).to(DEV)
        model.reset_parameters(seed=8)
        red = dp.attach(model, bucket_mb=0.25)
        opt = optim.Adam(model, learning_rate=1e-3)
        if overlap:
            opt.overlap_with(red)
        arena = model.arena()
        side = []
        for t in range(4):
            if t == 3:
                model.blocks[1].attn.proj.weight.requires_grad_(False)
            opt.zero_grad()
            red.start()
            cross_entropy(model(img), tgt).backward()
            red.finish()
            if overlap:
                side.append(opt._ov["done"])
            opt.step()
        torch.cuda.synchronize()
        runs.append((arena.flat.clone(), opt._m.clone(), opt._v.clone(), arena.flat_lp.clone()))
        if overlap:
            assert len(red.bounds) >= 4
            # steps 0-2: the buckets went on the side stream as the backward finished them (all
            # of them: the embedding's hooks close the backward); step 3 (a frozen weight): none
            assert all(d == arena.numel for d in side[:3]), side
            assert side[3] == 0, side
    for a, b in zip(*runs):
        assert torch.equal(a, b)
    assert torch.equal(runs[1][3], runs[1][0].to(torch.bfloat16))
