"""The drop-in nn.Module surface on its own: ConvEmbed, Attention, Mlp and Block built
standalone (not inside VisionTransformer), with the call signatures of the reference's
PyTorch twin (old_codes/MS_CvT.py: ConvEmbed.forward(x) :360 -> [B,D,h,w],
Attention.forward(x, h, w) :190, Mlp.forward(x) :53-74, Block.forward(x, h, w) :325),
checked forward and backward against the CPU oracle (oracle/vit_ref.py: embed / attention
/ mlp / block).  The last test is a user-written training loop that stacks two Blocks with
torch ops between and around them, so every incoming gradient of a vitmi backward comes from
a torch op and the caching allocator recycles gradient buffers between steps.

Tolerances: fp32 outputs max-abs <= 1e-4 x scale, grads ||d||/||g|| <= 1e-4; bf16 outputs
<= 2e-2 relative to the output scale, grads <= 2e-2 (SURVEY.md §8d bf16 bound)."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from oracle import vit_ref
from vitmi.config import ViTConfig
from vitmi.modules import LP_STATS, Attention, Block, ConvEmbed, Mlp

pytestmark = pytest.mark.gpu

D, H, N, B = 128, 2, 17, 3
TOL = {"fp32": (1e-4, 1e-4), "bf16": (2e-2, 2e-2)}


def _cfg(dtype, **kw):
    return ViTConfig(img_size=32, patch_size=8, embed_dim=D, depth=2, num_heads=H, num_classes=2,
                     dtype=dtype, **kw)


def _load(mod: nn.Module, params, prefix):
    with torch.no_grad():
        for k, p in mod.named_parameters():
            p.copy_(params[prefix + k].reshape(p.shape))


def _leaves(params):
    return {k: v.detach().clone().requires_grad_(True) for k, v in params.items()}


def _check(name, got, ref, tol):
    scale = max(1.0, ref.abs().max().item())
    err = (got.detach().float().cpu() - ref.detach()).abs().max().item()
    assert err <= tol * scale, f"{name}: max-abs {err:.3e} > {tol} x {scale:.2f}"


def _check_grads(mod, leaves, prefix, tol):
    for k, p in mod.named_parameters():
        r = vit_ref.rel_err(p.grad.cpu(), leaves[prefix + k].grad)
        assert r <= tol, f"{k}: grad rel {r:.3e} > {tol}"


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_conv_embed_standalone(dtype):
    """ConvEmbed.forward(x[B,C,H,W]) -> [B,D,h,w] (MS_CvT.py:360-369), Conv2D k=s=P
    (models/CvT(Par).py:203-212); weight/bias grads from an upstream torch gradient."""
    otol, gtol = TOL[dtype]
    cfg = _cfg(dtype)
    params = vit_ref.init_params(cfg, seed=2)
    img, _ = vit_ref.synthetic_batch(cfg, B, seed=4)
    emb = ConvEmbed(cfg.patch_size, cfg.in_chans, D, dtype=dtype).cuda()
    _load(emb, params, "patch_embed.")
    y = emb(img.cuda())
    G = cfg.img_size // cfg.patch_size
    assert tuple(y.shape) == (B, D, G, G)
    lv = _leaves(params)
    ref = F.conv2d(img, lv["patch_embed.proj.weight"], lv["patch_embed.proj.bias"], stride=cfg.patch_size)
    _check("conv_embed", y, ref, otol)
    gy = torch.randn(ref.shape, generator=torch.Generator().manual_seed(9))
    ref.backward(gy)
    y.backward(gy.cuda())
    _check_grads(emb, lv, "patch_embed.", gtol)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("knobs", [dict(), dict(qkv_bias=False, attn_scale="dim")])
def test_attention_standalone(dtype, knobs):
    """Attention.forward(x, h, w) (MS_CvT.py:190-212; ConvAttention.call with 'linear'
    projections, models/CvT(Par).py:144-191): output, d x and every parameter grad."""
    otol, gtol = TOL[dtype]
    cfg = _cfg(dtype, **knobs)
    params = vit_ref.init_params(cfg, seed=3)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, N, D, generator=g)
    attn = Attention(D, H, cfg.qkv_bias, cfg.attn_scale, dtype).cuda()
    _load(attn, params, "blocks.0.attn.")
    xg = x.cuda().requires_grad_(True)
    y = attn(xg, 4, 4)
    lv = _leaves(params)
    xr = x.clone().requires_grad_(True)
    ref = vit_ref.attention(xr, lv, "blocks.0.", cfg)
    _check("attention", y, ref, otol)
    gy = torch.randn(ref.shape, generator=g)
    ref.backward(gy)
    y.backward(gy.cuda())
    assert vit_ref.rel_err(xg.grad.cpu(), xr.grad) <= gtol
    _check_grads(attn, lv, "blocks.0.attn.", gtol)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_mlp_standalone(dtype):
    """Mlp.forward(x): Dense(4D, exact GELU) -> Dense(D) (models/CvT(Par).py:253-258)."""
    otol, gtol = TOL[dtype]
    cfg = _cfg(dtype)
    params = vit_ref.init_params(cfg, seed=4)
    g = torch.Generator().manual_seed(6)
    x = torch.randn(B, N, D, generator=g)
    mlp = Mlp(D, cfg.mlp_dim, dtype).cuda()
    _load(mlp, params, "blocks.1.mlp.")
    xg = x.cuda().requires_grad_(True)
    y = mlp(xg)
    lv = _leaves(params)
    xr = x.clone().requires_grad_(True)
    ref = vit_ref.mlp(xr, lv, "blocks.1.")
    _check("mlp", y, ref, otol)
    gy = torch.randn(ref.shape, generator=g)
    ref.backward(gy)
    y.backward(gy.cuda())
    assert vit_ref.rel_err(xg.grad.cpu(), xr.grad) <= gtol
    _check_grads(mlp, lv, "blocks.1.mlp.", gtol)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("tie", [False, True])
def test_block_standalone(dtype, tie):
    """Block.forward(x, h, w) (MS_CvT.py:325-333; ConvTransformerBlock.call,
    models/CvT(Par).py:261-289), separate or Keras-tied norms."""
    otol, gtol = TOL[dtype]
    cfg = _cfg(dtype, tie_norms=tie)
    params = vit_ref.init_params(cfg, seed=5)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(B, N, D, generator=g)
    blk = Block(D, H, cfg.mlp_ratio, cfg.qkv_bias, cfg.ln_eps, cfg.attn_scale, tie, dtype).cuda()
    _load(blk, params, "blocks.0.")
    xg = x.cuda().requires_grad_(True)
    y = blk(xg, 4, 4)
    lv = _leaves(params)
    xr = x.clone().requires_grad_(True)
    ref = vit_ref.block(xr, lv, 0, cfg)
    _check("block", y, ref, otol)
    gy = torch.randn(ref.shape, generator=g)
    ref.backward(gy)
    y.backward(gy.cuda())
    assert vit_ref.rel_err(xg.grad.cpu(), xr.grad) <= gtol
    _check_grads(blk, lv, "blocks.0.", gtol)


class _UserStack(nn.Module):
    """A user's model: torch ops between and around two vitmi Blocks."""

    def __init__(self, dtype):
        super().__init__()
        self.b0 = Block(D, H, dtype=dtype)
        self.b1 = Block(D, H, dtype=dtype)

    def forward(self, x):
        t = self.b0(x, 4, 4)
        t = t * 1.5 - 0.25                  # torch op between the blocks
        return self.b1(t, 4, 4)


def _ref_stack(x, lv, cfg):
    t = vit_ref.block(x, lv, 0, cfg)
    t = t * 1.5 - 0.25
    return vit_ref.block(t, lv, 1, cfg)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_user_stacked_blocks_training_loop(dtype):
    """Three SGD steps of a user-stacked 2-block model whose loss is a torch op: every
    step's gradients match the oracle's.  The bf16 copies a backward hands up the chain are
    owned by the gradient tensor object, so a gradient buffer the allocator recycles in a
    later step can never pick up a stale copy (the round-2 address-keyed table could)."""
    otol, gtol = TOL[dtype]
    cfg = _cfg(dtype)
    params = vit_ref.init_params(cfg, seed=8)
    model = _UserStack(dtype).cuda()
    for i, b in enumerate((model.b0, model.b1)):
        _load(b, params, f"blocks.{i}.")
    opt = torch.optim.SGD(model.parameters(), lr=0.5)
    lv = _leaves({k: v for k, v in params.items() if k.startswith("blocks.")})
    gen = torch.Generator().manual_seed(10)
    for step in range(3):
        x = torch.randn(B, N, D, generator=gen)
        tgt = torch.randn(B, N, D, generator=gen)
        opt.zero_grad()
        y = model(x.cuda())
        loss = ((y - tgt.cuda()) ** 2).mean()      # the gradient into b1 comes from torch ops
        loss.backward()
        for v in lv.values():
            v.grad = None
        ref = _ref_stack(x, lv, cfg)
        ((ref - tgt) ** 2).mean().backward()
        _check(f"step {step} output", y, ref, otol)
        for i, b in enumerate((model.b0, model.b1)):
            for k, p in b.named_parameters():
                r = vit_ref.rel_err(p.grad.cpu(), lv[f"blocks.{i}.{k}"].grad)
                assert r <= gtol, f"step {step} b{i}.{k}: grad rel {r:.3e}"
        opt.step()
        with torch.no_grad():
            for v in lv.values():
                v -= 0.5 * v.grad


def test_vit_chain_uses_handed_over_bf16_gradients():
    """Inside VisionTransformer the bf16 gradient copies do pass from each block's backward
    to the next one up the chain (no per-block cast of the incoming gradient)."""
    from vitmi.modules import VisionTransformer, cross_entropy
    cfg = _cfg("bf16").replace(depth=3)
    model = VisionTransformer(cfg).cuda()
    model.load_param_dict(vit_ref.init_params(cfg, seed=1))
    img, tgt = vit_ref.synthetic_batch(cfg, 4)
    LP_STATS.update(hit=0, miss=0)
    cross_entropy(model(img.cuda()), tgt.cuda()).backward()
    assert LP_STATS == {"hit": cfg.depth, "miss": 0}, LP_STATS
