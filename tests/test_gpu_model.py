"""End-to-end parity of the MI355X ViT path against the CPU oracle (oracle/vit_ref.py)
and against the golden vectors of the reference's own MS_CvT module / HF ViT.

Tolerances:  fp32: logits max-abs <= 1e-3 (north star; we assert
1e-4), loss rel <= 1e-5, every grad ||d||/||g|| <= 1e-3.  bf16: grads <= 2e-2; logits
max-abs measured and asserted against a bf16-appropriate bound (stated per test)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import vit_ref  # noqa: E402
from vitmi.config import ViTConfig, config_c1, config_c2, preset  # noqa: E402
from vitmi.modules import VisionTransformer, cross_entropy, mse_loss  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")

# bf16 logits bounds: about 2x the max-abs error measured on MI355X ("Oracle and
# parity"), so a numerics regression of a few x fails instead of hiding under a loose bound
BF16_VITB_LOGITS = 7e-3      # measured 2.7e-3 (bs 2, default init) / 3.6e-3 (randomised, fwd+bwd)
BF16_C1_LOGITS = 5e-3        # measured 2.2e-3
BF16_VITL_LOGITS = 1e-2      # measured 4.9e-3 (ViT-L/16@384, depth 4)
BF16_GRADS = 1.5e-2          # worst relative grad error measured 6.9e-3 (C1) / 7.5e-3 (ViT-B depth 12)
# ||d|| / sum_i ||g_i|| (per-image contributions, vit_ref.per_image_grad_scale): the bf16 backward's
# rounding relative to what it rounds; measured <= 4.5e-3 (C1 / 48 px / N = 290, bf16 and bf16x3,
# round 5), the bound about 2x that
BF16_GRADS_COND = 1e-2


def gpu_step(cfg, params, img, tgt):
    model = VisionTransformer(cfg).cuda()
    model.load_param_dict(params)
    logits = model(img.cuda())
    loss = cross_entropy(logits, tgt.cuda()) if cfg.num_classes > 1 else mse_loss(logits, tgt.cuda())
    loss.backward()
    grads = {k: p.grad.detach().cpu() for k, p in model.named_parameters()}
    return logits.detach().cpu(), loss.detach().cpu(), grads


def compare(cfg, params, img, tgt, logit_tol, grad_tol, loss_tol=1e-5):
    l_ref, loss_ref, g_ref = vit_ref.forward_backward(img, tgt, params, cfg)
    l, loss, g = gpu_step(cfg, params, img, tgt)
    err = (l - l_ref).abs().max().item()
    assert err <= logit_tol, f"logits max-abs {err:.3e} > {logit_tol}"
    assert abs(loss.item() - loss_ref.item()) <= loss_tol * max(1.0, abs(loss_ref.item())), (loss, loss_ref)
    worst = max((vit_ref.rel_err(g[k], g_ref[k]), k) for k in g_ref)
    assert worst[0] <= grad_tol, f"grad {worst[1]} rel {worst[0]:.3e}"
    return err, worst


def test_c1_fp32_matches_oracle():
    cfg = config_c1()                           # ViT-Ti/16 64x64 bs8 (BASELINE config 1)
    params = vit_ref.init_params(cfg, seed=0)
    img, tgt = vit_ref.synthetic_batch(cfg, 8)
    compare(cfg, params, img, tgt, logit_tol=1e-4, grad_tol=1e-4)


def test_c1_bf16_matches_oracle():
    cfg = config_c1(dtype="bf16")
    params = vit_ref.init_params(cfg, seed=0)
    img, tgt = vit_ref.synthetic_batch(cfg, 8)
    err, worst = compare(cfg, params, img, tgt, logit_tol=BF16_C1_LOGITS, grad_tol=BF16_GRADS, loss_tol=2e-2)
    print(f"C1 bf16: logits max-abs {err:.3e}, worst grad {worst[1]} rel {worst[0]:.3e}")


@pytest.mark.parametrize("variant", [dict(tie_norms=True), dict(qkv_bias=False, attn_scale="dim"),
                                     dict(num_classes=1), dict(embed_norm=True, pos_embed=False)])
def test_knob_variants_fp32(variant):
    cfg = ViTConfig(img_size=32, patch_size=8, embed_dim=128, depth=2, num_heads=2, num_classes=2,
                    dtype="fp32").replace(**variant)
    params = vit_ref.init_params(cfg, seed=1)
    img, tgt = vit_ref.synthetic_batch(cfg, 5, seed=7)
    compare(cfg, params, img, tgt, logit_tol=1e-4, grad_tol=1e-4)


def _golden(name):
    z = np.load(os.path.join(GOLD, name))
    params = {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("p::")}
    grads = {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("g::")}
    return z, params, grads


@pytest.mark.parametrize("name,cfg", [
    ("mscvt_vit_stage.npz", ViTConfig(img_size=32, patch_size=8, embed_dim=128, depth=2, num_heads=2,
                                      num_classes=2, attn_scale="dim", ln_eps=1e-5, qkv_bias=False,
                                      embed_norm=True, pos_embed=False, dtype="fp32")),
    ("hf_vit.npz", ViTConfig(img_size=32, patch_size=8, embed_dim=128, depth=2, num_heads=2, num_classes=2,
                             attn_scale="head", ln_eps=1e-6, qkv_bias=True, dtype="fp32")),
])
def test_gpu_matches_reference_goldens(name, cfg):
    """Replay the golden vectors of the reference's own MS_CvT module and of the offline HF
    ViT (tests/golden/gen_golden.py) through the HIP path: logits, loss and every gradient."""
    z, params, grads = _golden(name)
    img, tgt = torch.from_numpy(z["input"]), torch.from_numpy(z["target"])
    l, loss, g = gpu_step(cfg, params, img, tgt)
    assert np.abs(l.numpy() - z["logits"]).max() <= 1e-4
    assert abs(loss.item() - float(z["loss"])) <= 1e-5
    for k, ref in grads.items():
        assert vit_ref.rel_err(g[k], ref) <= 1e-4, k


def test_vit_b_bf16_logits_vs_oracle():
    """BASELINE config 3 architecture (ViT-B/16 224^2) in bf16 at bs=2 vs the fp32 CPU oracle."""
    cfg = preset("vit_base_16", img_size=224, num_classes=2, dtype="bf16")
    params = vit_ref.init_params(cfg, seed=0, randomize_all=False)
    img, _ = vit_ref.synthetic_batch(cfg, 2)
    with torch.no_grad():
        ref = vit_ref.forward(img, params, cfg)
        model = VisionTransformer(cfg).cuda()
        model.load_param_dict(params)
        out = model(img.cuda()).cpu()
    err = (out - ref).abs().max().item()
    print(f"ViT-B/16 bf16 logits max-abs vs fp32 oracle: {err:.3e}")
    assert err < BF16_VITB_LOGITS


def test_vit_b_bf16_full_depth_fwd_bwd_vs_oracle():
    """BASELINE config 3 architecture at full depth (ViT-B/16 224^2: D = 768, H = 12, N = 197,
    12 blocks) in bf16 at bs=2, forward AND backward against the fp32 CPU oracle on the same
    weights (randomised gamma/beta/biases so every backward term is exercised): logits, loss
    and every parameter gradient, ||d|| / ||g|| <= 2e-2 (SURVEY §8d bf16 bound)."""
    cfg = preset("vit_base_16", img_size=224, num_classes=2, dtype="bf16")
    params = vit_ref.init_params(cfg, seed=0)
    img, tgt = vit_ref.synthetic_batch(cfg, 2)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    err, worst = compare(cfg, params, img, tgt, logit_tol=BF16_VITB_LOGITS, grad_tol=BF16_GRADS, loss_tol=2e-2)
    print(f"ViT-B/16 bf16 depth 12 bs 2: logits max-abs {err:.3e}, worst grad {worst[1]} rel {worst[0]:.3e}")


def test_c2_fp32_fwd_bwd_vs_oracle():
    """BASELINE config 2 architecture (ViT-S/16 224^2, fp32) forward AND backward at bs=4 vs the
    CPU oracle: logits <= 1e-3 (north star), loss rel <= 1e-5, every grad rel <= 1e-3."""
    cfg = config_c2()
    params = vit_ref.init_params(cfg, seed=1)
    img, tgt = vit_ref.synthetic_batch(cfg, 4, seed=3)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    err, worst = compare(cfg, params, img, tgt, logit_tol=1e-5, grad_tol=1e-4, loss_tol=1e-5)  # measured 5.7e-7 / 6.2e-6
    print(f"ViT-S/16 fp32 bs 4: logits max-abs {err:.3e}, worst grad {worst[1]} rel {worst[0]:.3e}")


def test_c2_fp32_logits_vs_oracle():
    """BASELINE config 2: ViT-S/16 224^2 bs=128 fp32 on the GPU vs the CPU oracle, logits <= 1e-3."""
    cfg = config_c2()
    params = vit_ref.init_params(cfg, seed=0, randomize_all=False)
    img, _ = vit_ref.synthetic_batch(cfg, 128)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    with torch.no_grad():
        ref = vit_ref.forward(img, params, cfg)
        model = VisionTransformer(cfg).cuda()
        model.load_param_dict(params)
        out = model(img.cuda()).cpu()
    err = (out - ref).abs().max().item()
    print(f"ViT-S/16 fp32 bs=128 logits max-abs vs CPU oracle: {err:.3e}")
    assert err <= 1e-3


def test_c5_shape_fp32_fwd_bwd_matches_oracle():
    """BASELINE config 5 geometry (384^2, patch 16 -> N = 577 tokens: the streamed,
    LDS-tiled attention kernels, not the whole-sequence ones) at reduced width/depth in fp32,
    full forward + backward vs the CPU oracle at the fp32 tolerances."""
    cfg = ViTConfig(img_size=384, patch_size=16, embed_dim=128, depth=2, num_heads=2, num_classes=2,
                    dtype="fp32")
    assert cfg.seq_len == 577
    params = vit_ref.init_params(cfg, seed=3)
    img, tgt = vit_ref.synthetic_batch(cfg, 2, seed=5)
    compare(cfg, params, img, tgt, logit_tol=1e-4, grad_tol=1e-4)


def test_c5_vit_l_bf16_vs_oracle():
    """ViT-L/16 @384 (config 5 architecture: D = 1024, H = 16, N = 577) in bf16 at bs=2, depth
    cut to 4 so the CPU oracle's backward finishes in seconds: logits and every gradient vs fp32."""
    cfg = preset("vit_large_16", img_size=384, num_classes=2, dtype="bf16", depth=4)
    params = vit_ref.init_params(cfg, seed=0)
    img, tgt = vit_ref.synthetic_batch(cfg, 2)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    err, worst = compare(cfg, params, img, tgt, logit_tol=BF16_VITL_LOGITS, grad_tol=2e-2, loss_tol=2e-2)
    print(f"ViT-L/16@384 depth 4 bf16: logits max-abs {err:.3e}, worst grad {worst[1]} rel {worst[0]:.3e}")


def test_c5_full_depth_bf16_step_is_finite():
    """Full ViT-L/16 @384, 24 blocks, bs=64 (config 5 per-GPU batch): one fwd+bwd step runs,
    the loss is near ln 2 at init and every gradient is finite (size-independent checks)."""
    from vitmi.config import config_c5
    cfg = config_c5()
    model = VisionTransformer(cfg).cuda()
    model.reset_parameters(seed=0)
    g = torch.Generator(device="cuda").manual_seed(1234)
    img = torch.rand(64, 3, 384, 384, device="cuda", generator=g)
    tgt = torch.randint(0, 2, (64,), device="cuda", generator=g)
    loss = cross_entropy(model(img), tgt)
    loss.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - np.log(2)) < 0.5, loss.item()
    for k, p in model.named_parameters():
        assert torch.isfinite(p.grad).all(), k
    del model


def _train(cfg, params, img, tgt, steps, lr, on_gpu):
    """Adam steps (the reference's optimizer, models/CvT(Par).py:464) -> per-step losses."""
    if on_gpu:
        model = VisionTransformer(cfg).cuda()
        model.load_param_dict(params)
        ps = list(model.parameters())
        img, tgt = img.cuda(), tgt.cuda()
    else:
        leaves = {k: v.clone().requires_grad_(True) for k, v in params.items()}
        ps = list(leaves.values())
    opt = torch.optim.Adam(ps, lr=lr)
    out = []
    for _ in range(steps):
        opt.zero_grad()
        if on_gpu:
            loss = cross_entropy(model(img), tgt)
        else:
            loss = vit_ref.loss_fn(vit_ref.forward(img, leaves, cfg), tgt, cfg.num_classes)
        loss.backward()
        opt.step()
        out.append(loss.item())
    return out


def test_adam_training_tracks_oracle():
    """Several optimizer steps: the GPU model follows the CPU oracle's loss trajectory
    (fp32: 1e-4 abs), and bf16 stays within 2e-2 of it."""
    cfg = ViTConfig(img_size=32, patch_size=8, embed_dim=128, depth=2, num_heads=2, num_classes=2,
                    dtype="fp32")
    params = vit_ref.init_params(cfg, seed=3)
    img, tgt = vit_ref.synthetic_batch(cfg, 16)
    ref = _train(cfg, params, img, tgt, 8, 3e-4, on_gpu=False)
    got = _train(cfg, params, img, tgt, 8, 3e-4, on_gpu=True)
    assert max(abs(a - b) for a, b in zip(ref, got)) < 1e-4, (ref, got)
    got16 = _train(cfg.replace(dtype="bf16"), params, img, tgt, 8, 3e-4, on_gpu=True)
    assert max(abs(a - b) for a, b in zip(ref, got16)) < 2e-2, (ref, got16)
    assert ref[-1] < ref[0]


# ------------------------------------------------------------------ dropout (row a12)
def _drop_step(cfg, params, img, tgt, seed, train=True):
    model = VisionTransformer(cfg).cuda()
    model.load_param_dict(params)
    model.drop_seed = seed
    model.train(train)
    logits = model(img.cuda())
    loss = cross_entropy(logits, tgt.cuda())
    loss.backward()
    grads = {k: p.grad.detach().cpu() for k, p in model.named_parameters()}
    return logits.detach().cpu(), loss.detach().cpu(), grads


@pytest.mark.parametrize("dtype,ltol,gtol", [("fp32", 1e-4, 1e-4), ("bf16", 5e-2, 2e-2)])
def test_dropout_training_matches_oracle(dtype, ltol, gtol):
    """Keras' training-mode Dropout (models/CvT(Par).py:189,255,257) at rate 0.1: the device
    epilogues and masked backward copies drop exactly the oracle's elements (same hash)."""
    cfg = ViTConfig(img_size=32, patch_size=8, embed_dim=128, depth=2, num_heads=2, num_classes=2,
                    dtype=dtype, drop_rate=0.1)
    params = vit_ref.init_params(cfg, seed=0)
    img, tgt = vit_ref.synthetic_batch(cfg, 4)
    l_ref, loss_ref, g_ref = vit_ref.forward_backward(img, tgt, params, cfg, drop_seed=4242)
    l_nodrop, _, _ = vit_ref.forward_backward(img, tgt, params, cfg)
    assert (l_ref - l_nodrop).abs().max().item() > 1e-3      # the masks do act
    l, loss, g = _drop_step(cfg, params, img, tgt, 4242)
    print(f"dropout {dtype}: logits max-abs {(l - l_ref).abs().max().item():.3e}")
    assert (l - l_ref).abs().max().item() <= ltol
    worst = max((vit_ref.rel_err(g[k], g_ref[k]), k) for k in g_ref)
    assert worst[0] <= gtol, f"grad {worst[1]} rel {worst[0]:.3e}"


def test_dropout_eval_mode_is_identity():
    cfg = ViTConfig(img_size=32, patch_size=8, embed_dim=128, depth=2, num_heads=2, num_classes=2,
                    dtype="fp32", drop_rate=0.1)
    params = vit_ref.init_params(cfg, seed=0)
    img, tgt = vit_ref.synthetic_batch(cfg, 4)
    l_ref, _, g_ref = vit_ref.forward_backward(img, tgt, params, cfg)
    l, _, g = _drop_step(cfg, params, img, tgt, 4242, train=False)
    assert (l - l_ref).abs().max().item() <= 1e-4
    assert max(vit_ref.rel_err(g[k], g_ref[k]) for k in g_ref) <= 1e-4


def test_dropout_vit_shape_rate_and_scale():
    """ViT-B rows x 3072 GELU activations: the fused epilogue keeps ~90% and scales by 1/0.9."""
    from vitmi import ops
    g = torch.Generator(device="cuda").manual_seed(0)
    M, D, F = 197 * 16, 768, 3072
    x = (torch.rand(M, D, device="cuda", generator=g) - 0.5).to(torch.bfloat16)
    w = ((torch.rand(F, D, device="cuda", generator=g) - 0.5) * 0.1).to(torch.bfloat16)
    b = torch.zeros(F, device="cuda")
    a0, u0 = ops.linear_fwd(x, w, b, torch.bfloat16, ops.EPI_BIAS_GELU)
    a1, u1 = ops.linear_fwd(x, w, b, torch.bfloat16, ops.EPI_BIAS_GELU, dropout=(7, 1, 0.1))
    keep = vit_ref.dropout_hash(7, 1, np.arange(M), np.arange(F)) >= vit_ref.dropout_params(0.1)[0]
    keep_t = torch.from_numpy(keep).cuda()
    assert abs(keep.mean() - 0.9) < 0.005
    assert torch.all(a1[~keep_t] == 0) and torch.all(u1[~keep_t] == 0)
    ref = (a0.float() / 0.9)[keep_t]
    assert ((a1.float()[keep_t] - ref).abs() <= 1e-2 * ref.abs() + 1e-3).all()
    # the backward copy uses the same mask
    gsrc = torch.randn(M, F, device="cuda", generator=g)
    gm = ops.dropout_apply(gsrc, 7, 1, 0.1, torch.float32)
    assert torch.equal(gm[~keep_t], torch.zeros_like(gm[~keep_t]))
    assert torch.allclose(gm[keep_t], gsrc[keep_t] / 0.9, rtol=1e-6, atol=0)


# ------------------------------------------------------------------ determinism
@pytest.mark.parametrize("dtype,batch", [("bf16", 64), ("fp32", 4)])
def test_fwd_bwd_is_bitwise_deterministic(dtype, batch):
    """The HIP race check of SURVEY §5: the same step run twice gives bitwise-identical logits,
    loss and gradients.  No kernel of the path uses atomics; split-K, tail-split and column-sum
    partials are folded in a fixed order, and LDS tiles are barrier-ordered.  ViT-B/16 width at
    depth 2 and bs 64 puts every GEMM on the persistent kernel with its split-K / tail-split
    units (M = 12,608 rows)."""
    cfg = preset("vit_base_16", img_size=224, num_classes=2, dtype=dtype, depth=2)
    params = vit_ref.init_params(cfg, seed=5)
    img, tgt = vit_ref.synthetic_batch(cfg, batch, seed=6)
    runs = [gpu_step(cfg, params, img, tgt) for _ in range(2)]
    (l0, s0, g0), (l1, s1, g1) = runs
    assert torch.equal(l0, l1) and torch.equal(s0, s1)
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k


def test_vit_b_precision_knob_fp32_meets_1e3():
    """The precision knob: ViT-B/16 224^2 at full depth 12 with dtype='fp32'
    (exact-fp32 MFMA GEMMs and fp32 attention) meets the north star's logits-within-1e-3 against
    the fp32 CPU oracle, forward AND backward, on the randomised-parameter stress case where the
    bf16 default measures 3.6e-3."""
    cfg = preset("vit_base_16", img_size=224, num_classes=2, dtype="fp32")
    params = vit_ref.init_params(cfg, seed=0)
    img, tgt = vit_ref.synthetic_batch(cfg, 2)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    err, worst = compare(cfg, params, img, tgt, logit_tol=1e-3, grad_tol=1e-3, loss_tol=1e-5)
    print(f"ViT-B/16 fp32 depth 12 bs 2: logits max-abs {err:.3e}, worst grad {worst[1]} rel {worst[0]:.3e}")
    assert err <= 1e-4     # measured margin: fp32 sums in another order only


def test_vit_b_precision_knob_bf16x3_meets_1e3():
    """The split-bf16 precision knob (dtype='bf16x3': the forward GEMMs' weights, LayerNorm
    outputs, attention output and GELU output as hi + lo bf16 pairs; q, k, v and the softmax P
    bf16; tools/precision_emulate.py ranks those operands and puts this set at 1.5e-4) meets the
    north star's logits within 1e-3 against the fp32 CPU oracle at ViT-B/16 full depth 12, on the
    randomised-parameter stress case where the bf16 default measures 3.6e-3 (measured 1.7e-4).
    The backward is the bf16 one (grads at the bf16 bound)."""
    cfg = preset("vit_base_16", img_size=224, num_classes=2, dtype="bf16x3")
    params = vit_ref.init_params(cfg, seed=0)
    img, tgt = vit_ref.synthetic_batch(cfg, 2)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    err, worst = compare(cfg, params, img, tgt, logit_tol=1e-3, grad_tol=BF16_GRADS, loss_tol=1e-3)
    print(f"ViT-B/16 bf16x3 depth 12 bs 2: logits max-abs {err:.3e}, worst grad {worst[1]} rel {worst[0]:.3e}")


@pytest.mark.parametrize("split_qkv", [False, True, "weight", None])
def test_vit_b_precision_knob_bf16f8_meets_1e3(split_qkv):
    """The knob's cheaper form (dtype='bf16f8': split operands with hi.lo + lo.hi as one
    block-scaled e4m3 product, include/vitmi.h VITMI_BF16F8) meets the north star's logits within
    1e-3 against the fp32 CPU oracle at ViT-B/16 full depth 12, on the randomised-parameter stress
    case.  Its qkv GEMM: plain bf16 (False; tools/precision_emulate_fp8.py --classes: 6.4e-4 here),
    split (True, 1.8e-4) or, by default (None), with the weight-side correction alone ("weight",
    VITMI_BF16F8W; tools/precision_sides.py: 3.2e-4 on these 2 images, 8-image RMS 1.7e-4)."""
    cfg = preset("vit_base_16", img_size=224, num_classes=2, dtype="bf16f8", split_qkv=split_qkv)
    params = vit_ref.init_params(cfg, seed=0)
    img, tgt = vit_ref.synthetic_batch(cfg, 2)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    err, worst = compare(cfg, params, img, tgt, logit_tol=1e-3, grad_tol=BF16_GRADS, loss_tol=1e-3)
    print(f"ViT-B/16 bf16f8 (split qkv {split_qkv}) depth 12 bs 2: logits max-abs {err:.3e}, "
          f"worst grad {worst[1]} rel {worst[0]:.3e}")
    assert err <= (1e-3 if split_qkv is False else 5e-4)


@pytest.mark.parametrize("knob,split_qkv", [("bf16x3", False), ("bf16f8", True)])
def test_knob_split_qkv_override_small_model(knob, split_qkv):
    """ViTConfig.split_qkv against each knob's default (bf16x3 with the qkv GEMM plain bf16, bf16f8
    with it split), C1 shape: logits within 1e-3 of the fp32 oracle, gradients at the bf16 bound."""
    cfg = config_c1(dtype=knob, split_qkv=split_qkv)
    params = vit_ref.init_params(cfg, seed=3)
    img, tgt = vit_ref.synthetic_batch(cfg, 5)
    err, worst = compare(cfg, params, img, tgt, logit_tol=1e-3, grad_tol=2e-2, loss_tol=1e-3)
    print(f"C1 {knob} split_qkv={split_qkv}: logits {err:.3e}, worst grad {worst[1]} {worst[0]:.3e}")


@pytest.mark.parametrize("knob,split_qkv", [("bf16x3", False), ("bf16f8", True)])
def test_knob_split_qkv_override_streamed_n290(knob, split_qkv):
    """The split_qkv overrides on the streamed-attention path (ViT-Ti/16 272 px, N = 290, depth 4,
    the fp32 O of the knobs' streamed forward): logits within 1e-3 of the fp32 oracle."""
    cfg = config_c1(dtype=knob, img_size=272, depth=4, split_qkv=split_qkv)
    params = vit_ref.init_params(cfg, seed=8)
    img, tgt = vit_ref.synthetic_batch(cfg, 2)
    l_ref = vit_ref.forward(img, params, cfg)
    logits, _, _ = gpu_step(cfg, params, img, tgt)
    err = (logits - l_ref).abs().max().item()
    print(f"N=290 {knob} split_qkv={split_qkv}: logits {err:.3e}")
    assert err <= 1e-3


@pytest.mark.parametrize("knob", ["bf16x3", "bf16f8"])
def test_bf16x3_knob_streamed_attention_n290(knob):
    """bf16 and bf16x3 at N > 256 (ViT-Ti/16 at 272 px, N = 290, depth 4: the streamed attention
    kernels; the knob takes O from the fp32 streamed forward and o / lse from the bf16 one,
    vitmi/modules.py _forward_x3).  Logits of the knob within 1e-3 of the fp32 oracle.

    Gradients, against the ORACLE, two ways (SURVEY §8d bf16 bound 2e-2):
      * a well-conditioned batch (both images labelled 0): ||d|| / ||g|| <= 1.2e-2 per tensor;
      * the seed's own labels (0, 1): the two images' gradients nearly cancel here (the model
        gives both noise images almost the same logits, so g = g_0 + g_1 with ||g_i|| up to 75 x
        ||g||: kappa, oracle.vit_ref.per_image_grad_scale).  A backward that rounds each image's
        contribution to bf16 (2^-9) cannot meet 2e-2 of ||g|| there: even the fp32 path's error grows
        by the same factor (6e-7 at N = 197 -> 4.6e-5 here; tools/diag_grad_precision.py).  The bound
        is applied to what the rounding acts on: ||d|| <= tol * sum_i ||g_i|| (BF16_GRADS_COND; the
        same bound at kappa = 1), and kappa is asserted so the case stays the ill-conditioned one."""
    cfg = config_c1(dtype=knob, img_size=272, depth=4)
    params = vit_ref.init_params(cfg, seed=8)
    img, tgt = vit_ref.synthetic_batch(cfg, 2)
    assert tgt.tolist() == [0, 1]
    for labels in (torch.zeros_like(tgt), tgt):
        l_ref, _, g_ref = vit_ref.forward_backward(img, labels, params, cfg)
        scale = vit_ref.per_image_grad_scale(img, labels, params, cfg)
        kappa = max(scale[k] / g_ref[k].double().norm().item() for k in g_ref)
        for c in (cfg.replace(dtype="bf16"), cfg):
            l, _, g = gpu_step(c, params, img, labels)
            plain = max((vit_ref.rel_err(g[k], g_ref[k]), k) for k in g_ref)
            cond = max(((g[k] - g_ref[k]).double().norm().item() / scale[k], k) for k in g_ref)
            print(f"N=290 {c.dtype} labels {labels.tolist()}: kappa {kappa:.1f}; worst grad rel {plain[0]:.3e} "
                  f"({plain[1]}), conditioned {cond[0]:.3e} ({cond[1]})")
            if c.dtype == knob:
                err = (l - l_ref).abs().max().item()
                print(f"   {knob} logits max-abs {err:.3e}")
                assert err <= 1e-3
            if labels.sum() == 0:       # measured 5.8e-3 (bf16), 5.4e-3 (bf16x3)
                assert kappa < 1.5
                assert plain[0] <= 1.2e-2, plain
            else:                        # kappa 92; conditioned 4.1e-3 (bf16), 3.4e-3 (bf16x3)
                assert kappa > 30
                assert cond[0] <= BF16_GRADS_COND, cond


@pytest.mark.parametrize("knob", ["bf16x3", "bf16f8"])
def test_bf16x3_knob_small_model_matches_oracle(knob):
    """bf16x3 on the C1 shape (ViT-Ti/16 64^2, N = 17) and on a ragged token count (48^2, N = 10):
    logits within the north star's 1e-3 (C1 measures 3.4e-4: the bf16 q, k, v and P), gradients
    (the bf16 backward) at SURVEY §8d's bf16 bound 2e-2 against the oracle (the worst, block 0's
    norm1.bias at 5 images, measures 1.98e-2 for the knob and 1.92e-2 for bf16; a CPU emulation of
    the same roundings, tools/precision_emulate_bwd.py, finds no single bf16 rounding whose removal
    brings it under 1.1e-2: profiles/r05_precision/).  These batches are mildly ill-conditioned
    (labels 3:2 and 4:1, kappa up to 7, oracle.vit_ref.per_image_grad_scale), so the bf16 rounding
    of each image's contribution is also held to the conditioned bound ||d|| <= tol * sum_i ||g_i||
    with a tighter tol (BF16_GRADS_COND; measured <= 4.5e-3)."""
    for cfg in (config_c1(dtype=knob), config_c1(dtype=knob, img_size=48)):
        params = vit_ref.init_params(cfg, seed=3)
        img, tgt = vit_ref.synthetic_batch(cfg, 5)
        scale = vit_ref.per_image_grad_scale(img, tgt, params, cfg)
        _, _, g_ref = vit_ref.forward_backward(img, tgt, params, cfg)
        for c, ltol, lstol in ((cfg, 1e-3, 1e-3), (cfg.replace(dtype="bf16"), 5e-3, 2e-2)):
            e, w = compare(c, params, img, tgt, logit_tol=ltol, grad_tol=2e-2, loss_tol=lstol)
            _, _, g = gpu_step(c, params, img, tgt)
            cond = max(((g[k] - g_ref[k]).double().norm().item() / scale[k], k) for k in g_ref)
            print(f"{cfg.img_size}px {c.dtype}: logits {e:.3e}; worst grad {w[1]} {w[0]:.3e}; "
                  f"conditioned {cond[1]} {cond[0]:.3e}")
            assert cond[0] <= BF16_GRADS_COND, cond
