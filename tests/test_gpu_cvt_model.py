"""Model-level GPU parity of the CvT: vitmi.cvt.CvT (conv-embed im2col GEMMs,
dw_bn q/k/v projections, fused CvT blocks, LN(cls) head) against oracle/cvt_ref.py, the
restatement pinned by the MS_CvT golden vectors (tests/test_cvt_oracle.py).

Tolerances: fp32 compute — logits/loss 1e-4 relative, every parameter gradient 1e-3 relative
(norm floor 1e-4 for the ~1e-7 norm1 gradients, see test_cvt_oracle.py); bf16 compute (the
reference's mixed policy: bf16 GEMM/attention operands, fp32 residual stream, LN and BN
statistics) — logits 3e-2, gradients 8e-2 relative."""
import dataclasses

import numpy as np
import pytest
import torch

from oracle import cvt_ref
from vitmi import cvt
from vitmi.modules import cross_entropy, mse_loss

DEV = "cuda"


def product_cfg(ocfg: cvt_ref.CvTConfig, dtype=None) -> cvt.CvTConfig:
    d = dataclasses.asdict(ocfg)
    d["stages"] = [cvt.CvTStage(**s) for s in d["stages"]]
    if dtype is not None:
        d["dtype"] = dtype
    return cvt.CvTConfig(**d)


def mscvt_cfg():
    from test_cvt_oracle import mscvt_cfg as m
    return m()


def mscvt_avg_cfg():
    from test_cvt_oracle import mscvt_avg_cfg as m
    return m()


def with_method(ocfg, method):
    return ocfg.replace(stages=[dataclasses.replace(s, qkv_method=method) for s in ocfg.stages])


def rel(a, b, floor=1e-12):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / max(b.norm().item(), floor)).item()


def run_product(pcfg, params, img, tgt, proc=None):
    model = cvt.CvT(pcfg).to(DEV)
    model.load_param_dict(params)
    model.train()
    logits = model(img.to(DEV), None if proc is None else proc.to(DEV))
    if pcfg.num_classes == 1:
        loss = mse_loss(logits, tgt.to(DEV))
    else:
        loss = cross_entropy(logits, tgt.to(DEV))
    loss.backward()
    torch.cuda.synchronize()
    grads = {k: p.grad for k, p in model.named_parameters()}
    return model, logits.detach(), loss.detach(), grads


def test_param_names_match_oracle():
    # pure host check (no kernels): the module tree names every oracle parameter
    for ocfg in (mscvt_cfg(), cvt_ref.CvTConfig(img_size=64), mscvt_avg_cfg(),
                 with_method(cvt_ref.CvTConfig(img_size=64, proc_dim=5), "linear"),
                 cvt_ref.CvTConfig(img_size=64, keras_dense=True)):
        model = cvt.CvT(product_cfg(ocfg))
        shapes = {k: tuple(p.shape) for k, p in model.named_parameters()}
        assert shapes == {k: tuple(s) for k, s in cvt_ref.param_shapes(ocfg).items()}


@pytest.mark.gpu
@pytest.mark.parametrize("fixture", ["dwbn", "avg"])
def test_cvt_matches_mscvt_golden_fp32(fixture):
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", f"mscvt_cvt_{fixture}.npz"))
    params = {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("p::")}
    gref = {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("g::")}
    img, tgt = torch.from_numpy(z["input"]), torch.from_numpy(z["target"])
    ocfg = mscvt_cfg() if fixture == "dwbn" else mscvt_avg_cfg()
    _, logits, loss, grads = run_product(product_cfg(ocfg), params, img, tgt)
    assert rel(logits, torch.from_numpy(z["logits"])) < 1e-4
    assert abs(loss.item() - float(z["loss"])) < 1e-4 * max(1.0, abs(float(z["loss"])))
    for k, g in gref.items():
        assert rel(grads[k], g, 1e-4) < 1e-3, k


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,img_size,batch,ncls,method,proc_dim", [
    ("fp32", 64, 4, 1, "dw_bn", 0), ("fp32", 64, 3, 3, "dw_bn", 0), ("bf16", 64, 4, 1, "dw_bn", 0),
    ("bf16", 128, 2, 2, "dw_bn", 0),
    ("fp32", 64, 4, 1, "avg", 0), ("fp32", 64, 3, 1, "linear", 0), ("bf16", 64, 4, 1, "avg", 0),
    # the reference's production model: dw_bn + the 5-parameter process MLP head (:343-350)
    ("fp32", 64, 4, 1, "dw_bn", 5), ("bf16", 128, 4, 1, "dw_bn", 5)])
def test_cvt_keras_spec_vs_oracle(dtype, img_size, batch, ncls, method, proc_dim):
    ocfg = with_method(cvt_ref.CvTConfig(img_size=img_size, num_classes=ncls, dtype="fp32", proc_dim=proc_dim),
                       method)
    params = cvt_ref.init_params(ocfg, seed=5)
    img, tgt = cvt_ref.synthetic_batch(ocfg, batch, seed=7)
    proc = cvt_ref.synthetic_proc(ocfg, batch) if proc_dim else None
    logits_ref, loss_ref, gref = cvt_ref.forward_backward(img, tgt, params, ocfg, proc)
    _, logits, loss, grads = run_product(product_cfg(ocfg, dtype), params, img, tgt, proc)
    tl, tg = (1e-4, 1e-3) if dtype == "fp32" else (3e-2, 8e-2)
    assert rel(logits, logits_ref) < tl
    assert abs(loss.item() - loss_ref.item()) < tl * max(1.0, abs(loss_ref.item()))
    # the key biases (proj_k.bias and the k projection's BN beta) shift every key of a row by
    # the same vector: softmax is invariant to it, so their exact gradient is 0 and both sides
    # hold rounding noise only -- bound it against the matching query-bias gradient instead
    # (the BN beta only in stages without a cls token: the cls key bypasses dw_bn)
    zero = [k for k in gref if k.endswith("attn.proj_k.bias") or (
        k.endswith("attn.conv_proj_k.bn.bias") and not ocfg.stages[int(k[5])].with_cls_token)]
    # (the matching query bias exists only when the q projection has one)
    zero = [k for k in zero if k.replace("_k.", "_q.") in gref]
    bad = {}
    for k, g in gref.items():
        if k in zero:
            kq = k.replace("_k.", "_q.")
            r = grads[k].norm().item() / grads[kq].norm().item()
            if r >= tg:
                bad[k] = ("zero-grad", r, g.norm().item() / gref[kq].norm().item())
        else:
            r = rel(grads[k], g, 1e-4)
            if r >= tg:
                bad[k] = r
    assert not bad, bad


@pytest.mark.gpu
def test_cvt_moving_stats_and_eval_mode():
    """training steps update each dw_bn's moving mean/var (Keras momentum 0.99); eval mode
    normalises with them (BatchNormalization(training=False)) and leaves them unchanged."""
    ocfg = cvt_ref.CvTConfig(img_size=64, num_classes=2, dtype="fp32")
    params = cvt_ref.init_params(ocfg, seed=3)
    img, tgt = cvt_ref.synthetic_batch(ocfg, 4, seed=9)
    model, logits_tr, _, _ = run_product(product_cfg(ocfg), params, img, tgt)
    bn = model.stage0.blocks[0].attn.conv_proj_q.bn
    rm, rv = bn.running_mean.clone(), bn.running_var.clone()
    assert rm.abs().sum().item() > 0 and (rv - 1).abs().sum().item() > 0
    # batch statistics of the first q projection, recomputed on the CPU with the oracle's pieces
    F = torch.nn.functional
    st = ocfg.stages[0]
    x = cvt_ref.conv_embed(img, params["stage0.embed.weight"], params["stage0.embed.bias"], st)
    D = x.shape[1]
    t = F.layer_norm(x.permute(0, 2, 3, 1), (D,), params["stage0.blocks.0.norm1.weight"],
                     params["stage0.blocks.0.norm1.bias"], ocfg.ln_eps).permute(0, 3, 1, 2)
    zq = F.conv2d(t, params["stage0.blocks.0.attn.conv_proj_q.weight"], None, padding=1, groups=D)
    assert rel(rm, 0.01 * zq.mean(dim=(0, 2, 3))) < 1e-4
    assert rel(rv, 0.99 + 0.01 * zq.var(dim=(0, 2, 3), unbiased=True)) < 1e-4
    model.eval()
    with torch.no_grad():
        l1 = model(img.to(DEV))
        l2 = model(img.to(DEV))
    torch.cuda.synchronize()
    assert torch.equal(bn.running_mean, rm) and torch.equal(bn.running_var, rv)
    assert torch.equal(l1, l2)
    assert rel(l1, logits_tr) > 1e-6      # moving stats after one step differ from the batch stats


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K,act", [(256, 256, 5, 1), (7, 256, 256, 1), (33, 3, 17, 0)])
def test_dense_f32_kernels(M, N, K, act):
    """the small fp32 Dense kernels (Proc_Dense_1/2) vs torch fp32 autograd on the CPU"""
    from vitmi import ops
    g = torch.Generator().manual_seed(M + N + K)
    x, w, b = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) / K ** 0.5, torch.randn(N, generator=g)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    yr = torch.nn.functional.linear(xr, wr, br)
    if act:
        yr = torch.relu(yr)
    dy = torch.randn(M, N, generator=g)
    (yr * dy).sum().backward()
    y = ops.dense_f32_fwd(x.to(DEV), w.to(DEV), b.to(DEV), act)
    dw, db = torch.ones(N, K, device=DEV), torch.zeros(N, device=DEV)
    dx = ops.dense_f32_bwd(dy.to(DEV), y, x.to(DEV), w.to(DEV), dw, db, act)
    assert rel(y, yr) < 1e-6
    assert rel(dx, xr.grad) < 1e-6
    assert rel(dw - 1, wr.grad) < 1e-6          # accumulates
    assert rel(db, br.grad) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_cvt_dropout_matches_oracle(dtype):
    """Keras Dropout(0.1) after the out-projection and both MLP Dense layers (models/CvT(Par).py
    :141,189,255,257) in training mode: the build's counter-hash masks, fused into the GEMM
    epilogues, regenerated in the backward -- identical masks in the oracle for a fixed seed."""
    ocfg = cvt_ref.CvTConfig(img_size=64, num_classes=1, dtype="fp32", drop_rate=0.1, proc_dim=5)
    params = cvt_ref.init_params(ocfg, seed=6)
    img, tgt = cvt_ref.synthetic_batch(ocfg, 3, seed=8)
    proc = cvt_ref.synthetic_proc(ocfg, 3)
    logits_ref, loss_ref, gref = cvt_ref.forward_backward(img, tgt, params, ocfg, proc, drop_seed=4242)
    no_drop, _, _ = cvt_ref.forward_backward(img, tgt, params, ocfg.replace(drop_rate=0.0), proc)
    assert rel(no_drop, logits_ref) > 1e-3            # the masks change the output
    model = cvt.CvT(product_cfg(ocfg, dtype)).to(DEV)
    model.load_param_dict(params)
    model.train()
    model.drop_seed = 4242
    logits = model(img.to(DEV), proc.to(DEV))
    mse_loss(logits, tgt.to(DEV)).backward()
    tl, tg = (1e-4, 1e-3) if dtype == "fp32" else (3e-2, 8e-2)
    assert rel(logits, logits_ref) < tl
    bad = {}
    for k, p in model.named_parameters():
        if k.endswith("attn.proj_k.bias") or (k.endswith("attn.conv_proj_k.bn.bias") and "stage2" not in k):
            continue   # exact-zero gradients (softmax shift invariance), see test_cvt_keras_spec_vs_oracle
        r = rel(p.grad, gref[k], 1e-4)
        if r >= tg:
            bad[k] = r
    assert not bad, bad
    model.eval()                                       # inference: no dropout
    with torch.no_grad():
        assert torch.equal(model(img.to(DEV), proc.to(DEV)), model(img.to(DEV), proc.to(DEV)))


def _factored_cfg():
    # dh = 64 per head (the attention kernels' head dim); 8x8 tokens, then 4x4 + cls
    return cvt_ref.CvTConfig(img_size=32, num_classes=1, dtype="fp32", keras_dense=True,
                             stages=[cvt_ref.CvTStage(64, 7, 4, 1), cvt_ref.CvTStage(128, 3, 2, 2, with_cls_token=True)])


def test_keras_dense_param_names_match_oracle():
    # host check: the factored module tree names every factored oracle parameter (mha_{q,k,v,o})
    ocfg = _factored_cfg()
    model = cvt.CvT(product_cfg(ocfg))
    shapes = {k: tuple(p.shape) for k, p in model.named_parameters()}
    assert shapes == {k: tuple(s) for k, s in cvt_ref.param_shapes(ocfg).items()}
    assert any(".mha_o." in k for k in shapes)


@pytest.mark.gpu
def test_keras_dense_factored_adam_trajectory_matches_oracle():
    """CvTConfig.keras_dense (models/CvT(Par).py:132-137,180-188: Dense then MHA's own q/k/v
    projection; MHA's output projection then Dense): 8 Keras-Adam steps of vitmi.optim.Adam on the
    factored model against the factored oracle stepped by oracle/optim_ref.adam_step on the same
    batches (fp32): every parameter's total update within 2e-2 relative (the key biases and the
    k projection's BN beta in a stage without cls, whose exact gradient is 0 -- softmax ignores a
    per-row shift of the keys -- excluded, as in test_cvt_keras_spec_vs_oracle).  The composed model (keras_dense=False) started from the same
    map takes a different trajectory: its out-projection update differs by > 10 %."""
    from oracle.optim_ref import adam_step
    from vitmi.optim import Adam
    ocfg = _factored_cfg()
    params = cvt_ref.init_params(ocfg, seed=11)
    model = cvt.CvT(product_cfg(ocfg)).to(DEV)
    model.load_param_dict(params)
    model.train()
    opt = Adam(model.parameters(), learning_rate=1e-3)
    p = {k: v.numpy().copy() for k, v in params.items()}
    m = {k: np.zeros_like(v) for k, v in p.items()}
    v_ = {k: np.zeros_like(v) for k, v in p.items()}
    # the composed model from the same initial map
    comp_params = {}
    for k, t in params.items():
        if ".mha_" in k:
            continue
        comp_params[k] = t
    for i in range(len(ocfg.stages)):
        pre = f"stage{i}.blocks.0.attn."
        for c in "qkv":
            W1, b1 = params[pre + f"proj_{c}.weight"], params[pre + f"proj_{c}.bias"]
            W2, b2 = params[pre + f"mha_{c}.weight"], params[pre + f"mha_{c}.bias"]
            comp_params[pre + f"proj_{c}.weight"] = W2 @ W1
            comp_params[pre + f"proj_{c}.bias"] = W2 @ b1 + b2
        W1, b1 = params[pre + "mha_o.weight"], params[pre + "mha_o.bias"]
        W2, b2 = params[pre + "proj.weight"], params[pre + "proj.bias"]
        comp_params[pre + "proj.weight"] = W2 @ W1
        comp_params[pre + "proj.bias"] = W2 @ b1 + b2
    comp = cvt.CvT(product_cfg(ocfg.replace(keras_dense=False))).to(DEV)
    comp.load_param_dict(comp_params)
    comp.train()
    copt = Adam(comp.parameters(), learning_rate=1e-3)
    for step in range(1, 9):
        img, tgt = cvt_ref.synthetic_batch(ocfg, 4, seed=100 + step)
        for mod, o in ((model, opt), (comp, copt)):
            o.zero_grad()
            mse_loss(mod(img.to(DEV)), tgt.to(DEV)).backward()
            o.step()
        _, _, g = cvt_ref.forward_backward(img, tgt, {k: torch.from_numpy(t) for k, t in p.items()}, ocfg)
        for k in p:
            p[k], m[k], v_[k] = adam_step(p[k], g[k].numpy(), m[k], v_[k], 1e-3, step)
    torch.cuda.synchronize()
    got = {k: t.detach().cpu() for k, t in model.named_parameters()}
    zero = [k for k in p if k.endswith("attn.proj_k.bias") or k.endswith("attn.mha_k.bias") or (
        k.endswith("attn.conv_proj_k.bn.bias") and not ocfg.stages[int(k[5])].with_cls_token)]
    bad = {}
    for k in p:
        if k in zero:
            continue
        d_ref = torch.from_numpy(p[k]) - params[k]
        r = rel(got[k] - params[k], d_ref, 1e-6)
        if r >= 2e-2:
            bad[k] = r
    assert not bad, bad
    # the composed trajectory: compare the out-projection maps after 8 steps
    pre = "stage1.blocks.0.attn."
    Wf = got[pre + "proj.weight"] @ got[pre + "mha_o.weight"]
    Wc = dict(comp.named_parameters())[pre + "proj.weight"].detach().cpu()
    W0 = comp_params[pre + "proj.weight"]
    assert rel(Wc - W0, Wf - W0) > 0.1


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_keras_dense_one_step_grads_match_oracle(dtype):
    """keras_dense forward + backward against the factored oracle: logits and every factor's
    gradient (the chain-rule GEMMs of vitmi.cvt._chain) at the fp32 / bf16 bounds of
    test_cvt_keras_spec_vs_oracle.  The key biases have an exact gradient of 0 (softmax ignores a
    per-row shift of the keys): their error is bounded against the matching query bias gradient.
    The k projection's BN beta is such a shift too except for the cls key, which bypasses the BN
    (17 tokens here): its gradient nearly cancels, so its error is bounded against the norm of
    the same BN's gamma gradient."""
    ocfg = _factored_cfg().replace(num_classes=3)
    params = cvt_ref.init_params(ocfg, seed=13)
    img, tgt = cvt_ref.synthetic_batch(ocfg, 4, seed=14)
    logits_ref, loss_ref, gref = cvt_ref.forward_backward(img, tgt, params, ocfg)
    _, logits, loss, grads = run_product(product_cfg(ocfg, dtype), params, img, tgt)
    tl, tg = (1e-4, 1e-3) if dtype == "fp32" else (3e-2, 8e-2)
    assert rel(logits, logits_ref) < tl
    bad = {}
    for k, g in gref.items():
        if k.endswith("attn.proj_k.bias") or k.endswith("attn.mha_k.bias"):
            kq = k.replace("_k.", "_q.")
            r = (grads[k].detach().cpu() - g).norm().item() / gref[kq].norm().item()
        elif k.endswith("attn.conv_proj_k.bn.bias"):
            r = (grads[k].detach().cpu() - g).norm().item() / gref[k.replace("bn.bias", "bn.weight")].norm().item()
        else:
            r = rel(grads[k], g, 1e-4)
        if r >= tg:
            bad[k] = r
    assert not bad, bad
