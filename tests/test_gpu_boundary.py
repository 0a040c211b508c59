"""The per-op entry points under SURVEY.md §8(b)'s names (csrc/boundary.cpp:
vitmi_patch_embed_{fwd,bwd}, vitmi_linear_bwd, vitmi_xent_{fwd,bwd}, vitmi_mse_{fwd,bwd}),
called through the C ABI: bit-identical to the kernel-level entry points they compose, and
checked against the CPU oracle's restatement of the reference op (Conv2D k=s=P + cls + pos,
models/CvT(Par).py:203-212,244-245; Dense autodiff; the losses of :464-466)."""
import pytest
import torch
import torch.nn.functional as F

from vitmi import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,C,S,P,D", [(3, 3, 32, 8, 128), (2, 1, 64, 16, 192), (4, 3, 224, 16, 768)])
def test_patch_embed_entry_points(dtype, B, C, S, P, D):
    g = torch.Generator().manual_seed(B * S + D)
    img = torch.rand(B, C, S, S, generator=g)
    w = torch.randn(D, C, P, P, generator=g) * 0.05
    b = torch.randn(D, generator=g) * 0.1
    G = S // P
    cls = torch.randn(D, generator=g) * 0.02
    pos = torch.randn(G * G + 1, D, generator=g) * 0.02
    imgd, wd = img.to(DEV), w.reshape(D, -1).to(DEV).to(dtype)
    bd, clsd, posd = b.to(DEV), cls.to(DEV), pos.to(DEV)
    x, patches = ops.patch_embed_fwd(imgd, wd, bd, clsd, posd.reshape(-1), P, dtype)
    # the composed kernel-level entry points: bit-identical
    p2 = ops.patch_im2col(imgd, P, dtype)
    conv = ops.linear_fwd(p2, wd, bd, torch.float32)
    x2 = ops.tokens_assemble(conv, B, G * G, clsd, posd.reshape(-1))
    assert torch.equal(patches, p2) and torch.equal(x, x2)
    # the oracle op (fp32 conv on the operand-rounded weights and pixels)
    wr = wd.float().cpu().reshape(w.shape)
    ir = img.to(dtype).float()
    ref = F.conv2d(ir, wr, b, stride=P).flatten(2).transpose(1, 2)
    ref = torch.cat([cls.expand(B, 1, D), ref], 1) + pos
    tol = 1e-4 if dtype == torch.float32 else 2e-3
    assert (x.cpu() - ref).abs().max().item() <= tol * max(1.0, ref.abs().max().item())
    # backward: composite vs pieces, and vs the oracle's autograd
    dx = torch.randn(B, G * G + 1, D, generator=g)
    dxd = dx.to(DEV)
    grads = [torch.zeros(D, C * P * P, device=DEV), torch.zeros(D, device=DEV), torch.zeros(D, device=DEV),
             torch.zeros((G * G + 1) * D, device=DEV)]
    ops.patch_embed_bwd(dxd, patches, B, C, S, P, *grads)
    want = [torch.zeros_like(t) for t in grads]
    lp = None if dtype == torch.float32 else dtype
    dtok, dtok_lp = ops.tokens_assemble_bwd(dxd, B, G * G, dtype == torch.float32, lp, want[2], want[3])
    gg = dtok_lp if dtok_lp is not None else dtok
    ops.linear_wgrad(gg, patches, want[0])
    ops.bias_grad(gg, want[1])
    for a, e in zip(grads, want):
        assert torch.equal(a, e)
    wl = wr.clone().requires_grad_(True)
    bl = b.clone().requires_grad_(True)
    cl = cls.clone().requires_grad_(True)
    pl = pos.clone().requires_grad_(True)
    r = F.conv2d(ir, wl, bl, stride=P).flatten(2).transpose(1, 2)
    r = torch.cat([cl.expand(B, 1, D), r], 1) + pl
    r.backward(dx.to(dtype).float() if dtype != torch.float32 else dx)
    gtol = 1e-4 if dtype == torch.float32 else 2e-2
    for got, leaf in zip(grads, (wl, bl, cl, pl)):
        ref_g = leaf.grad.reshape(got.shape)
        assert (got.cpu() - ref_g).norm() <= gtol * ref_g.norm()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_linear_bwd_entry_point(dtype):
    g = torch.Generator().manual_seed(3)
    M, N, K = 197 * 4, 768, 384
    dy = torch.randn(M, N, generator=g).to(DEV).to(dtype)
    x = torch.randn(M, K, generator=g).to(DEV).to(dtype)
    w = (torch.randn(N, K, generator=g) * 0.05).to(DEV).to(dtype)
    dw, db = torch.zeros(N, K, device=DEV), torch.zeros(N, device=DEV)
    dx = ops.linear_bwd(dy, x, w, torch.float32, dw, db)
    dw2, db2 = torch.zeros_like(dw), torch.zeros_like(db)
    dx2 = ops.linear_dgrad(dy, w, torch.float32)
    ops.linear_wgrad(dy, x, dw2)
    ops.bias_grad(dy, db2)
    assert torch.equal(dx, dx2) and torch.equal(dw, dw2) and torch.equal(db, db2)
    f = lambda t: t.float().cpu()  # noqa: E731
    tol = 1e-4 if dtype == torch.float32 else 1e-2
    assert (dx.cpu() - f(dy) @ f(w)).norm() <= tol * (f(dy) @ f(w)).norm()
    assert (dw.cpu() - f(dy).T @ f(x)).norm() <= tol * (f(dy).T @ f(x)).norm()
    assert (db.cpu() - f(dy).sum(0)).norm() <= tol * f(dy).sum(0).norm()


@pytest.mark.parametrize("kind,C", [("xent", 2), ("xent", 1000), ("mse", 1), ("mse", 3)])
def test_loss_entry_points(kind, C):
    g = torch.Generator().manual_seed(C)
    B = 37
    logits = torch.randn(B, C, generator=g)
    if kind == "xent":
        tgt = torch.randint(0, C, (B,), generator=g)
        loss = ops.xent_fwd(logits.to(DEV), tgt.to(DEV))
        dl = ops.xent_bwd(logits.to(DEV), tgt.to(DEV))
        both = ops.loss_fwd_bwd(logits.to(DEV), tgt.to(DEV), ops.LOSS_CE)
        lr = logits.clone().requires_grad_(True)
        ref = F.cross_entropy(lr, tgt)
    else:
        tgt = torch.randn(B, C, generator=g)
        loss = ops.mse_fwd(logits.to(DEV), tgt.to(DEV))
        dl = ops.mse_bwd(logits.to(DEV), tgt.to(DEV))
        both = ops.loss_fwd_bwd(logits.to(DEV), tgt.to(DEV), ops.LOSS_MSE)
        lr = logits.clone().requires_grad_(True)
        ref = F.mse_loss(lr, tgt)
    ref.backward()
    assert torch.equal(loss, both[0]) and torch.equal(dl, both[1])
    assert abs(loss.item() - ref.item()) <= 1e-5 * max(1.0, abs(ref.item()))
    assert (dl.cpu() - lr.grad).abs().max().item() <= 1e-6
