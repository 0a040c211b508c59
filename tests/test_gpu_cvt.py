"""GPU parity of the CvT kernels against plain torch on the CPU: strided
'same' conv-embed im2col / col2im (models/CvT(Par).py:203-212) and the dw_bn projection
(depthwise 3x3 + training-mode BatchNorm, :92-94,104-106), forward and backward, including the
cls-row-skipping layout of stage 3 (:146-150).  fp32 throughout: tolerances 1e-5 relative."""
import pytest
import torch
import torch.nn.functional as F

from oracle import cvt_ref
from vitmi import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / max(b.norm().item(), 1e-12)).item()


def torch_patches(x_nhwc, k, s, pad):
    """reference patch rows in (kh, kw, c) order: x NHWC [B,H,W,C]; pad = (pt, pb, pl, pr)"""
    B, H, W, C = x_nhwc.shape
    xp = F.pad(x_nhwc.permute(0, 3, 1, 2), (pad[2], pad[3], pad[0], pad[1]))
    u = F.unfold(xp, k, stride=s)                       # [B, C*k*k, L], order (c, kh, kw)
    L = u.shape[-1]
    u = u.view(B, C, k * k, L).permute(0, 3, 2, 1)       # [B, L, kk, C]
    return u.reshape(B * L, k * k * C)


@pytest.mark.parametrize("B,H,C,k,s,padding", [(2, 128, 1, 7, 4, None), (3, 32, 64, 3, 2, None),
                                               (2, 16, 128, 3, 2, None), (2, 32, 4, 7, 4, 2), (2, 8, 64, 3, 2, 1)])
def test_conv_im2col_col2im(B, H, C, k, s, padding):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(B, H, H, C, generator=g)
    Ho, pt, pb = cvt_ref.conv_geometry(H, k, s, padding)
    geo = (Ho, Ho, pt, pt) if padding is not None else ops.conv_same_geometry(H, H, k, s)
    assert geo[0] == Ho and geo[2] == pt
    K = k * k * C
    Kp = (K + 63) // 64 * 64
    pat = ops.conv_im2col(x.view(B * H * H, C).to(DEV), B, H, H, C, k, s, geo, Kp, torch.float32)
    ref = torch_patches(x, k, s, (pt, pb, pt, pb))
    assert torch.equal(pat[:, :K].cpu(), ref)
    assert torch.count_nonzero(pat[:, K:]).item() == 0
    if C % 4 == 0:
        # adjoint: <im2col(x), P> == <x, col2im(P)>
        P = torch.randn(B * Ho * Ho, Kp, generator=g)
        P[:, K:] = 0
        dx = torch.zeros(B * H * H, C, device=DEV)
        ops.conv_col2im(P.to(DEV), B, H, H, C, k, s, geo, dx)
        lhs = (ref.double() * P[:, :K].double()).sum().item()
        rhs = (x.view(-1, C).double() * dx.cpu().double()).sum().item()
        assert abs(lhs - rhs) <= 1e-5 * max(1.0, abs(lhs))
        # accumulate mode adds
        dx2 = torch.ones(B * H * H, C, device=DEV)
        ops.conv_col2im(P.to(DEV), B, H, H, C, k, s, geo, dx2, accumulate=True)
        assert torch.allclose(dx2, dx + 1, atol=1e-5)


def test_conv_im2col_bf16_and_strided_rows():
    # stage-3-like input rows: images of 1 + H*W rows, pixel rows after the cls row
    B, H, C, k, s = 2, 8, 64, 3, 2
    g = torch.Generator().manual_seed(1)
    x = torch.randn(B, 1 + H * H, C, generator=g)
    geo = ops.conv_same_geometry(H, H, k, s)
    pat = ops.conv_im2col(x.view(-1, C).to(DEV), B, H, H, C, k, s, geo, 9 * C, torch.bfloat16,
                          img_stride=1 + H * H, row_off=1)
    Ho, pt, pb = cvt_ref.conv_geometry(H, k, s, None)
    ref = torch_patches(x[:, 1:].reshape(B, H, H, C), k, s, (pt, pb, pt, pb))
    assert torch.equal(pat.cpu(), ref.to(torch.bfloat16))


def dwbn_ref(x_sp, w, gamma, beta, eps):
    """x_sp [B, H, W, C] -> BN(dwconv(x)) NHWC, via the oracle"""
    y = cvt_ref.dw_bn(x_sp.permute(0, 3, 1, 2), w, gamma, beta, eps)
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize("B,H,C,cls", [(4, 32, 64, False), (3, 16, 128, False), (5, 8, 256, True), (2, 7, 64, True)])
def test_dwconv_bn_fwd_bwd(B, H, C, cls):
    g = torch.Generator().manual_seed(2)
    N = H * H + (1 if cls else 0)
    off = 1 if cls else 0
    x = torch.randn(B, N, C, generator=g)
    w = 0.3 * torch.randn(C, 1, 3, 3, generator=g)
    gamma = 1 + 0.1 * torch.randn(C, generator=g)
    beta = 0.1 * torch.randn(C, generator=g)
    eps = 1e-3
    # CPU reference with autograd
    xs = x[:, off:].reshape(B, H, H, C).clone().requires_grad_(True)
    wr, gr, br = (t.clone().requires_grad_(True) for t in (w, gamma, beta))
    yref = dwbn_ref(xs, wr, gr, br, eps)
    dy = torch.randn(B, H, H, C, generator=g)
    (yref * dy).sum().backward()
    # device: y written into rows of a [B, N, C] buffer after the cls row
    w9 = w.view(C, 9).t().contiguous().to(DEV)          # [3][3][C]
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    y = torch.zeros(B, N, C, device=DEV)
    xd = x.to(DEV)
    z, mean, rstd = ops.dwconv_bn_fwd(xd.view(-1, C), B, H, H, w9, gamma.to(DEV), beta.to(DEV), eps, 0.99, True, rm, rv,
                                      y.view(-1, C), x_img=N, x_off=off, y_img=N, y_off=off)
    assert rel(y[:, off:].reshape(B, H, H, C), yref) < 1e-5
    if cls:
        assert torch.count_nonzero(y[:, 0]).item() == 0
    # moving statistics (Keras convention, biased batch variance)
    zr = F.conv2d(xs.detach().permute(0, 3, 1, 2), w, None, padding=1, groups=C)
    assert rel(rm, 0.01 * zr.mean(dim=(0, 2, 3))) < 1e-5
    assert rel(rv, 0.99 + 0.01 * zr.var(dim=(0, 2, 3), unbiased=True)) < 1e-5
    # backward
    dyd = torch.zeros(B, N, C, device=DEV)
    dyd[:, off:] = dy.view(B, H * H, C).to(DEV)
    dx = torch.zeros(B, N, C, device=DEV)
    dw9 = torch.zeros(9, C, device=DEV)
    dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    ops.dwconv_bn_bwd(dyd.view(-1, C), xd.view(-1, C), B, H, H, w9, gamma.to(DEV), z, mean, rstd, dx.view(-1, C), dw9,
                      dg, db, x_img=N, x_off=off, dy_img=N, dy_off=off)
    assert rel(dx[:, off:].reshape(B, H, H, C), xs.grad) < 1e-5
    if cls:
        assert torch.count_nonzero(dx[:, 0]).item() == 0
    assert rel(dw9.t().reshape(C, 1, 3, 3), wr.grad) < 1e-5
    assert rel(dg, gr.grad) < 1e-5
    assert rel(db, br.grad) < 1e-5


def test_dwconv_bn_inference_uses_moving_stats():
    B, H, C = 2, 8, 64
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B * H * H, C, generator=g)
    w = 0.3 * torch.randn(C, 1, 3, 3, generator=g)
    rm, rv = 0.1 * torch.randn(C, generator=g), 0.5 + torch.rand(C, generator=g)
    gamma, beta = torch.ones(C), torch.zeros(C)
    y = torch.empty(B * H * H, C, device=DEV)
    ops.dwconv_bn_fwd(x.to(DEV), B, H, H, w.view(C, 9).t().contiguous().to(DEV), gamma.to(DEV), beta.to(DEV), 1e-3,
                      0.99, False, rm.to(DEV), rv.to(DEV), y)
    z = F.conv2d(x.view(B, H, H, C).permute(0, 3, 1, 2), w, None, padding=1, groups=C)
    ref = F.batch_norm(z, rm, rv, gamma, beta, training=False, eps=1e-3).permute(0, 2, 3, 1).reshape(-1, C)
    assert rel(y, ref) < 1e-5


@pytest.mark.parametrize("B,H,C,cls,count_pad", [(3, 8, 64, False, False), (2, 7, 128, True, False),
                                                 (2, 16, 64, False, True), (2, 5, 256, True, True)])
def test_avgpool3_fwd_bwd(B, H, C, cls, count_pad):
    """Projection('avg') (models/CvT(Par).py:95-96): 3x3 stride-1 'same' average pooling; the
    TF divisor counts in-bounds taps, count_pad divides by 9 (torch, MS_CvT)."""
    g = torch.Generator().manual_seed(4)
    N = H * H + (1 if cls else 0)
    off = 1 if cls else 0
    x = torch.randn(B, N, C, generator=g)
    xs = x[:, off:].reshape(B, H, H, C).permute(0, 3, 1, 2).clone().requires_grad_(True)
    ref = F.avg_pool2d(xs, 3, 1, 1, count_include_pad=count_pad)
    dy = torch.randn_like(ref)
    (ref * dy).sum().backward()
    y = torch.zeros(B, N, C, device=DEV, dtype=torch.float32)
    ops.avgpool3_fwd(x.to(DEV).view(-1, C), B, H, H, y.view(-1, C), x_img=N, x_off=off, y_img=N, y_off=off,
                     count_pad=count_pad)
    assert rel(y[:, off:].reshape(B, H, H, C), ref.detach().permute(0, 2, 3, 1)) < 1e-6
    dyd = torch.zeros(B, N, C, device=DEV)
    dyd[:, off:] = dy.permute(0, 2, 3, 1).reshape(B, H * H, C).to(DEV)
    dx = torch.ones(B, N, C, device=DEV)
    ops.avgpool3_bwd(dyd.view(-1, C), B, H, H, dx.view(-1, C), dy_img=N, dy_off=off, x_img=N, x_off=off,
                     count_pad=count_pad)
    assert rel(dx[:, off:].reshape(B, H, H, C) - 1, xs.grad.permute(0, 2, 3, 1)) < 1e-6
    if cls:
        assert torch.equal(dx[:, 0], torch.ones(B, C, device=DEV))
    yb = torch.zeros(B, N, C, device=DEV, dtype=torch.bfloat16)
    ops.avgpool3_fwd(x.to(DEV).view(-1, C), B, H, H, yb.view(-1, C), x_img=N, x_off=off, y_img=N, y_off=off,
                     count_pad=count_pad)
    assert torch.equal(yb.float(), y.to(torch.bfloat16).float())
