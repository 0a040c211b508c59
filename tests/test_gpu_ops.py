"""Per-kernel numerics on the MI355X: every HIP kernel against a plain PyTorch fp32
reference of the same op (computed on the CPU from the same rounded inputs)."""


import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from vitmi import ops  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1.0)).item()


def rnd(*shape, dtype=torch.float32, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dtype)


# ------------------------------------------------------------------ GEMM
@pytest.fixture(params=[1, 2, 3], ids=["tile128", "tile256", "tile256-persistent8"])
def policy(request):
    """Run each GEMM case through both kernels (vitmi_gemm_set_policy)."""
    from vitmi._lib import lib
    lib().vitmi_gemm_set_policy(request.param)
    yield request.param
    lib().vitmi_gemm_set_policy(0)


FWD_SHAPES = [(197 * 3, 320, 192), (256, 384, 64), (1000, 2304, 768), (5, 64, 128)]


@pytest.mark.parametrize("M,N,K", FWD_SHAPES)
@pytest.mark.parametrize("T", [BF, torch.float32])
def test_linear_fwd_store(M, N, K, T, policy):
    x, w, b = rnd(M, K, dtype=T, seed=1), rnd(N, K, dtype=T, seed=2, scale=0.05), rnd(N, seed=3)
    ref = x.float() @ w.float().t() + b
    y32 = ops.linear_fwd(x.to(DEV), w.to(DEV), b.to(DEV), torch.float32)
    assert rel(y32, ref) < 1e-5
    y = ops.linear_fwd(x.to(DEV), w.to(DEV), b.to(DEV), T)
    assert rel(y.float(), ref) < (8e-3 if T == BF else 1e-5)


def gelu_grad(u):
    """d/du of the exact-erf GELU: Phi(u) + u phi(u)."""
    return 0.5 * (1 + torch.erf(u / 2 ** 0.5)) + u * torch.exp(-0.5 * u * u) / (2 * torch.pi) ** 0.5


@pytest.mark.parametrize("T", [BF, torch.float32])
def test_linear_fwd_gelu_and_residual(T, policy):
    M, N, K = 394, 768, 192
    x, w, b = rnd(M, K, dtype=T, seed=4), rnd(N, K, dtype=T, seed=5, scale=0.05), rnd(N, seed=6)
    u_ref = x.float() @ w.float().t() + b
    a, gp = ops.linear_fwd(x.to(DEV), w.to(DEV), b.to(DEV), T, ops.EPI_BIAS_GELU)
    assert rel(gp.float(), gelu_grad(u_ref)) < (8e-3 if T == BF else 1e-5)   # saved gelu'(u)
    assert rel(a.float(), F.gelu(u_ref)) < (8e-3 if T == BF else 1e-5)
    r = rnd(M, N, seed=7)
    y = ops.linear_fwd(x.to(DEV), w.to(DEV), b.to(DEV), torch.float32, ops.EPI_RESIDUAL, residual=r.to(DEV))
    assert rel(y, u_ref + r) < 1e-5


@pytest.mark.parametrize("M,N,K", [(394, 768, 192), (197 * 4, 2304, 768), (64, 192, 576)])
@pytest.mark.parametrize("T", [BF, torch.float32])
def test_linear_dgrad(M, N, K, T, policy):
    dy, w = rnd(M, N, dtype=T, seed=8), rnd(N, K, dtype=T, seed=9, scale=0.05)
    ref = dy.float() @ w.float()
    dx = ops.linear_dgrad(dy.to(DEV), w.to(DEV), torch.float32)
    assert rel(dx, ref) < 1e-5
    u = rnd(M, K, seed=10)
    gp = gelu_grad(u).to(T)                       # what the BIAS_GELU forward saved
    dg = ops.linear_dgrad(dy.to(DEV), w.to(DEV), T, ops.EPI_DGELU, aux=gp.to(DEV))
    uu = u.requires_grad_(True)
    gl = torch.autograd.grad(F.gelu(uu), uu, ref)[0]
    assert rel(dg.float(), gl) < (8e-3 if T == BF else 1e-5)


@pytest.mark.parametrize("M,N,K", [(256 * 9, 256, 768), (256 * 8 + 100, 256 + 64, 512), (256 * 17, 256, 256)])
def test_gemm_tail_split(M, N, K):
    """Persistent gemm256 on an 8-block grid (policy 3): the tiles of an under-filled last
    round are split over K into fp32 partials + fix-up kernel.  Every epilogue goes through
    the fix-up path; the workspace query must size it."""
    from vitmi._lib import lib
    lib().vitmi_gemm_set_policy(3)
    try:
        assert lib().vitmi_linear_fwd_workspace_size(1, M, N, K) > 0
        x, w, b = rnd(M, K, dtype=BF, seed=41), rnd(N, K, dtype=BF, seed=42, scale=0.05), rnd(N, seed=43)
        u_ref = x.float() @ w.float().t() + b
        y = ops.linear_fwd(x.to(DEV), w.to(DEV), b.to(DEV), BF)
        assert rel(y.float(), u_ref) < 8e-3
        a, gp = ops.linear_fwd(x.to(DEV), w.to(DEV), b.to(DEV), BF, ops.EPI_BIAS_GELU)
        assert rel(a.float(), F.gelu(u_ref)) < 8e-3
        assert rel(gp.float(), gelu_grad(u_ref)) < 8e-3
        r = rnd(M, N, seed=44)
        y2 = ops.linear_fwd(x.to(DEV), w.to(DEV), b.to(DEV), torch.float32, ops.EPI_RESIDUAL, residual=r.to(DEV))
        assert rel(y2, u_ref + r) < 1e-5
        # dgrad: dx[M,K'] = dy[M,N'] W[N',K'] with the output [M, N] -> reduction K
        dy, w2 = rnd(M, K, dtype=BF, seed=45), rnd(K, N, dtype=BF, seed=46, scale=0.05)
        ref = dy.float() @ w2.float()
        gpv = gelu_grad(rnd(M, N, seed=47)).to(BF)
        dx = ops.linear_dgrad(dy.to(DEV), w2.to(DEV), BF, ops.EPI_DGELU, aux=gpv.to(DEV))
        assert rel(dx.float(), ref * gpv.float()) < 8e-3
    finally:
        lib().vitmi_gemm_set_policy(0)


@pytest.mark.parametrize("M,N,K,fpol,bpol", [(197 * 8 + 3, 1024, 256, 0, 0),      # gemm256, ragged M
                                              (256 * 8 + 100, 256 + 64, 512, 3, 3),  # tail split + fix-up
                                              (300, 320, 192, 1, 2),   # forward on the 128x128 kernel
                                              (300, 320, 192, 2, 1)])  # backward on the 128x128 kernel
def test_aux_tiled_matches_row_major(M, N, K, fpol, bpol):
    """gelu' in the tile-native layout (VITMI_EPI_AUX_TILED): the GELU activation (plain and
    with dropout) and the DGELU dgrad with its fused bias gradient are bit-identical to the
    row-major layout's, whichever kernel wrote gelu' and whichever read it."""
    from vitmi._lib import lib
    x, w, b = rnd(M, K, dtype=BF, seed=61).to(DEV), rnd(N, K, dtype=BF, seed=62, scale=0.05).to(DEV), rnd(N, seed=63).to(DEV)
    dy, w2 = rnd(M, 384, dtype=BF, seed=64).to(DEV), rnd(384, N, dtype=BF, seed=65, scale=0.05).to(DEV)
    out = {}
    try:
        for tiled in (False, True):
            lib().vitmi_gemm_set_policy(fpol)
            a, u = ops.linear_fwd(x, w, b, BF, ops.EPI_BIAS_GELU, aux_tiled=tiled)
            ad, ud = ops.linear_fwd(x, w, b, BF, ops.EPI_BIAS_GELU, dropout=(5, 2, 0.25), aux_tiled=tiled)
            if tiled:
                assert u.numel() * 2 == lib().vitmi_aux_tiled_bytes(M, N)
            lib().vitmi_gemm_set_policy(bpol)
            db = torch.zeros(N, device=DEV)
            dx = ops.linear_dgrad(dy, w2, BF, ops.EPI_DGELU, aux=u, bias_grad=db, aux_tiled=tiled)
            dxd = ops.linear_dgrad(dy, w2, BF, ops.EPI_DGELU, aux=ud, aux_tiled=tiled)
            out[tiled] = (a, ad, dx, db, dxd)
    finally:
        lib().vitmi_gemm_set_policy(0)
    for name, r, t in zip(("gelu", "gelu+dropout", "dgelu", "bias grad", "dgelu+dropout"), out[False], out[True]):
        assert torch.equal(r, t), name
    ref = (dy.float() @ w2.float()).cpu() * gelu_grad((x.float() @ w.float().t() + b).cpu())
    assert rel(out[True][2].float(), ref) < 8e-3


def test_gemm_tail_split_vit_shape():
    """The ViT-B/16 bs=256 N=768 shape on the real grid (591 tiles over the device's CUs),
    against torch's own GEMM on the GPU (the CPU reference would take minutes)."""
    M, N, K = 256 * 197, 768, 3072
    g = torch.Generator(device=DEV).manual_seed(5)
    h = (torch.rand(M, K, device=DEV, generator=g) * 2 - 1).to(BF)
    w2 = ((torch.rand(N, K, device=DEV, generator=g) * 2 - 1) * 0.05).to(BF)
    b2 = torch.rand(N, device=DEV, generator=g)
    res = torch.rand(M, N, device=DEV, generator=g)
    y = ops.linear_fwd(h, w2, b2, torch.float32, ops.EPI_RESIDUAL, residual=res)
    ref = res + h.float() @ w2.float().t() + b2
    assert ((y - ref).norm() / ref.norm()).item() < 1e-5
    dx = ops.linear_dgrad(h, w2.t().contiguous(), BF)          # [M,K] x [K,N] -> [M,N]
    ref2 = h.float() @ w2.float().t()
    assert ((dx.float() - ref2).norm() / ref2.norm()).item() < 8e-3


@pytest.mark.parametrize("M,N,K", [(197 * 2, 384, 192), (4000, 384, 768), (50, 64, 64), (20000, 192, 576)])
@pytest.mark.parametrize("T", [BF, torch.float32])
def test_linear_wgrad_accumulates(M, N, K, T, policy):
    dy, x = rnd(M, N, dtype=T, seed=11), rnd(M, K, dtype=T, seed=12)
    prev = rnd(N, K, seed=13)
    ref = prev + dy.float().t() @ x.float()
    dw = prev.clone().to(DEV)
    ops.linear_wgrad(dy.to(DEV), x.to(DEV), dw)
    assert rel(dw, ref) < 2e-5


@pytest.mark.parametrize("M,N,K", [(197 * 64, 768, 768), (197 * 32 + 5, 2304, 768), (9000, 768, 3072)])
def test_linear_wgrad_split_units(M, N, K):
    """Default policy at ViT shapes: gemm256 split-K folded into the persistent unit space
    (unit = slab * tiles + tile), with ragged reduction length."""
    dy, x = rnd(M, N, dtype=BF, seed=21), rnd(M, K, dtype=BF, seed=22)
    prev = rnd(N, K, seed=23)
    ref = prev + dy.float().t() @ x.float()
    dw = prev.clone().to(DEV)
    ops.linear_wgrad(dy.to(DEV), x.to(DEV), dw)
    assert rel(dw, ref) < 2e-5


@pytest.mark.parametrize("M,shapes", [
    (197 * 24, [(768, 3072), (3072, 768), (768, 768), (2304, 768)]),   # a ViT-B block's four wgrads
    (197 * 16 + 37, [(256, 512), (520, 264)]),                          # ragged rows and tile edges
    (4000, [(1024, 4096), (4096, 1024), (3072, 1024)]),                 # ViT-L-like, three problems
])
def test_linear_wgrad_group_matches_oracle(M, shapes):
    """vitmi_linear_wgrad_group: every problem's dW += dy^T x in one grouped launch (the split-K
    units of all problems in one persistent unit space) and one segment reduction, onto nonzero
    dW; one x row-strided (the hi part of a split operand).  Reference: fp32 products of the same
    bf16 operands.  Also run twice: bitwise deterministic."""
    items, refs = [], []
    for i, (n, k) in enumerate(shapes):
        dy = rnd(M, n, dtype=BF, seed=70 + 3 * i)
        xw = rnd(M, k + (8 if i == 1 else 0), dtype=BF, seed=71 + 3 * i)
        x = xw[:, :k]
        prev = rnd(n, k, seed=72 + 3 * i)
        refs.append(prev + dy.float().t() @ x.float())
        items.append((dy.to(DEV), xw.to(DEV)[:, :k], prev.to(DEV)))
    outs = []
    for _ in range(2):
        dws = [p.clone() for _, _, p in items]
        ops.linear_wgrad_group([(dy, x, dw) for (dy, x, _), dw in zip(items, dws)])
        torch.cuda.synchronize()
        outs.append(dws)
    for dw, ref in zip(outs[0], refs):
        assert rel(dw, ref) < 2e-5
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)


def test_linear_wgrad_group_falls_back_per_problem():
    """fp32 operands (and a bf16 group with one item) take the per-problem path: same results as
    ops.linear_wgrad."""
    M = 700
    its = [(rnd(M, 96, seed=81).to(DEV), rnd(M, 64, seed=82).to(DEV)),
           (rnd(M, 128, seed=83).to(DEV), rnd(M, 32, seed=84).to(DEV))]
    dws = [torch.zeros(96, 64, device=DEV), torch.zeros(128, 32, device=DEV)]
    ops.linear_wgrad_group([(dy, x, dw) for (dy, x), dw in zip(its, dws)])
    for (dy, x), dw in zip(its, dws):
        assert rel(dw, dy.t() @ x) < 1e-5
    dy, x = rnd(M, 256, dtype=BF, seed=85).to(DEV), rnd(M, 256, dtype=BF, seed=86).to(DEV)
    a, b = torch.zeros(256, 256, device=DEV), torch.zeros(256, 256, device=DEV)
    ops.linear_wgrad_group([(dy, x, a)])
    ops.linear_wgrad(dy, x, b)
    assert torch.equal(a, b)


@pytest.mark.parametrize("M,N,K", [(256 * 5 + 40, 768, 512), (296, 264, 128)])
def test_gemm_tn_layout_epilogues(M, N, K, policy):
    """The TN layout (A and B both m/n-major, the weight-gradient operands) through the generic
    entry with bf16 store, bias+GELU and fp32 residual epilogues: gemm256 remaps its half-tiles to
    contiguous 128-line blocks there (line_of<.., RMP>), so every epilogue's row/column mapping is
    exercised, ragged N included."""
    a = rnd(K, M, dtype=BF, seed=51)                 # A(m,k) at a[k][m]
    b = rnd(K, N, dtype=BF, seed=52, scale=0.05)     # B(k,n) at b[k][n]
    bias = rnd(N, seed=53)
    ref = a.float().t() @ b.float()
    ad, bd = a.to(DEV), b.to(DEV)
    y = ops.gemm(ad, bd, False, False, M, N, K, torch.empty(M, N, dtype=BF, device=DEV), ops.EPI_STORE,
                 bias=bias.to(DEV))
    assert rel(y.float(), ref + bias) < 8e-3
    gp = torch.empty(M, N, dtype=BF, device=DEV)
    a_ = ops.gemm(ad, bd, False, False, M, N, K, torch.empty(M, N, dtype=BF, device=DEV), ops.EPI_BIAS_GELU,
                  bias=bias.to(DEV), aux=gp)
    assert rel(a_.float(), F.gelu(ref + bias)) < 8e-3
    assert rel(gp.float(), gelu_grad(ref + bias)) < 8e-3
    res = rnd(M, N, seed=54)
    y2 = ops.gemm(ad, bd, False, False, M, N, K, torch.empty(M, N, device=DEV), ops.EPI_RESIDUAL,
                  bias=bias.to(DEV), residual=res.to(DEV))
    assert rel(y2, ref + bias + res) < 1e-5


@pytest.mark.parametrize("M,N,K,T,epi", [(197 * 64 + 3, 768, 3072, BF, "dgelu"), (50432 // 8, 768, 3072, BF, "dgelu"),
                                         (197 * 8, 256, 1024, BF, "dgelu"), (300, 128, 512, BF, "store"),
                                         (197 * 4, 768, 3072, torch.float32, "dgelu")])
def test_linear_dgrad_fused_bias(M, N, K, T, epi):
    """dgrad + the column sums of its output (fc1's bias gradient): fused into the gemm256
    DGELU epilogue for bf16 (ragged M), a second pass elsewhere; == dgrad then bias_grad."""
    dy = rnd(M, N, dtype=T, seed=31)
    w = (rnd(N, K, seed=32) * 0.05).to(T)
    aux = (rnd(M, K, seed=33).abs() + 0.1).to(T) if epi == "dgelu" else None
    e = ops.EPI_DGELU if epi == "dgelu" else ops.EPI_STORE
    dyd, wd = dy.to(DEV), w.to(DEV).contiguous()
    auxd = aux.to(DEV) if aux is not None else None
    ref = ops.linear_dgrad(dyd, wd, T, e, aux=auxd)
    db_ref = torch.full((K,), 0.5, device=DEV)
    ops.bias_grad(ref, db_ref)
    db = torch.full((K,), 0.5, device=DEV)
    dx = ops.linear_dgrad(dyd, wd, T, e, aux=auxd, bias_grad=db)
    # (the fused launch runs without the tail K-split: last-round tiles may round differently)
    assert rel(dx, ref) < (3e-3 if T == BF else 1e-6)
    # fused sums add the fp32 values before the bf16 rounding of dx: within bf16 noise
    tol = 2e-3 if T == BF else 1e-5
    assert rel(db, db_ref) < tol
    dxf = ref.float()
    assert rel(db - 0.5, dxf.sum(0)) < tol


@pytest.mark.parametrize("T", [BF, torch.float32])
def test_bias_grad(T):
    dy = rnd(197 * 3 + 1, 2304, dtype=T, seed=14)
    db = torch.ones(2304, device=DEV)
    ops.bias_grad(dy.to(DEV), db)
    assert rel(db, 1 + dy.float().sum(0)) < 1e-5


# ------------------------------------------------------------------ LayerNorm
@pytest.mark.parametrize("D", [64, 128, 192, 384, 768, 1024])
@pytest.mark.parametrize("T", [BF, torch.float32])
def test_layernorm_fwd_bwd(D, T):
    M = 197 * 2 + 3
    x = rnd(M, D, seed=15) * 2 + 0.5
    w, b = 1 + 0.1 * rnd(D, seed=16), 0.1 * rnd(D, seed=17)
    y, mean, rstd = ops.layernorm_fwd(x.to(DEV), w.to(DEV), b.to(DEV), 1e-6, T)
    ref = F.layer_norm(x, (D,), w, b, 1e-6)
    assert rel(y.float(), ref) < (5e-3 if T == BF else 1e-6)
    dy = rnd(M, D, seed=18).to(T)
    dres = rnd(M, D, seed=19)
    dg, dbb = torch.full((D,), 0.5, device=DEV), torch.full((D,), -0.5, device=DEV)
    dsum = torch.full((D,), 2.0, device=DEV)
    dx, dx_lp = ops.layernorm_bwd(dy.to(DEV), x.to(DEV), mean, rstd, w.to(DEV), dg, dbb, dres=dres.to(DEV),
                                  lp_dtype=BF, dxsum=dsum)
    xx, ww, bb = x.clone().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()
    F.layer_norm(xx, (D,), ww, bb, 1e-6).backward(dy.float())
    assert rel(dx, xx.grad + dres) < 1e-5
    assert rel(dx_lp.float(), xx.grad + dres) < 5e-3
    assert rel(dg, 0.5 + ww.grad) < 1e-5
    assert rel(dbb, -0.5 + bb.grad) < 1e-5
    assert rel(dsum, 2.0 + (xx.grad + dres).sum(0)) < 1e-5   # fused bias-grad column sums


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("dy_dtype", [BF, torch.float32])
@pytest.mark.parametrize("with_dres", [False, True])
def test_layernorm_small_d_backward_variants(D, dy_dtype, with_dres):
    """the several-rows-per-wave LayerNorm kernels (D = 64 / 128: L = 16 / 32 lanes
    per row) without the residual gradient, without the bf16 copy, with an fp32 dy, and the
    forward and backward over strided rows (the head-LN pattern x[:, 0]), against F.layer_norm."""
    B, N = 37, 9
    x = rnd(B, N, D, seed=40) * 2 + 0.5
    w, b = 1 + 0.1 * rnd(D, seed=41), 0.1 * rnd(D, seed=42)
    xd = x.to(DEV)
    # contiguous rows, no dres, no bf16 copy
    y, mean, rstd = ops.layernorm_fwd(xd.view(B * N, D), w.to(DEV), b.to(DEV), 1e-6, torch.float32)
    assert rel(y, F.layer_norm(x.view(B * N, D), (D,), w, b, 1e-6)) < 1e-6
    dy = rnd(B * N, D, seed=43).to(dy_dtype)
    dres = rnd(B * N, D, seed=44) if with_dres else None
    dg, dbb = torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)
    dx, dx_lp = ops.layernorm_bwd(dy.to(DEV), xd.view(B * N, D), mean, rstd, w.to(DEV), dg, dbb,
                                  dres=dres.to(DEV) if with_dres else None, lp_dtype=None)
    assert dx_lp is None
    xx, ww, bb = x.view(B * N, D).clone().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()
    F.layer_norm(xx, (D,), ww, bb, 1e-6).backward(dy.float())
    want = xx.grad + (dres if with_dres else 0)
    assert rel(dx, want) < 1e-5
    assert rel(dg, ww.grad) < 1e-5 and rel(dbb, bb.grad) < 1e-5
    # strided rows (every image's cls row), fp32 and bf16 outputs, backward into strided dx
    for T in (torch.float32, BF):
        yc, mc, rc = ops.layernorm_fwd(xd[:, 0], w.to(DEV), b.to(DEV), 1e-6, T)
        assert rel(yc.float(), F.layer_norm(x[:, 0], (D,), w, b, 1e-6)) < (5e-3 if T == BF else 1e-6)
    dxs = torch.zeros(B, N, D, device=DEV)
    dyc = rnd(B, D, seed=45).to(dy_dtype)
    ops.layernorm_bwd(dyc.to(DEV), xd[:, 0], mc, rc, w.to(DEV), None, None, dx=dxs[:, 0])
    xc = x[:, 0].clone().requires_grad_()
    F.layer_norm(xc, (D,), w, b, 1e-6).backward(dyc.float())
    assert rel(dxs[:, 0], xc.grad) < 1e-5
    assert dxs[:, 1:].abs().max().item() == 0.0


def test_layernorm_strided_rows():
    B, N, D = 5, 17, 192
    x = rnd(B, N, D, seed=20)
    w, b = torch.ones(D), torch.zeros(D)
    xd = x.to(DEV)
    y, mean, rstd = ops.layernorm_fwd(xd[:, 0], w.to(DEV), b.to(DEV), 1e-6, torch.float32)
    assert rel(y, F.layer_norm(x[:, 0], (D,), w, b, 1e-6)) < 1e-6
    dx = torch.zeros(B, N, D, device=DEV)
    dy = rnd(B, D, seed=21)
    ops.layernorm_bwd(dy.to(DEV), xd[:, 0], mean, rstd, w.to(DEV), None, None, dx=dx[:, 0])
    xx = x[:, 0].clone().requires_grad_()
    F.layer_norm(xx, (D,), w, b, 1e-6).backward(dy)
    assert rel(dx[:, 0], xx.grad) < 1e-5
    assert dx[:, 1:].abs().max().item() == 0.0


# ------------------------------------------------------------------ attention
def attn_ref(qkv, B, N, H, scale):
    D = qkv.shape[-1] // 3
    q, k, v = qkv.float().view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-1, -2)) * scale
    p = s.softmax(-1)
    o = (p @ v).transpose(1, 2).reshape(B * N, D)
    lse = torch.logsumexp(s, -1).reshape(B * H, N)
    return o, lse


ATT = [(2, 197, 2), (1, 17, 3), (2, 64, 1), (1, 577, 2), (3, 1, 2), (1, 130, 1), (1, 256, 1), (2, 255, 1),
       (1, 33, 2), (1, 96, 1), (1, 300, 1)]


# bf16 N <= 256 runs the whole-sequence kernels; attention policy 1 forces the streamed ones, so
# both are checked at the same sizes (other cases run the streamed / fp32 kernels either way)
ATT_CASES = [(B, N, H, T, "seq") for T in (BF, torch.float32) for (B, N, H) in ATT] + \
            [(B, N, H, BF, "stream") for (B, N, H) in ATT if N <= 256]


@pytest.fixture
def attn_policy():
    prev = ops.attention_set_policy(0)
    yield lambda path: ops.attention_set_policy(1 if path == "stream" else 0)
    ops.attention_set_policy(prev)


@pytest.mark.parametrize("B,N,H,T,path", ATT_CASES)
def test_attention_fwd_bwd(B, N, H, T, path, attn_policy):
    attn_policy(path)
    D = 64 * H
    scale = 64 ** -0.5
    qkv = rnd(B * N, 3 * D, dtype=T, seed=22)
    o, lse = ops.attention_fwd(qkv.to(DEV), B, N, H, scale)
    o_ref, lse_ref = attn_ref(qkv, B, N, H, scale)
    tol = 1e-2 if T == BF else 1e-5
    assert rel(o.float(), o_ref) < tol
    assert rel(lse, lse_ref) < 1e-5
    do = rnd(B * N, D, dtype=T, seed=23)
    dqkv = ops.attention_bwd(qkv.to(DEV), o, do.to(DEV), lse, B, N, H, scale)
    qq = qkv.float().clone().requires_grad_()
    o2, _ = attn_ref(qq, B, N, H, scale)
    o2.backward(do.float())
    g = qq.grad.view(B * N, 3, D)
    d = dqkv.float().cpu().view(B * N, 3, D)
    for i, name in enumerate("qkv"):
        assert rel(d[:, i], g[:, i]) < (2e-2 if T == BF else 1e-5), name


@pytest.mark.parametrize("B,N,H", [(48, 197, 12), (24, 224, 12), (40, 193, 9), (3, 197, 1)])
def test_attention_persistent_many_pairs(B, N, H):
    """N in (192, 224] at many (batch, head) pairs: the persistent dK/dV kernel walks several
    pairs per workgroup with the next pair's Q | dO (inline-asm LDS-DMA) and K/V rows (inline-asm
    loads) in flight (more pairs than CUs here, and fewer: B*H = 3); vs the fp32 reference, vs
    the streamed kernels, and bitwise equal across runs."""
    D = 64 * H
    scale = 64 ** -0.5
    qkv = rnd(B * N, 3 * D, dtype=BF, seed=41)
    do = rnd(B * N, D, dtype=BF, seed=42)
    o, lse = ops.attention_fwd(qkv.to(DEV), B, N, H, scale)
    o_again, lse_again = ops.attention_fwd(qkv.to(DEV), B, N, H, scale)
    assert torch.equal(o, o_again) and torch.equal(lse, lse_again)
    o_ref, lse_ref = attn_ref(qkv, B, N, H, scale)
    assert rel(o.float(), o_ref) < 1e-2
    assert rel(lse, lse_ref) < 1e-5
    dqkv = ops.attention_bwd(qkv.to(DEV), o, do.to(DEV), lse, B, N, H, scale)
    assert torch.equal(dqkv, ops.attention_bwd(qkv.to(DEV), o, do.to(DEV), lse, B, N, H, scale))
    prev = ops.attention_set_policy(1)
    try:
        o_s, lse_s = ops.attention_fwd(qkv.to(DEV), B, N, H, scale)
        d_s = ops.attention_bwd(qkv.to(DEV), o_s, do.to(DEV), lse_s, B, N, H, scale)
    finally:
        ops.attention_set_policy(prev)
    assert rel(o.float(), o_s.float()) < 1e-2
    assert rel(dqkv.float(), d_s.float()) < 2e-2
    qq = qkv.float().clone().requires_grad_()
    o2, _ = attn_ref(qq, B, N, H, scale)
    o2.backward(do.float())
    g = qq.grad.view(B * N, 3, D)
    d = dqkv.float().cpu().view(B * N, 3, D)
    for i, name in enumerate("qkv"):
        assert rel(d[:, i], g[:, i]) < 2e-2, name


@pytest.mark.parametrize("B,N,H", [(48, 197, 12), (3, 224, 2), (2, 193, 1), (5, 64, 3), (2, 250, 2)])
def test_attention_64query_forms_bitwise_equal(B, N, H):
    """The whole-sequence forward and dQ run 4 waves of 64 queries (attn_fwd_seq64_bf16,
    attn_bwd_dq_seq64_bf16; policies 0 and 3); policy 2 runs the 32-query forms.  Per query block
    the arithmetic and the q-bias column-sum fold order are the same, so o and lse (policy 0 vs 2)
    and the two-kernel backward's dqkv and fused bias gradient (policy 3 vs 2) are bitwise equal."""
    D = 64 * H
    qkv = rnd(B * N, 3 * D, dtype=BF, seed=51).to(DEV)
    do = rnd(B * N, D, dtype=BF, seed=52).to(DEV)
    out = {}
    prev = ops.attention_set_policy(0)
    try:
        for pol in (0, 2, 3):
            ops.attention_set_policy(pol)
            o, lse = ops.attention_fwd(qkv, B, N, H, 0.125)
            db = torch.zeros(3 * D, device=DEV)
            dqkv = ops.attention_bwd(qkv, o, do, lse, B, N, H, 0.125, bias_grad=db)
            out[pol] = (o, lse, dqkv, db)
    finally:
        ops.attention_set_policy(prev)
    for a, b, name in zip(out[0][:2], out[2][:2], ("o", "lse")):
        assert torch.equal(a, b), name
    for a, b, name in zip(out[3][2:], out[2][2:], ("dqkv", "dbias")):
        assert torch.equal(a, b), name


@pytest.mark.parametrize("B,N,H", [(16, 197, 12), (3, 250, 2), (2, 33, 1)])
def test_attention_fwd_knob_outputs_64query_bitwise_equal(B, N, H):
    """The precision knobs' attention forward (vitmi_attention_fwd_x3 / _f8) in its 64-query form
    (auto policy, round 6) against the 32-query form (policy 2): o, lse and the split outputs o3 /
    o8 are bitwise equal (the same per-query-block arithmetic and the same fp32 O)."""
    D = 64 * H
    qkv = rnd(B * N, 3 * D, dtype=BF, seed=71).to(DEV)
    out = {}
    prev = ops.attention_set_policy(0)
    try:
        for pol in (0, 2):
            ops.attention_set_policy(pol)
            out[pol] = ops.attention_fwd_x3(qkv, B, N, H, 0.125) + ops.attention_fwd_f8(qkv, B, N, H, 0.125)
    finally:
        ops.attention_set_policy(prev)
    for a, b, name in zip(out[0], out[2], ("o", "o3", "lse", "o (f8)", "o8", "lse (f8)")):
        assert torch.equal(a, b), name


@pytest.mark.parametrize("B,N,H", [(48, 197, 12), (3, 224, 2), (2, 193, 1), (5, 64, 3), (2, 17, 3), (1, 1, 2),
                                   (3, 100, 2)])
def test_attention_single_pass_bwd_vs_two_kernel(B, N, H):
    """The single-pass whole-sequence backward (attn_bwd_fused_seq_bf16, auto policy, N <= 224)
    against the two-kernel one (policy 3): dK and dV are the dK/dV kernel's arithmetic in the same
    order (bitwise equal), dQ is dS K from the same dS the dK product takes (the two-kernel dQ
    recomputes dS in the swapped orientation: equal to bf16 rounding), the fused q/k/v bias
    gradient agrees likewise, and the single-pass result is bitwise reproducible."""
    D = 64 * H
    scale = 0.125
    qkv = rnd(B * N, 3 * D, dtype=BF, seed=61).to(DEV)
    do = rnd(B * N, D, dtype=BF, seed=62).to(DEV)
    prev = ops.attention_set_policy(0)
    try:
        o, lse = ops.attention_fwd(qkv, B, N, H, scale)
        db1 = torch.zeros(3 * D, device=DEV)
        d1 = ops.attention_bwd(qkv, o, do, lse, B, N, H, scale, bias_grad=db1)
        db1b = torch.zeros(3 * D, device=DEV)
        assert torch.equal(d1, ops.attention_bwd(qkv, o, do, lse, B, N, H, scale, bias_grad=db1b))
        assert torch.equal(db1, db1b)
        ops.attention_set_policy(3)
        db2 = torch.zeros(3 * D, device=DEV)
        d2 = ops.attention_bwd(qkv, o, do, lse, B, N, H, scale, bias_grad=db2)
    finally:
        ops.attention_set_policy(prev)
    a, b = d1.view(B * N, 3, D), d2.view(B * N, 3, D)
    assert torch.equal(a[:, 1:], b[:, 1:]), "dK / dV"
    assert torch.equal(db1[D:], db2[D:]), "k / v bias gradient"
    assert rel(a[:, 0].float(), b[:, 0].float()) < 1e-2, "dQ"
    assert rel(db1[:D], db2[:D]) < 1e-2, "q bias gradient"
    # and against the fp32 reference
    qq = qkv.float().cpu().clone().requires_grad_()
    o2, _ = attn_ref(qq, B, N, H, scale)
    o2.backward(do.float().cpu())
    g = qq.grad.view(B * N, 3, D)
    for i, name in enumerate("qkv"):
        assert rel(a[:, i].float().cpu(), g[:, i]) < 2e-2, name


@pytest.mark.parametrize("B,N,H,T", [(2, 197, 2, BF), (3, 17, 1, BF), (1, 256, 3, BF), (2, 1, 2, BF),
                                     (2, 300, 1, BF), (3, 577, 2, BF), (2, 33, 2, torch.float32)])
def test_attention_bwd_fused_bias(B, N, H, T):
    """the q/k/v bias gradient out of the attention backward kernels (column sums of the dQ,
    dK, dV tiles as stored, formed from the LDS image they leave through) == a column-sum pass
    over dqkv up to the summation order"""
    D = 64 * H
    qkv = rnd(B * N, 3 * D, dtype=T, seed=25).to(DEV)
    o, lse = ops.attention_fwd(qkv, B, N, H, 0.125)
    do = rnd(B * N, D, dtype=T, seed=26).to(DEV)
    ref = ops.attention_bwd(qkv, o, do, lse, B, N, H, 0.125)
    db_ref = torch.full((3 * D,), 0.25, device=DEV)
    ops.bias_grad(ref, db_ref)
    db = torch.full((3 * D,), 0.25, device=DEV)
    dqkv = ops.attention_bwd(qkv, o, do, lse, B, N, H, 0.125, bias_grad=db, fused_bias=True)
    assert torch.equal(dqkv, ref)
    # the fused sums add the same bf16-rounded values in another order
    assert rel(db, db_ref) < 1e-5
    assert rel(db - 0.25, ref.float().sum(0)) < 1e-5


@pytest.mark.parametrize("path", ["seq", "stream"])
def test_attention_softmax_spike(path, attn_policy):
    """A key row that dominates one query forces the online-softmax rescale branch."""
    attn_policy(path)
    B, N, H = 1, 197, 1
    qkv = rnd(B * N, 192, seed=24) * 0.5
    qkv[150, 64:128] = qkv[3, 0:64] * 40   # k_150 aligned with q_3 -> huge score at tile 2
    qkv = qkv.to(BF)
    o, lse = ops.attention_fwd(qkv.to(DEV), B, N, H, 0.125)
    o_ref, lse_ref = attn_ref(qkv, B, N, H, 0.125)
    assert rel(o.float(), o_ref) < 1e-2
    assert rel(lse, lse_ref) < 1e-5


# ------------------------------------------------------------------ embed / head / loss / cast
@pytest.mark.parametrize("C,S,P", [(3, 64, 16), (1, 32, 8), (3, 224, 16)])
@pytest.mark.parametrize("T", [BF, torch.float32])
def test_im2col(C, S, P, T):
    img = torch.rand(2, C, S, S)
    out = ops.patch_im2col(img.to(DEV), P, T)
    G = S // P
    ref = img.view(2, C, G, P, G, P).permute(0, 2, 4, 1, 3, 5).reshape(2 * G * G, C * P * P)
    assert torch.equal(out.cpu(), ref.to(T))


@pytest.mark.parametrize("B", [3, 11])
def test_tokens_assemble_roundtrip(B):
    np_, D = 16, 192
    tok, cls, pos = rnd(B * np_, D, seed=25), rnd(D, seed=26), rnd(np_ + 1, D, seed=27)
    x = ops.tokens_assemble(tok.to(DEV), B, np_, cls.to(DEV), pos.to(DEV))
    ref = torch.cat([cls.expand(B, 1, D), tok.view(B, np_, D)], 1) + pos
    assert torch.allclose(x.cpu(), ref)
    dx = rnd(B, np_ + 1, D, seed=28)
    dcls, dpos = torch.zeros(D, device=DEV), torch.ones((np_ + 1) * D, device=DEV)
    dtok, dtok_lp = ops.tokens_assemble_bwd(dx.to(DEV), B, np_, True, BF, dcls, dpos)
    assert torch.equal(dtok.cpu(), dx[:, 1:].reshape(B * np_, D))
    assert torch.equal(dtok_lp.cpu(), dx[:, 1:].reshape(B * np_, D).to(BF))
    assert rel(dpos.view(np_ + 1, D), 1 + dx.sum(0)) < 1e-6
    assert rel(dcls, dx[:, 0].sum(0)) < 1e-6


@pytest.mark.parametrize("B,D,C", [(37, 192, 3), (300, 768, 1000)])
def test_head_and_losses(B, D, C):
    y, w, b = rnd(B, D, seed=29), rnd(C, D, seed=30), rnd(C, seed=31)
    logits = ops.head_fwd(y.to(DEV), w.to(DEV), b.to(DEV))
    assert rel(logits, y @ w.t() + b) < 1e-6
    tgt = torch.randint(0, C, (B,))
    loss, dl = ops.loss_fwd_bwd(logits, tgt.to(DEV), ops.LOSS_CE)
    z = (y @ w.t() + b).requires_grad_()
    ref = F.cross_entropy(z, tgt)
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-5 * max(1.0, abs(ref.item()))
    assert rel(dl, z.grad) < 1e-5
    t2 = rnd(B, C, seed=32)
    loss2, dl2 = ops.loss_fwd_bwd(logits, t2.to(DEV), ops.LOSS_MSE)
    z2 = (y @ w.t() + b).requires_grad_()
    r2 = F.mse_loss(z2, t2)
    r2.backward()
    assert abs(loss2.item() - r2.item()) < 1e-5 * max(1.0, abs(r2.item())) and rel(dl2, z2.grad) < 1e-5
    dw, db = torch.zeros(C, D, device=DEV), torch.zeros(C, device=DEV)
    dy = ops.head_bwd(dl, y.to(DEV), w.to(DEV), dw, db)
    assert rel(dy, z.grad @ w) < 1e-5
    assert rel(dw, z.grad.t() @ y) < 1e-5 and rel(db, z.grad.sum(0)) < 1e-5


def test_cast():
    x = rnd(1000003, seed=33)
    y = ops.cast_bf16(x.to(DEV))
    assert torch.equal(y.cpu(), x.to(BF))





@pytest.mark.parametrize("rows,K", [(197 * 3, 768), (37, 3072), (5, 4)])
def test_split_bf16x3_layout_and_residual(rows, K):
    """vitmi_split_bf16x3: hi = bf16(x), lo = bf16(x - hi) in the [hi | hi | lo] / [hi | lo | hi]
    layouts (row-strided source), hi + lo within 2^-16 of x, and the optional hi copy."""
    x = (rnd(rows, K + 8, seed=91) * 3).to(DEV)[:, 4:4 + K]
    x = x.contiguous() if (x.data_ptr() % 16) else x
    a3, hi = ops.split_bf16x3(x, 0, hi_copy=True)
    w3, none = ops.split_bf16x3(x, 1)
    assert none is None
    h = x.to(BF)
    lo = (x - h.float()).to(BF)
    assert torch.equal(a3[:, :K], h) and torch.equal(a3[:, K:2 * K], h) and torch.equal(a3[:, 2 * K:], lo)
    assert torch.equal(w3[:, :K], h) and torch.equal(w3[:, K:2 * K], lo) and torch.equal(w3[:, 2 * K:], h)
    assert torch.equal(hi, h)
    assert ((h.float() + lo.float() - x).abs() <= x.abs() * 2.0 ** -16 + 1e-30).all()


def test_bf16x3_gemm_is_fp32_accurate():
    """One GEMM over K' = 3K of the split operands (hi.hi + hi.lo + lo.hi) against an fp64
    product: ~2^-16 relative, where the plain bf16 GEMM is ~2^-9."""
    M, N, K = 197 * 4, 768, 768
    x = rnd(M, K, seed=92).to(DEV)
    w = (rnd(N, K, seed=93) * 0.05).to(DEV)
    exact = x.double() @ w.double().t()
    x3, _ = ops.split_bf16x3(x, 0)
    w3, _ = ops.split_bf16x3(w, 1)
    y3 = ops.linear_fwd(x3, w3, None, torch.float32)
    y1 = ops.linear_fwd(x.to(BF), w.to(BF), None, torch.float32)
    e3 = ((y3.double() - exact).norm() / exact.norm()).item()
    e1 = ((y1.double() - exact).norm() / exact.norm()).item()
    assert e3 < 3e-5 and e1 > 20 * e3, (e3, e1)


@pytest.mark.parametrize("M,N,K", [(197 * 8, 3072, 3 * 768), (50, 256, 3 * 192), (197 * 2, 520, 3 * 64)])
def test_linear_fwd_gelu_split_x3(M, N, K):
    """VITMI_EPI_SPLIT_X3: the fc1 epilogue writes the GELU output as [hi | hi | lo] rows.  hi and
    gelu' are bit for bit the plain BIAS_GELU epilogue's (same accumulation, same GELU), and
    hi + lo carries gelu(u) to ~2^-16 (u = the fp32 GEMM output).  Shapes: gemm256 with the
    tail split (K' = 2304), the 128-tile kernel, ragged N."""
    x = rnd(M, K, seed=101).to(DEV).to(BF)
    w = (rnd(N, K, seed=102) * 0.05).to(DEV).to(BF)
    b = (rnd(N, seed=103) * 0.5).to(DEV)
    y3, g3 = ops.linear_fwd(x, w, b, BF, ops.EPI_BIAS_GELU, split_x3=True)
    y1, g1 = ops.linear_fwd(x, w, b, BF, ops.EPI_BIAS_GELU)
    assert y3.shape == (M, 3 * N)
    assert torch.equal(y3[:, :N], y1) and torch.equal(y3[:, N:2 * N], y1) and torch.equal(g3, g1)
    # with the tile-native gelu' (the model's form; the opaque buffer's padding rows are not
    # compared): the same split output
    y3t, _ = ops.linear_fwd(x, w, b, BF, ops.EPI_BIAS_GELU, aux_tiled=True, split_x3=True)
    assert torch.equal(y3t, y3)
    u = ops.linear_fwd(x, w, b, torch.float32).double()
    ref = torch.nn.functional.gelu(u)
    got = y3[:, :N].double() + y3[:, 2 * N:].double()
    assert ((got - ref).abs() <= ref.abs() * 2.0 ** -15 + 2e-6).all(), (got - ref).abs().max().item()


@pytest.mark.parametrize("M,D", [(197 * 3, 768), (37, 192), (5, 1024)])
def test_layernorm_fwd_writes_split_rows(M, D):
    """layernorm_fwd with out_dtype BF16X3 (VITMI_BF16X3): the [hi | hi | lo] rows of the fp32
    LayerNorm output, bit for bit what split_bf16x3 makes of the fp32 kernel's y; mean/rstd equal."""
    x = (rnd(M, D + 4, seed=95) * 2 + 0.5).to(DEV)[:, :D]
    w = (1 + 0.3 * rnd(D, seed=96)).to(DEV)
    b = (0.2 * rnd(D, seed=97)).to(DEV)
    y3, m3, r3 = ops.layernorm_fwd(x, w, b, 1e-6, ops.BF16X3)
    yf, mf, rf = ops.layernorm_fwd(x, w, b, 1e-6, torch.float32)
    ref, _ = ops.split_bf16x3(yf, 0)
    assert y3.shape == (M, 3 * D) and torch.equal(y3, ref)
    assert torch.equal(m3, mf) and torch.equal(r3, rf)


@pytest.mark.parametrize("B,N,H", [(3, 197, 12), (2, 17, 3), (1, 256, 2)])
def test_attention_fwd_x3_split_output(B, N, H):
    """vitmi_attention_fwd_x3: o and lse are the bf16 whole-sequence kernel's, bit for bit; o3 rows
    are [hi | hi | lo] with hi = o, and hi + lo tracks the softmax-attention of the same bf16 q, k, v
    (fp64) ~2^-9 relative (the kernel's bf16 P), where hi alone is 2^-9 rounding on top."""
    D = 64 * H
    qkv = (rnd(B * N, 3 * D, seed=98) * 0.7).to(DEV).to(BF)
    o, o3, lse = ops.attention_fwd_x3(qkv, B, N, H, 0.125)
    o_ref, lse_ref = ops.attention_fwd(qkv, B, N, H, 0.125)
    assert torch.equal(o, o_ref) and torch.equal(lse, lse_ref)
    assert torch.equal(o3[:, :D], o) and torch.equal(o3[:, D:2 * D], o)
    q, k, v = (t.double().view(B, N, H, 64).transpose(1, 2) for t in qkv.split(D, dim=1))
    ref = torch.softmax(q @ k.transpose(-1, -2) * 0.125, -1) @ v
    ref = ref.transpose(1, 2).reshape(B * N, D)
    full = o3[:, :D].double() + o3[:, 2 * D:].double()
    scale = ref.abs().max().item()
    e_full = (full - ref).abs().max().item() / scale
    e_hi = (o.double() - ref).abs().max().item() / scale
    assert e_full < 4e-3, (e_full, e_hi)
    # lo is the residual of the fp32 O below hi's rounding step
    assert (o3[:, 2 * D:].double().abs() <= o.double().abs() * 2.0 ** -8 + 1e-30).all()
