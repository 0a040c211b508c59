"""The bf16f8 precision knob's kernels (include/vitmi.h VITMI_BF16F8): rows [hi | e4m3 parts] with
hi = bf16(x), hi8 = e4m3(hi), lo8 = e4m3((x - hi) * 2^9), and the GEMM that takes them (hi.hi
in bf16, hi.lo + lo.hi as one block-scaled fp8 product).  References are built on the CPU with
torch's float8_e4m3fn (OCP, round-to-nearest-even) from the same fp32 values."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from vitmi import ops  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16
E4 = torch.float8_e4m3fn


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * scale


def e4m3(x):
    """fp32 -> e4m3 bytes (saturating at +-448 as the kernels do)."""
    return x.clamp(-448.0, 448.0).to(E4).view(torch.uint8)


def ref_parts(x):
    """(hi bf16, hi8 bytes, lo8 bytes) of fp32 x on the CPU."""
    x = x.float().cpu()
    hi = x.to(BF)
    return hi, e4m3(hi.float()), e4m3((x - hi.float()) * 512.0)


def parts(y8, K):
    """(hi bf16 [rows, K], first e4m3 part, second e4m3 part) of VITMI_BF16F8 rows [rows, 2K]; the
    e4m3 part is laid out in 64-k blocks [first | second] (common.h f8_off)."""
    rows = y8.shape[0]
    b = y8.contiguous().cpu().view(torch.uint8)[:, 2 * K:].reshape(rows, K // 64, 2, 64)
    return y8[:, :K].cpu(), b[:, :, 0].reshape(rows, K), b[:, :, 1].reshape(rows, K)


def deq(b):
    return b.view(E4).double()


@pytest.mark.parametrize("rows,K", [(197 * 3, 768), (37, 3072), (5, 64)])
def test_split_bf16f8_bytes(rows, K):
    """vitmi_split_bf16f8: hi, hi8 and lo8 bit for bit the CPU conversions, in the A ([hi|hi8|lo8]) and
    weight ([hi|lo8|hi8]) layouts, from a row-strided source; values spread over 2^-12 .. 2^10 so
    e4m3 subnormals and the +-448 saturation are both exercised."""
    g = torch.Generator().manual_seed(7)
    mag = torch.exp2(torch.randint(-12, 11, (rows, K + 8), generator=g).float())
    x = (rnd(rows, K + 8, seed=71) * mag).to(DEV)[:, 4:4 + K]
    x = x.contiguous() if (x.data_ptr() % 16) else x
    a8, hi = ops.split_bf16f8(x, 0, hi_copy=True)
    w8, none = ops.split_bf16f8(x, 1)
    assert none is None and a8.shape == (rows, 2 * K)
    h, h8, l8 = ref_parts(x)
    ah, a1, a2 = parts(a8, K)
    wh, w1, w2 = parts(w8, K)
    assert torch.equal(ah, h) and torch.equal(hi.cpu(), h) and torch.equal(wh, h)
    assert torch.equal(a1, h8) and torch.equal(a2, l8)
    assert torch.equal(w1, l8) and torch.equal(w2, h8)


@pytest.mark.parametrize("M,D", [(197 * 3, 768), (37, 192), (5, 1024)])
def test_layernorm_fwd_writes_f8_rows(M, D):
    """layernorm_fwd with out_dtype BF16F8: what split_bf16f8 makes of the fp32 kernel's y, bit for bit."""
    x = (rnd(M, D + 4, seed=95) * 2 + 0.5).to(DEV)[:, :D]
    w = (1 + 0.3 * rnd(D, seed=96)).to(DEV)
    b = (0.2 * rnd(D, seed=97)).to(DEV)
    y8, m8, r8 = ops.layernorm_fwd(x, w, b, 1e-6, ops.BF16F8)
    yf, mf, rf = ops.layernorm_fwd(x, w, b, 1e-6, torch.float32)
    ref, _ = ops.split_bf16f8(yf, 0)
    assert y8.shape == (M, 2 * D) and torch.equal(y8, ref)
    assert torch.equal(m8, mf) and torch.equal(r8, rf)


def _emulated(x, w):
    """The knob's product in fp64 from the CPU parts: hi.hi + (hi8.lo8 + lo8.hi8) / 2^9."""
    xh, x8h, x8l = ref_parts(x)
    wh, w8h, w8l = ref_parts(w)
    return (xh.double() @ wh.double().t()
            + (deq(x8h) @ deq(w8l).t() + deq(x8l) @ deq(w8h).t()) / 512.0)


@pytest.mark.parametrize("M,N,K", [(300, 320, 192), (197 * 4, 768, 768), (25600, 768, 704)])
def test_bf16f8_gemm(M, N, K):
    """One GEMM over the VITMI_BF16F8 rows: K/64 bf16 K-steps, then K/64 block-scaled e4m3 K-steps.
    Against the same product emulated in fp64 from the CPU parts (fp32-accumulation close), and
    against the exact fp64 product (the knob's residual error, far below the plain bf16 GEMM's).
    (300, 320, 192): ragged M, the bf16 / fp8 switch inside a unit; (25600, 768, 704): the tail
    split, one of whose K-ranges straddles the switch."""
    x = rnd(M, K, seed=92).to(DEV)
    w = (rnd(N, K, seed=93) * 0.05).to(DEV)
    b = (rnd(N, seed=94) * 0.1).to(DEV)
    x8, _ = ops.split_bf16f8(x, 0)
    w8, _ = ops.split_bf16f8(w, 1)
    y = ops.linear_fwd(x8, w8, b, torch.float32, f8=True).double().cpu()
    emu = _emulated(x, w) + b.double().cpu()
    exact = x.double().cpu() @ w.double().cpu().t() + b.double().cpu()
    y1 = ops.linear_fwd(x.to(BF), w.to(BF), b, torch.float32).double().cpu()
    scale = exact.norm()
    e_emu = ((y - emu).norm() / scale).item()
    e_exact = ((y - exact).norm() / scale).item()
    e_bf16 = ((y1 - exact).norm() / scale).item()
    print(f"bf16f8 GEMM {M}x{N}x{K}: vs emulation {e_emu:.2e}, vs exact {e_exact:.2e}, plain bf16 {e_bf16:.2e}")
    assert e_emu < 1e-5, e_emu
    assert e_exact < 1.5e-4 and e_bf16 > 10 * e_exact, (e_exact, e_bf16)


def test_bf16f8_gemm_residual_and_bf16_out():
    """The knob's other epilogues on VITMI_BF16F8 operands: the fp32 residual one (proj / fc2) and
    the bf16 store (qkv): each equals the fp32 store plus the residual / rounded to bf16."""
    M, N, K = 197 * 2, 768, 768
    x = rnd(M, K, seed=41).to(DEV)
    w = (rnd(N, K, seed=42) * 0.05).to(DEV)
    b = (rnd(N, seed=43) * 0.1).to(DEV)
    res = rnd(M, N, seed=44).to(DEV)
    x8, _ = ops.split_bf16f8(x, 0)
    w8, _ = ops.split_bf16f8(w, 1)
    y = ops.linear_fwd(x8, w8, b, torch.float32, f8=True)
    yr = ops.linear_fwd(x8, w8, b, torch.float32, ops.EPI_RESIDUAL, residual=res, f8=True)
    yb = ops.linear_fwd(x8, w8, b, BF, f8=True)
    assert torch.allclose(yr, res + y, rtol=0, atol=1e-5)
    assert torch.equal(yb, y.to(BF))


def parts_w(y8, K):
    """(hi bf16 [rows, K], e4m3 bytes [rows, K]) of VITMI_BF16F8W rows [rows, 1.5K] (one byte per k)."""
    b = y8.contiguous().cpu().view(torch.uint8)[:, 2 * K:]
    return y8[:, :K].cpu(), b


@pytest.mark.parametrize("rows,K", [(197 * 3, 768), (37, 3072), (5, 128)])
def test_split_bf16f8w_bytes(rows, K):
    """vitmi_split_bf16f8 patterns 2 / 3 (VITMI_BF16F8W): [hi | hi8] and [hi | lo8], bit for bit the CPU
    conversions, from a row-strided source with values over 2^-12 .. 2^10; and the mixed weight
    splitter (one launch, a pattern per weight) gives the same rows as the single-tensor calls."""
    g = torch.Generator().manual_seed(17)
    mag = torch.exp2(torch.randint(-12, 11, (rows, K + 8), generator=g).float())
    x = (rnd(rows, K + 8, seed=171) * mag).to(DEV)[:, 4:4 + K]
    x = x.contiguous() if (x.data_ptr() % 16) else x
    a8, hi = ops.split_bf16f8(x, 2, hi_copy=True)
    w8, _ = ops.split_bf16f8(x, 3)
    assert a8.shape == (rows, K + K // 2) and w8.shape == (rows, K + K // 2)
    h, h8, l8 = ref_parts(x)
    ah, a1 = parts_w(a8, K)
    wh, w1 = parts_w(w8, K)
    assert torch.equal(ah, h) and torch.equal(hi.cpu(), h) and torch.equal(wh, h)
    assert torch.equal(a1, h8) and torch.equal(w1, l8)
    xc = x.contiguous()
    w_mix = ops.split_bf16f8_weights([xc, xc], [3, 1])
    assert torch.equal(w_mix[0], w8) and torch.equal(w_mix[1], ops.split_bf16f8(xc, 1)[0])


@pytest.mark.parametrize("M,D", [(197 * 3, 768), (37, 256), (5, 1024)])
def test_layernorm_fwd_writes_f8w_rows(M, D):
    """layernorm_fwd with out_dtype BF16F8W: what split_bf16f8(.., 2) makes of the fp32 kernel's y."""
    x = (rnd(M, D + 4, seed=195) * 2 + 0.5).to(DEV)[:, :D]
    w = (1 + 0.3 * rnd(D, seed=196)).to(DEV)
    b = (0.2 * rnd(D, seed=197)).to(DEV)
    y8, m8, r8 = ops.layernorm_fwd(x, w, b, 1e-6, ops.BF16F8W)
    yf, mf, rf = ops.layernorm_fwd(x, w, b, 1e-6, torch.float32)
    ref, _ = ops.split_bf16f8(yf, 2)
    assert y8.shape == (M, D + D // 2) and torch.equal(y8, ref)
    assert torch.equal(m8, mf) and torch.equal(r8, rf)


@pytest.mark.parametrize("M,N,K", [(300, 320, 256), (197 * 4, 2304, 768), (25600, 768, 768)])
def test_bf16f8w_gemm(M, N, K):
    """The weight-side form (VITMI_BF16F8W, the knob's qkv GEMM): K/64 bf16 K-steps, then K/128 e4m3
    K-steps of hi8(x) . lo8(w) / 2^9.  Against that product emulated in fp64 from the CPU parts, and
    against the exact product: it removes the weight rounding's share of the plain bf16 GEMM's
    error (x's rounding stays).  (300, 320, 256): ragged M with the switch inside a unit; (25600,
    768, 768): the tail split."""
    x = rnd(M, K, seed=292).to(DEV)
    w = (rnd(N, K, seed=293) * 0.05).to(DEV)
    b = (rnd(N, seed=294) * 0.1).to(DEV)
    x8, _ = ops.split_bf16f8(x, 2)
    w8, _ = ops.split_bf16f8(w, 3)
    y = ops.linear_fwd(x8, w8, b, torch.float32, f8="w").double().cpu()
    xh, x8h, _ = ref_parts(x)
    wh, _, w8l = ref_parts(w)
    emu = xh.double() @ wh.double().t() + (deq(x8h) @ deq(w8l).t()) / 512.0 + b.double().cpu()
    xb = xh.double()
    half = xb @ w.double().cpu().t() + b.double().cpu()       # x rounded, w exact
    scale = half.norm()
    e_emu = ((y - emu).norm() / scale).item()
    e_half = ((y - half).norm() / scale).item()
    y1 = ops.linear_fwd(x.to(BF), w.to(BF), b, torch.float32).double().cpu()
    e_plain = ((y1 - half).norm() / scale).item()
    print(f"bf16f8w GEMM {M}x{N}x{K}: vs emulation {e_emu:.2e}, vs (bf16 x) . (fp32 w) {e_half:.2e}, plain {e_plain:.2e}")
    assert e_emu < 1e-5, e_emu
    assert e_half < 2e-4 and e_plain > 5 * e_half, (e_half, e_plain)
    yb = ops.linear_fwd(x8, w8, b, BF, f8="w")
    assert torch.equal(yb.cpu(), y.float().to(BF))


@pytest.mark.parametrize("M,N,K", [(197 * 8, 3072, 768), (50, 256, 192)])
def test_linear_fwd_gelu_split_f8(M, N, K):
    """VITMI_EPI_SPLIT_F8: the fc1 epilogue writes gelu(u) as VITMI_BF16F8 A-operand rows.  hi8 is
    e4m3(hi) exactly; hi + lo8 / 2^9 carries gelu(u) (u from the fp32 store of the same GEMM) to
    ~2^-13; gelu' (bf16) against torch's exact derivative."""
    x = rnd(M, K, seed=101).to(DEV)
    w = (rnd(N, K, seed=102) * 0.05).to(DEV)
    b = (rnd(N, seed=103) * 0.5).to(DEV)
    x8, _ = ops.split_bf16f8(x, 0)
    w8, _ = ops.split_bf16f8(w, 1)
    y8, gp = ops.linear_fwd(x8, w8, b, BF, ops.EPI_BIAS_GELU, split_f8=True, f8=True)
    assert y8.shape == (M, 2 * N)
    u = ops.linear_fwd(x8, w8, b, torch.float32, f8=True).double().cpu()
    hi, p1, p2 = parts(y8, N)
    assert torch.equal(p1, e4m3(hi.float()))
    ref = torch.nn.functional.gelu(u)
    got = hi.double() + deq(p2) / 512.0
    assert ((got - ref).abs() <= ref.abs() * 2.0 ** -12 + 2e-6).all(), (got - ref).abs().max().item()
    # gelu'(u) = Phi(u) + u phi(u), bf16
    dref = 0.5 * (1 + torch.erf(u / 2 ** 0.5)) + u * torch.exp(-0.5 * u * u) / (2 * torch.pi) ** 0.5
    assert ((gp.double().cpu() - dref).abs() <= dref.abs() * 2.0 ** -7 + 1e-3).all()
    # the tile-native gelu' (the model's form): the same activation rows
    y8t, _ = ops.linear_fwd(x8, w8, b, BF, ops.EPI_BIAS_GELU, aux_tiled=True, split_f8=True, f8=True)
    assert torch.equal(y8t, y8)


@pytest.mark.parametrize("B,N,H", [(3, 197, 12), (2, 17, 3), (1, 256, 2)])
def test_attention_fwd_f8_output(B, N, H):
    """vitmi_attention_fwd_f8: o and lse are the bf16 whole-sequence kernel's, bit for bit; o8's hi
    is o, its hi8 = e4m3(o), and hi + lo8 / 2^9 equals the x3 kernel's hi + lo (the same fp32 O)
    to lo8's e4m3 precision."""
    D = 64 * H
    qkv = (rnd(B * N, 3 * D, seed=98) * 0.7).to(DEV).to(BF)
    o, o8, lse = ops.attention_fwd_f8(qkv, B, N, H, 0.125)
    o_ref, lse_ref = ops.attention_fwd(qkv, B, N, H, 0.125)
    assert torch.equal(o, o_ref) and torch.equal(lse, lse_ref)
    hi, p1, p2 = parts(o8, D)
    assert torch.equal(hi, o.cpu()) and torch.equal(p1, e4m3(o.float().cpu()))
    _, o3, _ = ops.attention_fwd_x3(qkv, B, N, H, 0.125)
    lo3 = o3[:, 2 * D:].double().cpu()
    lo8 = deq(p2) / 512.0
    # (lo8 / 2^9 resolves 2^-18 at the bottom of e4m3's subnormal range)
    assert ((lo8 - lo3).abs() <= lo3.abs() * 2.0 ** -3 + o.double().cpu().abs() * 2.0 ** -16 + 2.0 ** -18).all()


def test_split_bf16f8_weights_batch_matches_single():
    """vitmi_split_bf16f8_weights (one launch for a block's four weights) writes what
    split_bf16f8(w, 1) writes for each, bit for bit."""
    shapes = [(2304, 768), (768, 768), (3072, 768), (768, 3072)]
    ws = [(rnd(*s, seed=60 + i) * 0.05).to(DEV) for i, s in enumerate(shapes)]
    outs = ops.split_bf16f8_weights(ws)
    for w, o in zip(ws, outs):
        ref, _ = ops.split_bf16f8(w, 1)
        assert o.shape == ref.shape and torch.equal(o, ref)


@pytest.mark.parametrize("amp,bound", [(200.0, "knob"), (2000.0, "bf16")])
def test_bf16f8_gemm_large_magnitudes(amp, bound):
    """the fixed e4m3 scales bound where the corrections hold (csrc/common.h).  With
    activations of |x| up to ~200 (lo8 = lo * 2^9 <= 2|x| stays under e4m3's 448) the product keeps
    the knob's accuracy, >= 10x better than plain bf16; at |x| ~ 2000 hi8 and lo8 saturate and the
    product only keeps roughly plain-bf16 accuracy (no worse than 2x the bf16 GEMM's error)."""
    M, N, K = 197 * 2, 768, 768
    x = (rnd(M, K, seed=131).clamp(-3, 3) * (amp / 3)).to(DEV)
    w = (rnd(N, K, seed=132) * 0.05).to(DEV)
    x8, _ = ops.split_bf16f8(x, 0)
    w8, _ = ops.split_bf16f8(w, 1)
    y = ops.linear_fwd(x8, w8, None, torch.float32, f8=True).double().cpu()
    exact = x.double().cpu() @ w.double().cpu().t()
    y1 = ops.linear_fwd(x.to(BF), w.to(BF), None, torch.float32).double().cpu()
    scale = exact.norm()
    e8 = ((y - exact).norm() / scale).item()
    e16 = ((y1 - exact).norm() / scale).item()
    print(f"bf16f8 GEMM |x| <= {amp:g}: rel err {e8:.2e}, plain bf16 {e16:.2e}")
    if bound == "knob":
        assert e8 < 1.5e-4 and e16 > 10 * e8, (e8, e16)
    else:
        assert e8 < 2 * e16, (e8, e16)
