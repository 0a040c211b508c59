// tools/proto/ln_variants.hip — LayerNorm variants measured slower in round 3 and removed
// from libvitmi.so ('Measured and not kept'): the residual add fused into the
// forward (VITMI_RES_IN_LN), the transposed bf16 copies for token-contiguous weight-gradient
// operands (VITMI_WGRAD_T), and the software-pipelined backward rows (VITMI_LN_BWD_PIPE).
// Kept as source for reference only; not compiled by any build.

// ---- VITMI_LN_BWD_PIPE: the row loop of ln_bwd_kernel with the next row's loads in flight
#if VITMI_LN_BWD_PIPE
  // software-pipelined rows: the wave's next row (x, dy, the residual gradient, its statistics)
  // is loaded before this row is reduced, so two rows' loads are in flight per wave
  const int64_t rstep = (int64_t)gridDim.x * 4;
  f32x4 cx[NV], cd[NV], cr[NV];
  float cmu = 0.f, crs = 0.f;
  auto load_row = [&](int64_t r, f32x4 (&lx)[NV], f32x4 (&ld)[NV], f32x4 (&lr)[NV], float& lmu, float& lrs) {
    lmu = mean[r];
    lrs = rstd[r];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (lane + 64 * i) * 4;
      const bool ok = c < D;
      lr[i] = (dres && ok) ? *(const f32x4*)(dres + r * ldres + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      lx[i] = ok ? *(const f32x4*)(x + r * ldx + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      ld[i] = ok ? load4<TDY>(dy + r * lddy + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  int64_t row = (int64_t)blockIdx.x * 4 + wave;
  if (row < M) load_row(row, cx, cd, cr, cmu, crs);
  for (; row < M; row += rstep) {
    const int64_t nrow = row + rstep;
    f32x4 nx[NV], nd[NV], nr[NV];
    float nmu = 0.f, nrs = 0.f;
    if (nrow < M) load_row(nrow, nx, nd, nr, nmu, nrs);
    const float mu = cmu, rs = crs;
    f32x4 xh[NV], gy[NV];
    f32x4* rv = cr;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (lane + 64 * i) * 4;
      if (c < D) {
        const f32x4 xv = cx[i];
        const f32x4 dyv = cd[i];
#else
  ... (row math as ln_bwd_kernel) ...
#if VITMI_LN_BWD_PIPE
    if (nrow < M) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        cx[i] = nx[i];
        cd[i] = nd[i];
        cr[i] = nr[i];
      }
      cmu = nmu;
      crs = nrs;
    }
#endif

// ------------------------------------------------ residual add fused into the forward
// xo = x + y (fp32 residual stream + the bf16 branch output), then LayerNorm of xo: the
// out-projection GEMM of the block then stores its output as bf16 (a plain-store epilogue)
// instead of loading and storing the fp32 residual tile in its epilogue, where those loads and
// stores sit serialised after the K-loop (K = 768: about half that GEMM's time).
template <int NV, typename TY>
__global__ __launch_bounds__(256) void ln_fwd_res_kernel(int64_t M, int D, const float* __restrict__ x, int64_t ldx,
                                                         const bf16* __restrict__ yb, int64_t ldyb,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float eps,
                                                         float* __restrict__ xo, int64_t ldxo,
                                                         TY* __restrict__ y, int64_t ldy,
                                                         float* __restrict__ mean, float* __restrict__ rstd) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float* xr = x + row * ldx;
  f32x4 v[NV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (lane + 64 * i) * 4;
    v[i] = c < D ? *(const f32x4*)(xr + c) + load4<bf16>(yb + row * ldyb + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (lane + 64 * i) * 4;
    if (c < D) *(f32x4*)(xo + row * ldxo + c) = v[i];   // default policy: LN backward re-reads it
  }
  const float mu = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (lane + 64 * i) * 4;
    if (c < D) {
      const f32x4 d = v[i] - mu;
      q += d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3];
    }
  }
  const float rs = rsqrtf(wave_sum(q) / D + eps);
  TY* yr = y + row * ldy;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (lane + 64 * i) * 4;
    if (c < D) {
      const f32x4 g = *(const f32x4*)(gamma + c);
      const f32x4 b = *(const f32x4*)(beta + c);
      store4<TY>(yr + c, (v[i] - mu) * rs * g + b);
    }
  }
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

// ------------------------------------------------ transposed bf16 copies (weight-gradient operands)
// The weight-gradient GEMMs reduce over tokens; with both operands token-major (TN) every
// fragment is a transposed LDS read, and the A side's reads bound the loop (tools/wgrad_layout.py:
// with A given token-contiguous the ViT-B wgrads run 15 % faster, with both 23 %).  These
// variants also write the bf16 output transposed, yT[col][row] (row stride ldt >= M), from a
// 32-row tile staged in LDS: each lane stores 16 B = 8 tokens of one column, 4 lanes one
// column's 64 B.  Tile image pitch D + 4 bf16: the 8-token column reads of a wave (16 columns x
// 4 row groups) fall on distinct banks.
constexpr int TT_ROWS = 32;

// Blocks are dealt to the 8 XCDs round-robin; the tiles are remapped so that every XCD walks a
// contiguous range: the two 64-B halves of a transposed output line (tiles t and t^1) are then
// written through the same L2 instead of two XCDs' L2s each writing back a half-dirty line.
__device__ __forceinline__ int64_t xcd_tile(int64_t b, int64_t nb) {
  const int64_t x = b & 7, q = nb >> 3, r = nb & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

template <int NV>
__device__ __forceinline__ void tile_transpose_store(const bf16* tile, int pitch, int D, int64_t m0, int64_t M,
                                                     bf16* __restrict__ yt, int64_t ldt) {
#ifdef VITMI_LNT_NOTR
  return;   // DIAGNOSTIC build: the row phase alone
#endif
  for (int item = threadIdx.x; item < 4 * D; item += blockDim.x) {
    const int q = item & 3, c = item >> 2;
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = tile[(8 * q + j) * pitch + c];
    const int64_t m = m0 + 8 * q;
    bf16* dst = yt + (int64_t)c * ldt + m;
    if (m + 8 <= M) {
      if constexpr (VITMI_NT_LN) __builtin_nontemporal_store(v, (bf16x8*)dst);
      else *(bf16x8*)dst = v;
    } else {
      for (int j = 0; j < 8 && m + j < M; ++j) dst[j] = v[j];
    }
  }
}

// forward: 8 waves x 4 rows of a 32-row tile; y (row-major bf16) + yT + mean/rstd
template <int NV>
__global__ __launch_bounds__(512) void ln_fwd_t_kernel(int64_t M, int D, const float* __restrict__ x, int64_t ldx,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       float eps, bf16* __restrict__ y, int64_t ldy,
                                                       bf16* __restrict__ yt, int64_t ldt, float* __restrict__ mean,
                                                       float* __restrict__ rstd) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  bf16* tile = (bf16*)lds_raw;
  const int pitch = D + 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t m0 = xcd_tile(blockIdx.x, gridDim.x) * TT_ROWS;
  // the wave's 4 rows are loaded before any is reduced (4 x NV loads in flight)
  f32x4 vv[4][NV];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int64_t row = m0 + wave * 4 + rr;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (lane + 64 * i) * 4;
      vv[rr][i] = (row < M && c < D) ? *(const f32x4*)(x + row * ldx + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int r = wave * 4 + rr;
    const int64_t row = m0 + r;
    bf16* trow = tile + r * pitch;
    if (row >= M) {   // rows past M: zeros in the image (their yT columns are not stored)
      for (int c = lane * 4; c < D; c += 256) *(bf16x4*)(trow + c) = bf16x4{};
      continue;
    }
    f32x4* v = vv[rr];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
    const float mu = wave_sum(s) / D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (lane + 64 * i) * 4;
      if (c < D) {
        const f32x4 d = v[i] - mu;
        q += d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3];
      }
    }
    const float rs = rsqrtf(wave_sum(q) / D + eps);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (lane + 64 * i) * 4;
      if (c < D) {
        const f32x4 g = *(const f32x4*)(gamma + c);
        const f32x4 b = *(const f32x4*)(beta + c);
        const f32x4 o = (v[i] - mu) * rs * g + b;
        bf16x4 ob;
        ob[0] = (bf16)o[0]; ob[1] = (bf16)o[1]; ob[2] = (bf16)o[2]; ob[3] = (bf16)o[3];
        put((bf16x4*)(y + row * ldy + c), ob);
        *(bf16x4*)(trow + c) = ob;
      }
    }
    if (lane == 0) {
      mean[row] = mu;
      rstd[row] = rs;
    }
  }
  __syncthreads();
  tile_transpose_store<NV>(tile, pitch, D, m0, M, yt, ldt);
}

// backward with the bf16 copy of dx also written transposed: blocks walk 32-row tiles
// (8 waves x 4 rows); otherwise ln_bwd_kernel's math and per-block parameter partials
template <int NV, typename TDY>
__global__ __launch_bounds__(512) void ln_bwd_t_kernel(
    int64_t M, int D, const TDY* __restrict__ dy, int64_t lddy, const float* __restrict__ x, int64_t ldx,
    const float* __restrict__ mean, const float* __restrict__ rstd, const float* __restrict__ gamma,
    const float* __restrict__ dres, int64_t ldres, float* __restrict__ dx, int64_t lddx, bf16* __restrict__ dx_lp,
    int64_t lddx_lp, bf16* __restrict__ dxt, int64_t ldt, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  bf16* tile = (bf16*)lds_raw;
  const int pitch = D + 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  f32x4 g[NV], dg[NV], db[NV], ds[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (lane + 64 * i) * 4;
    g[i] = c < D ? *(const f32x4*)(gamma + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    dg[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    db[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    ds[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // each XCD's blocks walk one contiguous range of tiles (see xcd_tile), in turn
  const int64_t ntile = (M + TT_ROWS - 1) / TT_ROWS;
  const int64_t G = gridDim.x, x8 = blockIdx.x & 7, gq = G >> 3, gr = G & 7;
  const int64_t nbx = gq + (x8 < gr ? 1 : 0), jx = blockIdx.x >> 3;   // blocks of this XCD group
  const int64_t tq = ntile >> 3, trm = ntile & 7;
  const int64_t t0 = x8 < trm ? x8 * (tq + 1) : trm * (tq + 1) + (x8 - trm) * tq;
  const int64_t t1 = t0 + tq + (x8 < trm ? 1 : 0);
  for (int64_t t = t0 + jx; t < t1; t += nbx) {
    const int64_t m0 = t * TT_ROWS;
#pragma unroll 1
    for (int rr = 0; rr < 4; ++rr) {
      const int r = wave * 4 + rr;
      const int64_t row = m0 + r;
      bf16* trow = tile + r * pitch;
      if (row >= M) {
        for (int c = lane * 4; c < D; c += 256) *(bf16x4*)(trow + c) = bf16x4{};
        continue;
      }
      const float mu = mean[row], rs = rstd[row];
      f32x4 xh[NV], gy[NV], rv[NV];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = (lane + 64 * i) * 4;
        rv[i] = (dres && c < D) ? *(const f32x4*)(dres + row * ldres + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = (lane + 64 * i) * 4;
        if (c < D) {
          const f32x4 xv = *(const f32x4*)(x + row * ldx + c);
          const f32x4 dyv = load4<TDY>(dy + row * lddy + c);
          xh[i] = (xv - mu) * rs;
          gy[i] = dyv * g[i];
          dg[i] += dyv * xh[i];
          db[i] += dyv;
          s1 += gy[i][0] + gy[i][1] + gy[i][2] + gy[i][3];
          const f32x4 tt = gy[i] * xh[i];
          s2 += tt[0] + tt[1] + tt[2] + tt[3];
        } else {
          xh[i] = f32x4{0.f, 0.f, 0.f, 0.f};
          gy[i] = xh[i];
        }
      }
      const float c1 = wave_sum(s1) / D, c2 = wave_sum(s2) / D;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = (lane + 64 * i) * 4;
        if (c < D) {
          const f32x4 o = (gy[i] - c1 - xh[i] * c2) * rs + rv[i];
          ds[i] += o;
          put((f32x4*)(dx + row * lddx + c), o);
          bf16x4 ob;
          ob[0] = (bf16)o[0]; ob[1] = (bf16)o[1]; ob[2] = (bf16)o[2]; ob[3] = (bf16)o[3];
          put((bf16x4*)(dx_lp + row * lddx_lp + c), ob);
          *(bf16x4*)(trow + c) = ob;
        }
      }
    }
    __syncthreads();
    tile_transpose_store<NV>(tile, pitch, D, m0, M, dxt, ldt);
    __syncthreads();   // the image is rewritten by the next tile
  }
  // block-reduce dgamma / dbeta / colsum(dx) over the 8 waves, one array at a time through the
  // (now free) tile image: 8 x 64 x NV f32x4 <= 8 * 64 * 3 * 16 = 24 KiB
  f32x4* red = (f32x4*)lds_raw;
#pragma unroll 1
  for (int which = 0; which < 3; ++which) {
#pragma unroll
    for (int i = 0; i < NV; ++i) red[(wave * NV + i) * 64 + lane] = which == 0 ? dg[i] : which == 1 ? db[i] : ds[i];
    __syncthreads();
    for (int e = threadIdx.x; e < NV * 64; e += blockDim.x) {
      f32x4 a = red[e];
      for (int w = 1; w < 8; ++w) a += red[w * NV * 64 + e];
      const int i = e / 64, l = e % 64;
      const int c = (l + 64 * i) * 4;
      if (c < D) *(f32x4*)(part + ((int64_t)which * gridDim.x + blockIdx.x) * D + c) = a;
    }
    __syncthreads();
  }
}

extern "C" int vitmi_layernorm_fwd_t(int64_t M, int D, const float* x, int64_t ldx, const float* gamma,
                                     const float* beta, float eps, void* y, int64_t ldy, void* yt, int64_t ldt,
                                     float* mean, float* rstd, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(D > 0 && D % 4 == 0 && D <= 1024, "layernorm_fwd_t: D must be a multiple of 4 in [4, 1024]");
  VITMI_CHECK_ARG(ldx % 4 == 0 && ldy % 4 == 0, "layernorm_fwd_t: strides must be multiples of 4");
  VITMI_CHECK_ARG(ldt >= M && ldt % 8 == 0, "layernorm_fwd_t: ldt must be >= M and a multiple of 8");
  if (M == 0) return VITMI_OK;
  VITMI_CHECK_ARG(x && gamma && beta && y && yt && mean && rstd, "layernorm_fwd_t: null pointer");
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)((M + TT_ROWS - 1) / TT_ROWS));
  const size_t lds = (size_t)TT_ROWS * (D + 4) * 2;
  const int nv = (D + 255) / 256;
#define LNFT(NV)                                                                                  \
  hipLaunchKernelGGL((ln_fwd_t_kernel<NV>), grid, dim3(512), lds, s, M, D, x, ldx, gamma, beta, eps, \
                     (bf16*)y, ldy, (bf16*)yt, ldt, mean, rstd);                                   \
  VITMI_STAT((ln_fwd_t_kernel<NV>), 0, (double)M * D * (4 + 2 + 2) + 8.0 * M);
  switch (nv) {
    case 1: LNFT(1) break;
    case 2: LNFT(2) break;
    case 3: LNFT(3) break;
    default: LNFT(4) break;
  }
#undef LNFT
  VITMI_LAUNCH_CHECK("layernorm_fwd_t");
  return VITMI_OK;
}

extern "C" int vitmi_layernorm_bwd_t(int64_t M, int D, const void* dy, int dy_dtype, int64_t lddy,
                                     const float* x, int64_t ldx, const float* mean, const float* rstd,
                                     const float* gamma, const float* dres, int64_t ldres, float* dx,
                                     int64_t lddx, void* dx_lp, int64_t lddx_lp, void* dxt, int64_t ldt,
                                     float* dgamma, float* dbeta, float* dxsum, void* workspace,
                                     size_t ws_bytes, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(D > 0 && D % 4 == 0 && D <= 1024, "layernorm_bwd_t: D must be a multiple of 4 in [4, 1024]");
  VITMI_CHECK_ARG(ldt >= M && ldt % 8 == 0, "layernorm_bwd_t: ldt must be >= M and a multiple of 8");
  if (M == 0) return VITMI_OK;
  VITMI_CHECK_ARG(dy && x && mean && rstd && gamma && dx && dx_lp && dxt, "layernorm_bwd_t: null pointer");
  VITMI_CHECK_ARG(workspace && ws_bytes >= vitmi_layernorm_bwd_workspace_size(M, D),
                  "layernorm_bwd_t: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int G = ln_blocks_bwd(M);
  float* part = (float*)workspace;
  const int nv = (D + 255) / 256;
  // the tile image, reused after the loop for the 8-wave parameter-partial fold
  const size_t lds = std::max((size_t)TT_ROWS * (D + 4) * 2, (size_t)8 * (nv > 3 ? 4 : nv) * 64 * 16);
  const double b = (double)M * D * ((dy_dtype == VITMI_BF16 ? 2 : 4) + 4 + (dres ? 4 : 0) + 4 + 2 + 2) + 8.0 * M;
#define LNBT(NV, TDY)                                                                              \
  hipLaunchKernelGGL((ln_bwd_t_kernel<NV, TDY>), dim3(G), dim3(512), lds, s, M, D, (const TDY*)dy, lddy, x, ldx, \
                     mean, rstd, gamma, dres, ldres, dx, lddx, (bf16*)dx_lp, lddx_lp, (bf16*)dxt, ldt, part); \
  VITMI_STAT((ln_bwd_t_kernel<NV, TDY>), 0, b);
#define LNBT2(NV) if (dy_dtype == VITMI_BF16) { LNBT(NV, bf16) } else { LNBT(NV, float) }
  switch (nv) {
    case 1: LNBT2(1) break;
    case 2: LNBT2(2) break;
    case 3: LNBT2(3) break;
    default: LNBT2(4) break;
  }
#undef LNBT2
#undef LNBT
  hipLaunchKernelGGL(ln_param_reduce, dim3((D + 15) / 16), dim3(1024), 0, s, (const float*)part, G, D, dgamma,
                     dbeta, dxsum);
  VITMI_LAUNCH_CHECK("layernorm_bwd_t");
  return VITMI_OK;
}

extern "C" int vitmi_layernorm_fwd_res(int64_t M, int D, const float* x, int64_t ldx, const void* yb,
                                       int64_t ldyb, const float* gamma, const float* beta, float eps,
                                       float* xo, int64_t ldxo, void* y, int y_dtype, int64_t ldy, float* mean,
                                       float* rstd, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(D > 0 && D % 4 == 0 && D <= 2048, "layernorm_fwd_res: D must be a multiple of 4 in [4, 2048]");
  VITMI_CHECK_ARG(ldx % 4 == 0 && ldyb % 4 == 0 && ldxo % 4 == 0 && ldy % 4 == 0,
                  "layernorm_fwd_res: strides must be multiples of 4");
  if (M == 0) return VITMI_OK;
  VITMI_CHECK_ARG(x && yb && gamma && beta && xo && y && mean && rstd, "layernorm_fwd_res: null pointer");
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)((M + 3) / 4));
  const int nv = (D + 255) / 256;
  const double by = (double)M * D * (4 + 2 + 4 + (y_dtype == VITMI_BF16 ? 2 : 4)) + 8.0 * M;
#define LNFR(NV)                                                                                  \
  if (y_dtype == VITMI_BF16) {                                                                    \
    hipLaunchKernelGGL((ln_fwd_res_kernel<NV, bf16>), grid, dim3(256), 0, s, M, D, x, ldx, (const bf16*)yb, ldyb, \
                       gamma, beta, eps, xo, ldxo, (bf16*)y, ldy, mean, rstd);                    \
    VITMI_STAT((ln_fwd_res_kernel<NV, bf16>), 0, by);                                             \
  } else {                                                                                        \
    hipLaunchKernelGGL((ln_fwd_res_kernel<NV, float>), grid, dim3(256), 0, s, M, D, x, ldx, (const bf16*)yb, ldyb, \
                       gamma, beta, eps, xo, ldxo, (float*)y, ldy, mean, rstd);                   \
    VITMI_STAT((ln_fwd_res_kernel<NV, float>), 0, by);                                            \
  }
  switch (nv) {
    case 1: LNFR(1) break;
    case 2: LNFR(2) break;
    case 3: LNFR(3) break;
    case 4: LNFR(4) break;
    default: LNFR(8) break;
  }
#undef LNFR
  VITMI_LAUNCH_CHECK("layernorm_fwd_res");
  return VITMI_OK;
}

// ---- VITMI_ADAM_V2 (optim.hip): two float4 groups per lane, non-temporal stores
// streaming form (A/B builds): two float4 groups per thread and iteration (8 loads in flight per
// lane) and non-temporal stores (p, m, v are next read by the next step's Adam; the bf16 shadow
// by the next forward's GEMMs, from the MALL at best)
#ifndef VITMI_ADAM_V2
#define VITMI_ADAM_V2 0
#endif
template <typename V>
__device__ __forceinline__ void st_stream(V* p, V v) {
  if constexpr (VITMI_ADAM_V2) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <bool LP>
__device__ __forceinline__ void adam4(const AdamArgs& a, int64_t i, float* __restrict__ p, const float* __restrict__ g,
                                      float* __restrict__ m, float* __restrict__ v, bf16* __restrict__ lp,
                                      f32x4 pv, f32x4 gv, f32x4 mv, f32x4 vv) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float pe = pv[e], me = mv[e], ve = vv[e];
    adam1(a, pe, gv[e], me, ve);
    pv[e] = pe;
    mv[e] = me;
    vv[e] = ve;
  }
  st_stream((f32x4*)p + i, pv);
  st_stream((f32x4*)m + i, mv);
  st_stream((f32x4*)v + i, vv);
  if constexpr (LP) {
    bf16x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = from_f32<bf16>(pv[e]);
    st_stream((bf16x4*)lp + i, o);
  }
}

#if VITMI_ADAM_V2
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + stride < n4; i += 2 * stride) {
    const f32x4 p0 = ((const f32x4*)p)[i], g0 = ((const f32x4*)g)[i], m0 = ((const f32x4*)m)[i], v0 = ((const f32x4*)v)[i];
    const int64_t j = i + stride;
    const f32x4 p1 = ((const f32x4*)p)[j], g1 = ((const f32x4*)g)[j], m1 = ((const f32x4*)m)[j], v1 = ((const f32x4*)v)[j];
    adam4<LP>(a, i, p, g, m, v, lp, p0, g0, m0, v0);
    adam4<LP>(a, j, p, g, m, v, lp, p1, g1, m1, v1);
  }
  if (i < n4) adam4<LP>(a, i, p, g, m, v, lp, ((const f32x4*)p)[i], ((const f32x4*)g)[i], ((const f32x4*)m)[i], ((const f32x4*)v)[i]);
#else

// ---- attention.hip: the two-key-blocks-per-wave dK/dV kernel (old policy 3) and the single-pass
// fused backward (old policy 2), both measured slower end to end
// Column sums of two consecutive 32-row tiles (rows row0.., row0+32..) that store_tile32 just wrote
// into the images s0 and s1, folded over the workgroup's waves in wave order into colpart[0..63]
// (tile32_colsum for a wave that owns 64 rows; fixed summation order).
__device__ __forceinline__ void tile32x2_colsum(const char* s0, const char* s1, int row0, int nvalid, float* colpart,
                                                float (*red)[64], int wave, int nw, int lane) {
  const int rr = lane >> 3, cc = lane & 7;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const char* scr = t ? s1 : s0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (row0 + 32 * t + 8 * j + rr < nvalid) {
        const bf16x8 b = *(const bf16x8*)(scr + (8 * j + rr) * ST_PITCH + cc * 16);
#pragma unroll
        for (int e = 0; e < 8; ++e) cs[e] += (float)b[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    cs[e] += __shfl_xor(cs[e], 8, 64);
    cs[e] += __shfl_xor(cs[e], 16, 64);
    cs[e] += __shfl_xor(cs[e], 32, 64);
  }
  __syncthreads();                       // red is free (an earlier call's fold is done)
  if (lane < 8) {
#pragma unroll
    for (int e = 0; e < 8; ++e) red[wave][lane * 8 + e] = cs[e];
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    float t = 0.f;
    for (int w = 0; w < nw; ++w) t += red[w][threadIdx.x];
    colpart[threadIdx.x] = t;
  }
}

// dK/dV with TWO 32-key blocks per wave and one wave per SIMD (4 waves, up to 512 VGPRs): wave w
// owns keys 64w..64w+63.  Each Q | dO fragment read from LDS feeds both blocks' MFMAs (half the
// LDS reads per MFMA of attn_bwd_dkv_seq_bf16), and the two blocks' chains are independent, so
// one block's MFMAs can run under the other's exp / dS VALU inside the wave instead of relying
// on a co-resident wave.  Otherwise as attn_bwd_dkv_seq_bf16: persistent over the (batch, head)
// pairs, the next pair's Q | dO by LDS-DMA under this pair's loop, K / V rows, lse and delta in
// registers.  Key blocks past ceil(N/32) run on zero K / V rows and are never stored (rows >= N
// fall outside the store descriptor).  N <= 256; NQC > 0: ceil(N/32) as a compile-time constant.
template <int NPMAX, int NQC = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void attn_bwd_dkv_seq2_bf16(
    const bf16* __restrict__ qkv, const bf16* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, bf16* __restrict__ dqkv, int N, int H, float scale,
    float* __restrict__ colsum, int npairs) {
  constexpr int NW = 4;
  __shared__ __attribute__((aligned(16))) char smem[2][2 * NPMAX * 128];   // [buffer][Q | dO]
  __shared__ __attribute__((aligned(16))) float l2s[NPMAX];
  __shared__ __attribute__((aligned(16))) float dls[NPMAX];
  __shared__ float red[NW][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nq = NQC > 0 ? NQC : (N + 31) / 32, NP = nq * 32;
  const int D = H * DH;
  const int64_t ld = 3 * (int64_t)D, ldb = ld * 2, ldo = (int64_t)D * 2;
  const int h = lane >> 5;
  const uint32_t bytes = (uint32_t)((int64_t)N * ldb);
  const uint32_t obytes = (uint32_t)((int64_t)N * ldo);
  const int key0 = wave * 64 + (lane & 31);   // block j: key0 + 32 j
  const float c2 = scale * LOG2E;
  auto stage_pair = [&](int bh, int buf) {
    const int b = bh / H, hd = bh - b * H;
    const bf16* base = qkv + (int64_t)b * N * ld;
    stage_seq_dma(smem[buf], make_rsrc(base + hd * DH, bytes - hd * DH * 2), ldb, NP, NW, wave, lane);
    stage_seq_dma(smem[buf] + NP * 128, make_rsrc(dout + (int64_t)b * N * D + hd * DH, obytes - hd * DH * 2), ldo,
                  NP, NW, wave, lane);
  };
  auto load_regs = [&](int bh, bf16x8 (&kf)[2][4], bf16x8 (&vf)[2][4], float& ls, float& dv) {
    const int b = bh / H, hd = bh - b * H;
    const bf16* base = qkv + (int64_t)b * N * ld;
    const __amdgpu_buffer_rsrc_t rk = make_rsrc(base + D + hd * DH, bytes - (D + hd * DH) * 2);
    const __amdgpu_buffer_rsrc_t rv = make_rsrc(base + 2 * D + hd * DH, bytes - (2 * D + hd * DH) * 2);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint32_t kvoff = (uint32_t)((int64_t)(key0 + 32 * j) * ldb + 16 * h);   // 0 past N
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        kf[j][s] = __builtin_bit_cast(bf16x8, asm_load16(rk, kvoff, 32 * s));
        vf[j][s] = __builtin_bit_cast(bf16x8, asm_load16(rv, kvoff, 32 * s));
      }
    }
    const uint32_t ioff = (uint32_t)threadIdx.x * 4;
    ls = asm_load4(make_rsrc(lse + (int64_t)bh * N, (uint32_t)N * 4), ioff);
    dv = asm_load4(make_rsrc(delta + (int64_t)bh * N, (uint32_t)N * 4), ioff);
  };

  int bh = blockIdx.x;
  if (bh >= npairs) return;
  bf16x8 kf[2][4], vf[2][4];
  float ls, dv;
  stage_pair(bh, 0);
  load_regs(bh, kf, vf, ls, dv);
  int buf = 0;
  bool first = true;
  for (;;) {
    // everything but the previous pair's dK/dV stores (16 per wave, + 2 column-sum stores on
    // wave 0), which are younger; see attn_bwd_dkv_seq_bf16 for the inline-asm loads and the pin
    if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (colsum && wave == 0) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    first = false;
    asm volatile("" : "+v"(kf[0][0]), "+v"(kf[0][1]), "+v"(kf[0][2]), "+v"(kf[0][3]), "+v"(vf[0][0]), "+v"(vf[0][1]),
                 "+v"(vf[0][2]), "+v"(vf[0][3]), "+v"(kf[1][0]), "+v"(kf[1][1]), "+v"(kf[1][2]), "+v"(kf[1][3]),
                 "+v"(vf[1][0]), "+v"(vf[1][1]), "+v"(vf[1][2]), "+v"(vf[1][3]), "+v"(ls), "+v"(dv));
    if (threadIdx.x < NP) {
      const int i = threadIdx.x;
      l2s[i] = i < N ? ls * LOG2E : INFINITY;
      dls[i] = i < N ? dv : 0.f;
    }
    __syncthreads();   // Q | dO and l2s / dls visible; every wave is done with the other buffer
    const int nbh = bh + gridDim.x;
    const bool more = nbh < npairs;
    if (more) stage_pair(nbh, buf ^ 1);
    const char* qt = smem[buf];
    const char* dt_ = qt + NP * 128;
    f32x16 dvt[2][2] = {{zero16(), zero16()}, {zero16(), zero16()}};
    f32x16 dkt[2][2] = {{zero16(), zero16()}, {zero16(), zero16()}};
    auto qblock = [&](const int q0) {
      f32x16 sa[2], dp[2];
      f32x4 L2[4];
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {   // row constants: dP - delta straight from the MFMA chain
        const int q4 = q0 + 8 * g4 + 4 * h;   // rows acc_row(4*g4 + i, h) = q4 + i
        L2[g4] = *(const f32x4*)(l2s + q4);
        const f32x4 dl = *(const f32x4*)(dls + q4);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) dp[j][4 * g4 + i] = -dl[i];
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) sa[j] = zero16();
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 qa = frag_row(qt, q0, s, lane), da = frag_row(dt_, q0, s, lane);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          sa[j] = mfma32(qa, kf[j][s], sa[j]);    // S[q][key]
          dp[j] = mfma32(da, vf[j][s], dp[j]);    // dP[q][key] - delta[q]
        }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float p = fexp2(fmaf(sa[j][4 * g4 + i], c2, -L2[g4][i]));
            sa[j][4 * g4 + i] = p;
            dp[j][4 * g4 + i] = p * dp[j][4 * g4 + i];
          }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 td[2], tq[2];
#pragma unroll
        for (int d2 = 0; d2 < 2; ++d2) {
          td[d2] = frag_tr(dt_, q0 + 16 * s, 32 * d2, lane);
          tq[d2] = frag_tr(qt, q0 + 16 * s, 32 * d2, lane);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const bf16x8 pb = pack8(sa[j], s), sb = pack8(dp[j], s);
#pragma unroll
          for (int d2 = 0; d2 < 2; ++d2) {
            dvt[j][d2] = mfma32(td[d2], pb, dvt[j][d2]);
            dkt[j][d2] = mfma32(tq[d2], sb, dkt[j][d2]);
          }
        }
      }
    };
    if constexpr (NQC > 0) {
#pragma unroll
      for (int q0 = 0; q0 < NQC * 32; q0 += 32) qblock(q0);
    } else {
#pragma unroll 1
      for (int q0 = 0; q0 < NP; q0 += 32) qblock(q0);
    }
    if (more) load_regs(nbh, kf, vf, ls, dv);   // (kf / vf are dead until the next pair)
    // dK, dV through this pair's (now free) Q | dO image: every wave must be done reading it
    __syncthreads();
    {
      const int b = bh / H, hd = bh - b * H;
      const bf16* db = dqkv + (int64_t)b * N * ld;
      const __amdgpu_buffer_rsrc_t rdk = make_rsrc(db + D + hd * DH, bytes - (D + hd * DH) * 2);
      const __amdgpu_buffer_rsrc_t rdv = make_rsrc(db + 2 * D + hd * DH, bytes - (2 * D + hd * DH) * 2);
      char* s0 = smem[buf] + (2 * wave) * ST_BYTES;
      char* s1 = s0 + ST_BYTES;
      float* part = colsum + (int64_t)b * 3 * D + hd * DH;   // the k- and v-bias gradient partials
      const int ln = lane_here();
      store_tile32(s0, dkt[0], scale, rdk, ldb, wave * 64, ln);
      store_tile32(s1, dkt[1], scale, rdk, ldb, wave * 64 + 32, ln);
      if (colsum) tile32x2_colsum(s0, s1, wave * 64, N, part + D, red, wave, NW, ln);
      else asm volatile("" ::: "memory");
      store_tile32(s0, dvt[0], 1.f, rdv, ldb, wave * 64, ln);
      store_tile32(s1, dvt[1], 1.f, rdv, ldb, wave * 64 + 32, ln);
      if (colsum) tile32x2_colsum(s0, s1, wave * 64, N, part + 2 * D, red, wave, NW, ln);
    }
    if (!more) break;
    bh = nbh;
    buf ^= 1;
  }
}

// ---------------------------------------------- fused single-pass backward (N <= NPMAX)
// One workgroup per (batch, head), NW = ceil(N/32) waves; wave w owns keys 32w..32w+31 exactly
// as in attn_bwd_dkv_seq_bf16 (dK, dV accumulate in registers), and S, P, dP and dS of every
// 32x32 block are formed ONCE (the two-kernel path forms them in both kernels: 28 MFMAs + two
// exp passes per block, here 20 + one).  dQ needs a sum over keys, i.e. over waves:
//   * the wave's dS block (accumulator: key on the lane) goes to a per-wave LDS scratch as
//     dS^T[key][q] with 8-B writes, and comes back with ds_read_b64_tr_b16 as the B operand
//     with q on the lane;
//   * dQ^T[d][q] += K^T[d][key] dS^T[key][q], with the wave's K^T fragments in registers;
//   * the partial goes into an fp32 dQ image in LDS by read-add-write.  At step t wave w works
//     on query tile (w + t) mod NW and adds only after the tile's turn counter says step t-1's
//     add is in, so every tile has one writer at a time and its sum order (w = tile, tile-1, ...)
//     is fixed: deterministic, no atomics, no workgroup barrier inside the loop.
// Delta = rowsum(dO * O) is formed in the prologue (each wave its own 32 query rows).
// LDS (NPMAX = 256): Q | dO images 64 KiB + dQ fp32 [256][68] 68 KiB + L2 | delta 2 KiB +
// scratch 8 x 2 KiB = 150 KiB: one workgroup per CU.
__device__ __forceinline__ int scr_off(int key, int chunk) { return key * 64 + ((chunk ^ (key & 7)) << 3); }

template <int NPMAX>
__global__ __launch_bounds__(NPMAX * 2) void attn_bwd_fused_seq_bf16(
    const bf16* __restrict__ qkv, const bf16* __restrict__ o, const bf16* __restrict__ dout,
    const float* __restrict__ lse, bf16* __restrict__ dqkv, int N, int H, float scale) {
  constexpr int DQP = 68;                                  // dQ image row pitch (floats)
  constexpr int OFF_DQ = 2 * NPMAX * 128;
  constexpr int OFF_ROW = OFF_DQ + NPMAX * DQP * 4;
  constexpr int OFF_SCR = OFF_ROW + 2 * NPMAX * 4;
  constexpr int OFF_TURN = OFF_SCR + (NPMAX / 32) * 2048;
  __shared__ __attribute__((aligned(16))) char smem[OFF_TURN + (NPMAX / 32) * 4];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = blockDim.x >> 6, NP = nw * 32;
  const int bh = blockIdx.x, b = bh / H, hd = bh % H;
  const int D = H * DH;
  const int64_t ld = 3 * (int64_t)D, ldb = ld * 2, ldo = (int64_t)D * 2;
  const int h = lane >> 5;
  const bf16* base = qkv + (int64_t)b * N * ld;
  const uint32_t bytes = (uint32_t)((int64_t)N * ldb);
  const uint32_t obytes = (uint32_t)((int64_t)N * ldo);
  __amdgpu_buffer_rsrc_t rq = make_rsrc(base + hd * DH, bytes - hd * DH * 2);
  __amdgpu_buffer_rsrc_t rk = make_rsrc(base + D + hd * DH, bytes - (D + hd * DH) * 2);
  __amdgpu_buffer_rsrc_t rv = make_rsrc(base + 2 * D + hd * DH, bytes - (2 * D + hd * DH) * 2);
  __amdgpu_buffer_rsrc_t rdo = make_rsrc(dout + (int64_t)b * N * D + hd * DH, obytes - hd * DH * 2);
  __amdgpu_buffer_rsrc_t ro = make_rsrc(o + (int64_t)b * N * D + hd * DH, obytes - hd * DH * 2);
  char* qt = smem;
  char* dt_ = smem + NPMAX * 128;
  float* dqs = (float*)(smem + OFF_DQ);
  float* l2s = (float*)(smem + OFF_ROW);
  float* dls = l2s + NPMAX;
  char* scr = smem + OFF_SCR + wave * 2048;

  // prologue: Q, dO images; the K image (128-B rows) parked in the dQ area for the K^T fragments
  stage_seq(qt, rq, ldb, NP, nw, wave, lane);
  stage_seq(dt_, rdo, ldo, NP, nw, wave, lane);
  stage_seq(smem + OFF_DQ, rk, ldb, NP, nw, wave, lane);
  const int r32 = wave * 32 + (lane & 31);   // this lane's key (dK/dV) and query (delta) row
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = load_row16(rk, (uint32_t)((int64_t)r32 * ldb + (16 * s + 8 * h) * 2));
    vf[s] = load_row16(rv, (uint32_t)((int64_t)r32 * ldb + (16 * s + 8 * h) * 2));
  }
  float dl;
  {
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const uint32_t off = (uint32_t)((int64_t)r32 * ldo + (16 * s + 8 * h) * 2);
      const bf16x8 dv = load_row16(rdo, off), ov = load_row16(ro, off);
#pragma unroll
      for (int j = 0; j < 8; ++j) part += (float)ov[j] * (float)dv[j];
    }
    dl = part + __shfl_xor(part, 32, 64);
  }
  const bool rok = r32 < N;
  const float l2v = rok ? lse[(int64_t)bh * N + r32] * LOG2E : INFINITY;   // q >= N -> P = 0
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (h == 0) {
    l2s[r32] = l2v;
    dls[r32] = rok ? dl : 0.f;
  }
  __syncthreads();
  // K^T[d][key] fragments of this wave's keys (A operands of dQ^T = K^T dS^T)
  bf16x8 ktf[2][2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int d2 = 0; d2 < 2; ++d2) ktf[s][d2] = frag_tr(smem + OFF_DQ, wave * 32 + 16 * s, 32 * d2, lane);
  __syncthreads();   // (the barrier's fence retires the reads before the area is zeroed)
  for (int i = threadIdx.x; i < NP * DQP / 4; i += blockDim.x) ((f32x4*)dqs)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  int* turn = (int*)(smem + OFF_TURN);   // turn[tile] = steps whose dQ add into the tile is done
  if (threadIdx.x < nw) turn[threadIdx.x] = 0;
  __syncthreads();

  const float c2 = scale * LOG2E;
  const int g16 = lane >> 4, tl = lane & 15, qq = tl >> 2, pp = tl & 3;
  f32x16 dvt[2] = {zero16(), zero16()}, dkt[2] = {zero16(), zero16()};
#pragma unroll 1
  for (int t = 0; t < nw; ++t) {
    int qi = wave + t;
    if (qi >= nw) qi -= nw;
    const int q0 = qi * 32;
    f32x16 sa = zero16(), dp = zero16();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      sa = mfma32(frag_row(qt, q0, s, lane), kf[s], sa);    // S[q][key]
      dp = mfma32(frag_row(dt_, q0, s, lane), vf[s], dp);   // dP[q][key]
    }
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int q4 = q0 + 8 * g4 + 4 * h;
      const f32x4 L2 = *(const f32x4*)(l2s + q4);
      const f32x4 d4 = *(const f32x4*)(dls + q4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = fexp2(fmaf(sa[4 * g4 + i], c2, -L2[i]));
        sa[4 * g4 + i] = p;
        dp[4 * g4 + i] = p * (dp[4 * g4 + i] - d4[i]);
      }
    }
    // dS^T[key][q] into the scratch: rows q = 8*g4 + 4h + 0..3 of this lane's key column
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      bf16x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (bf16)dp[4 * g4 + i];
      *(bf16x4*)(scr + scr_off(lane & 31, 2 * g4 + h)) = v;
    }
    asm volatile("" ::: "memory");   // scratch writes stay ahead of the transposed reads
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 pb = pack8(sa, s), sb = pack8(dp, s);
#pragma unroll
      for (int d2 = 0; d2 < 2; ++d2) {
        dvt[d2] = mfma32(frag_tr(dt_, q0 + 16 * s, 32 * d2, lane), pb, dvt[d2]);
        dkt[d2] = mfma32(frag_tr(qt, q0 + 16 * s, 32 * d2, lane), sb, dkt[d2]);
      }
    }
    // dQ^T[d][q] partial of this wave's 32 keys; B = dS^T with q on the lane (transposed read
    // of the scratch: element j <-> key 16s + 8(j>>2) + 4h + (j&3), the frag_tr k order)
    f32x16 dqp[2] = {zero16(), zero16()};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 sbt;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = 16 * s + 8 * i + 4 * (g16 >> 1) + qq;
        s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, scr + scr_off(row, 4 * (g16 & 1) + pp)));
        bf16x4 bv = __builtin_bit_cast(bf16x4, v);
#pragma unroll
        for (int j = 0; j < 4; ++j) sbt[4 * i + j] = bv[j];
      }
#pragma unroll
      for (int d2 = 0; d2 < 2; ++d2) dqp[d2] = mfma32(ktf[s][d2], sbt, dqp[d2]);
    }
    // this step's only writer of query tile qi: dQ[q][d] += partial (lane q, d = 32d2 + acc_row).
    // Step t-1 of tile qi belonged to wave w+1; wait for its add (turn[qi] == t) instead of a
    // workgroup barrier, so the waves drift apart and one wave's MFMAs overlap another's softmax.
    // The waits form a chain (w waits on w+1 one step earlier), so they always resolve; the
    // bound only guards against a logic error hanging the device.  Should it ever be hit, the
    // tile's dQ is poisoned with NaN (the parity tests then fail loudly) instead of being
    // summed out of order.
    bool late;
    {
      volatile int* tp = turn + qi;
      for (int spin = 0; *tp != t && spin < (1 << 22); ++spin) __builtin_amdgcn_s_sleep(1);
      late = *tp != t;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    float* dq_row = dqs + (q0 + (lane & 31)) * DQP;
    const float poison = late ? __builtin_nanf("") : 0.f;
#pragma unroll
    for (int d2 = 0; d2 < 2; ++d2)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        f32x4* pq = (f32x4*)(dq_row + 32 * d2 + 8 * g4 + 4 * h);
        f32x4 a = *pq;
        a[0] += dqp[d2][4 * g4] + poison;
        a[1] += dqp[d2][4 * g4 + 1] + poison;
        a[2] += dqp[d2][4 * g4 + 2] + poison;
        a[3] += dqp[d2][4 * g4 + 3] + poison;
        *pq = a;
      }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    *(volatile int*)(turn + qi) = t + 1;
  }
  __syncthreads();   // every tile's last add is in
  // dK, dV of the wave's keys
  if (rok) {
    bf16* row = dqkv + ((int64_t)b * N + r32) * ld;
#pragma unroll
    for (int d2 = 0; d2 < 2; ++d2)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = 32 * d2 + 8 * g4 + 4 * h;
        store4(row + D + hd * DH + d, dkt[d2][4 * g4] * scale, dkt[d2][4 * g4 + 1] * scale,
               dkt[d2][4 * g4 + 2] * scale, dkt[d2][4 * g4 + 3] * scale);
        store4(row + 2 * D + hd * DH + d, dvt[d2][4 * g4], dvt[d2][4 * g4 + 1], dvt[d2][4 * g4 + 2],
               dvt[d2][4 * g4 + 3]);
      }
    // dQ of query row r32 (all writers finished at the loop's last barrier): half h = d 32h..
    bf16* qrow = row + hd * DH + 32 * h;
    const float* src = dqs + r32 * DQP + 32 * h;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const f32x4 a = *(const f32x4*)(src + 4 * c);
      store4(qrow + 4 * c, a[0] * scale, a[1] * scale, a[2] * scale, a[3] * scale);
    }
  }
}

// ---- gemm.hip: weight gradients from token-contiguous operand copies (VITMI_WGRAD_T; the
// EPI_PARTIAL epilogue also had a transposed-slab branch, GemmArgs::ct)
extern "C" size_t vitmi_linear_wgrad_xt_workspace_size(int dtype, int64_t M, int64_t N, int64_t K) {
  // the transposed product dW^T[K,N]: GEMM rows K, cols N, reduction M; at least one slab
  const int splits = choose_splits(dtype, K, N, M);
  return (size_t)(splits > 1 ? splits : 1) * N * K * sizeof(float);
}

extern "C" int vitmi_linear_wgrad_xt(int dtype, int64_t M, int64_t N, int64_t K, const void* dy, const void* xt,
                                     int64_t ldxt, float* dw, void* workspace, size_t ws_bytes,
                                     vitmi_stream_t stream) {
  // dW[N,K] += sum_m dy[m][n] xt[k][m], formed as the product dW^T = xt dy: A(k,m) = xt (m
  // contiguous: k-major in GEMM terms), B(m,n) = dy (n contiguous); the slabs are written transposed
  return gemm_impl(dtype, 1, 0, K, N, M, xt, ldxt, dy, N, dw, K, VITMI_F32, VITMI_EPI_ACCUM, nullptr, nullptr, 0,
                   nullptr, 0, workspace, ws_bytes, (hipStream_t)stream, true, nullptr, nullptr, nullptr, true);
}

extern "C" int vitmi_linear_wgrad_dyt(int dtype, int64_t M, int64_t N, int64_t K, const void* dyt, int64_t lddyt,
                                      const void* x, float* dw, void* workspace, size_t ws_bytes,
                                      vitmi_stream_t stream) {
  // dW[N,K] += sum_m dyt[n][m] x[m][k]: A(n,m) = dyt (m contiguous), B(m,k) = x (k contiguous);
  // workspace: vitmi_linear_wgrad_workspace_size
  return gemm_impl(dtype, 1, 0, N, K, M, dyt, lddyt, x, K, dw, K, VITMI_F32, VITMI_EPI_ACCUM, nullptr, nullptr, 0,
                   nullptr, 0, workspace, ws_bytes, (hipStream_t)stream, true);
}

