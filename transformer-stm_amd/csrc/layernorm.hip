// layernorm.hip — LayerNorm forward/backward (layers.LayerNormalization(epsilon=1e-6),
// models/CvT(Par).py:248,272,278,328; nn.LayerNorm old_codes/MS_CvT.py:39-45,307,315).
//
// HBM-bound: one wave per row, the row held in registers as float4 (D <= 2048),
// fp32 statistics.  Forward writes y in the GEMM operand dtype plus mean/rstd;
// backward fuses the residual-gradient add (dx = dres + LN'(dy)) and the bf16 copy
// the next GEMM consumes, and produces per-block dgamma/dbeta partials that a
// second pass folds into the fp32 parameter gradients (+=).
#include "common.h"
#include <algorithm>

namespace vitmi {

// Outputs leave with the non-temporal hint, as gemm256's bf16 outputs (VITMI_NT_LN): forward
// 36.7 -> 34.9 us, backward 126 -> 122 us, step +0.4 % (profiles/r03_store_nt/ln_*)
#ifndef VITMI_NT_LN
#define VITMI_NT_LN 1
#endif
// backward: the next row's loads issued before this row is reduced (A/B builds)
#ifndef VITMI_LN_BWD_PIPE
#define VITMI_LN_BWD_PIPE 0
#endif
template <typename V>
__device__ __forceinline__ void put(V* p, V v) {
  if constexpr (VITMI_NT_LN) __builtin_nontemporal_store(v, p);
  else *p = v;
}
template <typename TY>
__device__ __forceinline__ void store4(TY* p, f32x4 v);
template <>
__device__ __forceinline__ void store4<float>(float* p, f32x4 v) { put((f32x4*)p, v); }
template <>
__device__ __forceinline__ void store4<bf16>(bf16* p, f32x4 v) {
  bf16x4 b;
  b[0] = (bf16)v[0]; b[1] = (bf16)v[1]; b[2] = (bf16)v[2]; b[3] = (bf16)v[3];
  put((bf16x4*)p, b);
}
template <typename T>
__device__ __forceinline__ f32x4 load4(const T* p);
template <>
__device__ __forceinline__ f32x4 load4<float>(const float* p) { return *(const f32x4*)p; }
template <>
__device__ __forceinline__ f32x4 load4<bf16>(const bf16* p) {
  bf16x4 b = *(const bf16x4*)p;
  return f32x4{(float)b[0], (float)b[1], (float)b[2], (float)b[3]};
}

// ---------------------------------------------------------------- forward
template <int NV, typename TY>
__global__ __launch_bounds__(256) void ln_fwd_kernel(int64_t M, int D, const float* __restrict__ x,
                                                     int64_t ldx, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps,
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
    v[i] = c < D ? *(const f32x4*)(xr + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
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

// ---------------------------------------------------------------- backward
// grid = G blocks x 256 threads; wave w of block b handles rows b*4+w, +4G, ...
template <int NV, typename TDY, bool LP>
__global__ __launch_bounds__(256) void ln_bwd_kernel(
    int64_t M, int D, const TDY* __restrict__ dy, int64_t lddy, const float* __restrict__ x,
    int64_t ldx, const float* __restrict__ mean, const float* __restrict__ rstd,
    const float* __restrict__ gamma, const float* __restrict__ dres, int64_t ldres,
    float* __restrict__ dx, int64_t lddx, bf16* __restrict__ dx_lp, int64_t lddx_lp,
    float* __restrict__ part) {
  __shared__ f32x4 red[4][64 * NV * 3];
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
  for (int64_t row = (int64_t)blockIdx.x * 4 + wave; row < M; row += (int64_t)gridDim.x * 4) {
    const float mu = mean[row], rs = rstd[row];
    f32x4 xh[NV], gy[NV], rv[NV];
    float s1 = 0.f, s2 = 0.f;
    // the residual gradient is loaded with x and dy: one memory round trip per row
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
#endif
        xh[i] = (xv - mu) * rs;
        gy[i] = dyv * g[i];
        dg[i] += dyv * xh[i];
        db[i] += dyv;
        s1 += gy[i][0] + gy[i][1] + gy[i][2] + gy[i][3];
        const f32x4 t = gy[i] * xh[i];
        s2 += t[0] + t[1] + t[2] + t[3];
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
        if (LP) store4<bf16>(dx_lp + row * lddx_lp + c, o);
      }
    }
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
  }
  // block-reduce dgamma / dbeta / colsum(dx) partials over the 4 waves
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    red[wave][i * 64 + lane] = dg[i];
    red[wave][(NV + i) * 64 + lane] = db[i];
    red[wave][(2 * NV + i) * 64 + lane] = ds[i];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < NV * 3 * 64; e += 256) {
    const f32x4 t = red[0][e] + red[1][e] + red[2][e] + red[3][e];
    const int which = e / (NV * 64);          // 0 = dgamma, 1 = dbeta, 2 = colsum(dx)
    const int i = (e % (NV * 64)) / 64, l = e % 64;
    const int c = (l + 64 * i) * 4;
    if (c < D) *(f32x4*)(part + ((int64_t)which * gridDim.x + blockIdx.x) * D + c) = t;
  }
}

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

// out[d] += sum_b part[b][d] for dgamma (rows 0..G-1), dbeta (G..2G-1), colsum(dx) (2G..3G-1),
// in a fixed order (deterministic).
// loads in flight per thread of the partial folds (A/B builds; the fold is latency-bound)
#ifndef VITMI_LNR_UNROLL
#define VITMI_LNR_UNROLL 8
#endif
__global__ __launch_bounds__(1024) void ln_param_reduce(const float* __restrict__ part, int G, int D,
                                                        float* __restrict__ dgamma,
                                                        float* __restrict__ dbeta,
                                                        float* __restrict__ dxsum) {
  // block = 16 columns x 64 row groups (48 blocks at D = 768, not 12: the fold is latency-
  // bound, 13.4 us with 64-column blocks); row group gi sums partials gi, gi+64, ..., then
  // thread (array, column) adds the 64 group sums in order
  __shared__ float red[3][64][17];
  const int c = threadIdx.x & 15, gi = threadIdx.x >> 4;
  const int d = blockIdx.x * 16 + c;
  float a = 0.f, b = 0.f, e = 0.f;
  if (d < D) {
#pragma unroll VITMI_LNR_UNROLL
    for (int i = gi; i < G; i += 64) {
      a += part[(int64_t)i * D + d];
      b += part[(int64_t)(G + i) * D + d];
      if (dxsum) e += part[(int64_t)(2 * G + i) * D + d];
    }
  }
  red[0][gi][c] = a;
  red[1][gi][c] = b;
  red[2][gi][c] = e;
  __syncthreads();
  if (threadIdx.x < 48) {
    const int w = threadIdx.x >> 4, c2 = threadIdx.x & 15, d2 = blockIdx.x * 16 + c2;
    float* out = w == 0 ? dgamma : (w == 1 ? dbeta : dxsum);
    if (d2 < D && out) {
      float sum = 0.f;
      for (int k = 0; k < 64; ++k) sum += red[w][k][c2];
      out[d2] += sum;
    }
  }
}

#ifndef VITMI_LN_BWD_BLOCKS
#define VITMI_LN_BWD_BLOCKS 512
#endif
static int ln_blocks_bwd(int64_t M) {
  int64_t g = (M + 3) / 4;
  return (int)(g < VITMI_LN_BWD_BLOCKS ? (g < 1 ? 1 : g) : VITMI_LN_BWD_BLOCKS);
}

template <int NV>
static void ln_fwd_launch(hipStream_t s, int64_t M, int D, const float* x, int64_t ldx,
                          const float* gamma, const float* beta, float eps, void* y, int ydt,
                          int64_t ldy, float* mean, float* rstd) {
  dim3 grid((unsigned)((M + 3) / 4));
  if (ydt == VITMI_BF16)
    hipLaunchKernelGGL((ln_fwd_kernel<NV, bf16>), grid, dim3(256), 0, s, M, D, x, ldx, gamma, beta,
                       eps, (bf16*)y, ldy, mean, rstd);
  else
    hipLaunchKernelGGL((ln_fwd_kernel<NV, float>), grid, dim3(256), 0, s, M, D, x, ldx, gamma, beta,
                       eps, (float*)y, ldy, mean, rstd);
  // x (fp32) read, y written, mean/rstd written
  const double ysz = ydt == VITMI_BF16 ? 2 : 4;
  if (ydt == VITMI_BF16) VITMI_STAT((ln_fwd_kernel<NV, bf16>), 0, (double)M * D * (4 + ysz) + 8.0 * M);
  else VITMI_STAT((ln_fwd_kernel<NV, float>), 0, (double)M * D * (4 + ysz) + 8.0 * M);
}

template <int NV, typename TDY>
static void ln_bwd_launch(hipStream_t s, int G, int64_t M, int D, const void* dy, int64_t lddy,
                          const float* x, int64_t ldx, const float* mean, const float* rstd,
                          const float* gamma, const float* dres, int64_t ldres, float* dx,
                          int64_t lddx, void* dx_lp, int64_t lddx_lp, float* part) {
  if (dx_lp)
    hipLaunchKernelGGL((ln_bwd_kernel<NV, TDY, true>), dim3(G), dim3(256), 0, s, M, D,
                       (const TDY*)dy, lddy, x, ldx, mean, rstd, gamma, dres, ldres, dx, lddx,
                       (bf16*)dx_lp, lddx_lp, part);
  else
    hipLaunchKernelGGL((ln_bwd_kernel<NV, TDY, false>), dim3(G), dim3(256), 0, s, M, D,
                       (const TDY*)dy, lddy, x, ldx, mean, rstd, gamma, dres, ldres, dx, lddx,
                       (bf16*)nullptr, 0, part);
  // dy + x (+ dres) read, dx (+ bf16 copy) written
  const double b = (double)M * D * (sizeof(TDY) + 4 + (dres ? 4 : 0) + 4 + (dx_lp ? 2 : 0)) + 8.0 * M;
  if (dx_lp) VITMI_STAT((ln_bwd_kernel<NV, TDY, true>), 0, b);
  else VITMI_STAT((ln_bwd_kernel<NV, TDY, false>), 0, b);
}

}  // namespace vitmi

using namespace vitmi;

extern "C" int vitmi_layernorm_fwd(int64_t M, int D, const float* x, int64_t ldx,
                                   const float* gamma, const float* beta, float eps, void* y,
                                   int y_dtype, int64_t ldy, float* mean, float* rstd,
                                   vitmi_stream_t stream) {
  VITMI_CHECK_ARG(D > 0 && D % 4 == 0 && D <= 2048, "layernorm: D must be a multiple of 4 in [4, 2048]");
  VITMI_CHECK_ARG(ldx % 4 == 0 && ldy % 4 == 0, "layernorm: strides must be multiples of 4");
  if (M == 0) return VITMI_OK;
  VITMI_CHECK_ARG(x && gamma && beta && y && mean && rstd, "layernorm_fwd: null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int nv = (D + 255) / 256;
  switch (nv) {
    case 1: ln_fwd_launch<1>(s, M, D, x, ldx, gamma, beta, eps, y, y_dtype, ldy, mean, rstd); break;
    case 2: ln_fwd_launch<2>(s, M, D, x, ldx, gamma, beta, eps, y, y_dtype, ldy, mean, rstd); break;
    case 3: ln_fwd_launch<3>(s, M, D, x, ldx, gamma, beta, eps, y, y_dtype, ldy, mean, rstd); break;
    case 4: ln_fwd_launch<4>(s, M, D, x, ldx, gamma, beta, eps, y, y_dtype, ldy, mean, rstd); break;
    default: ln_fwd_launch<8>(s, M, D, x, ldx, gamma, beta, eps, y, y_dtype, ldy, mean, rstd); break;
  }
  VITMI_LAUNCH_CHECK("layernorm_fwd");
  return VITMI_OK;
}

extern "C" size_t vitmi_layernorm_bwd_workspace_size(int64_t M, int D) {
  return (size_t)3 * ln_blocks_bwd(M) * D * sizeof(float);
}

extern "C" int vitmi_layernorm_bwd(int64_t M, int D, const void* dy, int dy_dtype, int64_t lddy,
                                   const float* x, int64_t ldx, const float* mean,
                                   const float* rstd, const float* gamma, const float* dres,
                                   int64_t ldres, float* dx, int64_t lddx, void* dx_lp,
                                   int64_t lddx_lp, float* dgamma, float* dbeta, float* dxsum,
                                   void* workspace, size_t ws_bytes, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(D > 0 && D % 4 == 0 && D <= 2048, "layernorm: D must be a multiple of 4 in [4, 2048]");
  if (M == 0) return VITMI_OK;
  VITMI_CHECK_ARG(dy && x && mean && rstd && gamma && dx, "layernorm_bwd: null pointer");
  VITMI_CHECK_ARG(workspace && ws_bytes >= vitmi_layernorm_bwd_workspace_size(M, D),
                  "layernorm_bwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int G = ln_blocks_bwd(M);
  float* part = (float*)workspace;
  const int nv = (D + 255) / 256;
#define LNB(NV)                                                                                  \
  if (dy_dtype == VITMI_BF16)                                                                    \
    ln_bwd_launch<NV, bf16>(s, G, M, D, dy, lddy, x, ldx, mean, rstd, gamma, dres, ldres, dx,    \
                            lddx, dx_lp, lddx_lp, part);                                         \
  else                                                                                           \
    ln_bwd_launch<NV, float>(s, G, M, D, dy, lddy, x, ldx, mean, rstd, gamma, dres, ldres, dx,   \
                             lddx, dx_lp, lddx_lp, part);
  switch (nv) {
    case 1: LNB(1) break;
    case 2: LNB(2) break;
    case 3: LNB(3) break;
    case 4: LNB(4) break;
    default: LNB(8) break;
  }
#undef LNB
  hipLaunchKernelGGL(ln_param_reduce, dim3((D + 15) / 16), dim3(1024), 0, s, (const float*)part, G,
                     D, dgamma, dbeta, dxsum);
  VITMI_LAUNCH_CHECK("layernorm_bwd");
  return VITMI_OK;
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
