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
#include <type_traits>

namespace vitmi {

// Outputs leave with the non-temporal hint, as gemm256's bf16 outputs (VITMI_NT_LN): forward
// 36.7 -> 34.9 us, backward 126 -> 122 us, step +0.4 % (profiles/r03_store_nt/ln_*)
#ifndef VITMI_NT_LN
#define VITMI_NT_LN 1
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
// y dtype tag of the precision knob's A operand (VITMI_BF16X3): bf16 rows [hi | hi | lo] of 3D
// columns, hi = bf16(y), lo = bf16(y - hi) (csrc/split.hip), written straight from the fp32 row
struct SplitX3 {};
// ... and of the VITMI_BF16F8 knob: rows of 2D bf16 units, [hi | hi8 | lo8] (common.h split_f8)
struct SplitF8 {};
// ... and of its weight-side form (VITMI_BF16F8W): rows of 1.5D bf16 units, [hi | hi8] (one byte per k)
struct SplitF8W {};

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
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (lane + 64 * i) * 4;
    if (c < D) {
      const f32x4 g = *(const f32x4*)(gamma + c);
      const f32x4 b = *(const f32x4*)(beta + c);
      const f32x4 o = (v[i] - mu) * rs * g + b;
      if constexpr (std::is_same_v<TY, SplitX3>) {
        bf16* yr = (bf16*)y + row * ldy + c;
        bf16x4 hi, lo;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          hi[e] = (bf16)o[e];
          lo[e] = (bf16)(o[e] - (float)hi[e]);
        }
        put((bf16x4*)yr, hi);
        put((bf16x4*)(yr + D), hi);
        put((bf16x4*)(yr + 2 * D), lo);
      } else if constexpr (std::is_same_v<TY, SplitF8>) {
        bf16* yr = (bf16*)y + row * ldy;
        bf16x4 hi;
        uint32_t hi8, lo8;
        split_f8(o, hi, hi8, lo8);
        put((bf16x4*)(yr + c), hi);
        uint8_t* f8 = (uint8_t*)(yr + D) + f8_off(c);
        *(uint32_t*)f8 = hi8;
        *(uint32_t*)(f8 + 64) = lo8;
      } else if constexpr (std::is_same_v<TY, SplitF8W>) {
        bf16* yr = (bf16*)y + row * ldy;
        bf16x4 hi;
        uint32_t hi8, lo8;
        split_f8(o, hi, hi8, lo8);
        put((bf16x4*)(yr + c), hi);
        *(uint32_t*)((uint8_t*)(yr + D) + c) = hi8;
      } else {
        store4<TY>(y + row * ldy + c, o);
      }
    }
  }
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

// D = 4L <= 128 (the CvT's stages 1 and 2): L lanes per row, 64 / L rows per wave, row sums by xor
// shuffles inside the row's lanes (the one-row kernel keeps 16 / 32 of 64 lanes busy there)
template <int L, typename TY>
__global__ __launch_bounds__(256) void ln_fwd_small_kernel(int64_t M, const float* __restrict__ x, int64_t ldx,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float eps,
                                                           TY* __restrict__ y, int64_t ldy,
                                                           float* __restrict__ mean, float* __restrict__ rstd) {
  constexpr int D = 4 * L, RW = 64 / L;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = (lane % L) * 4;
  const int64_t row = ((int64_t)blockIdx.x * 4 + wave) * RW + lane / L;
  const bool ok = row < M;
  const f32x4 v = ok ? *(const f32x4*)(x + row * ldx + c) : f32x4{0.f, 0.f, 0.f, 0.f};
  float s = v[0] + v[1] + v[2] + v[3];
#pragma unroll
  for (int o = 1; o < L; o <<= 1) s += __shfl_xor(s, o, 64);
  const float mu = s / D;
  const f32x4 d = v - mu;
  float q = d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3];
#pragma unroll
  for (int o = 1; o < L; o <<= 1) q += __shfl_xor(q, o, 64);
  const float rs = rsqrtf(q / D + eps);
  if (ok) {
    const f32x4 g = *(const f32x4*)(gamma + c);
    const f32x4 b = *(const f32x4*)(beta + c);
    store4<TY>(y + row * ldy + c, (v - mu) * rs * g + b);
    if (c == 0) {
      mean[row] = mu;
      rstd[row] = rs;
    }
  }
}

// ---------------------------------------------------------------- backward
// VITMI_LN_BWD_NTLD: the backward's once-read inputs (x, dy, dres) with the non-temporal hint
#ifndef VITMI_LN_BWD_NTLD
#define VITMI_LN_BWD_NTLD 1
#endif
template <typename V>
__device__ __forceinline__ V ldg_s(const V* p) {
  if constexpr (VITMI_LN_BWD_NTLD) return __builtin_nontemporal_load(p);
  else return *p;
}
template <typename T>
__device__ __forceinline__ f32x4 load4s(const T* p);
template <>
__device__ __forceinline__ f32x4 load4s<float>(const float* p) { return ldg_s((const f32x4*)p); }
template <>
__device__ __forceinline__ f32x4 load4s<bf16>(const bf16* p) {
  const bf16x4 b = ldg_s((const bf16x4*)p);
  return f32x4{(float)b[0], (float)b[1], (float)b[2], (float)b[3]};
}
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
  for (int64_t row = (int64_t)blockIdx.x * 4 + wave; row < M; row += (int64_t)gridDim.x * 4) {
    const float mu = mean[row], rs = rstd[row];
    f32x4 xh[NV], gy[NV], rv[NV];
    float s1 = 0.f, s2 = 0.f;
    // the residual gradient is loaded with x and dy: one memory round trip per row
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (lane + 64 * i) * 4;
      rv[i] = (dres && c < D) ? ldg_s((const f32x4*)(dres + row * ldres + c)) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (lane + 64 * i) * 4;
      if (c < D) {
        const f32x4 xv = ldg_s((const f32x4*)(x + row * ldx + c));
        const f32x4 dyv = load4s<TDY>(dy + row * lddy + c);
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

// D = 4L <= 128 (the CvT's stages 1 and 2: D = 64, 128): L lanes per row and 64 / L rows per wave
// (the one-row-per-wave kernel above left 48 / 32 of the 64 lanes idle there).  Same math, the
// row sums over the row's L lanes by xor shuffles, same partial layout (fixed order).
template <int L, typename TDY, bool LP>
__global__ __launch_bounds__(256) void ln_bwd_small_kernel(
    int64_t M, const TDY* __restrict__ dy, int64_t lddy, const float* __restrict__ x, int64_t ldx,
    const float* __restrict__ mean, const float* __restrict__ rstd, const float* __restrict__ gamma,
    const float* __restrict__ dres, int64_t ldres, float* __restrict__ dx, int64_t lddx,
    bf16* __restrict__ dx_lp, int64_t lddx_lp, float* __restrict__ part) {
  constexpr int D = 4 * L, RW = 64 / L;
  __shared__ f32x4 red[4][64 * 3];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane / L, c = (lane % L) * 4;
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  const f32x4 g = *(const f32x4*)(gamma + c);
  f32x4 dg = zero, db = zero, ds = zero;
  for (int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * RW; r0 < M; r0 += (int64_t)gridDim.x * 4 * RW) {
    const int64_t row = r0 + sub;
    const bool ok = row < M;
    float mu = 0.f, rs = 0.f;
    f32x4 xv = zero, dyv = zero, rv = zero;
    if (ok) {
      mu = mean[row];
      rs = rstd[row];
      if (dres) rv = ldg_s((const f32x4*)(dres + row * ldres + c));
      xv = ldg_s((const f32x4*)(x + row * ldx + c));
      dyv = load4s<TDY>(dy + row * lddy + c);
    }
    const f32x4 xh = (xv - mu) * rs;
    const f32x4 gy = dyv * g;
    dg += dyv * xh;
    db += dyv;
    float s1 = gy[0] + gy[1] + gy[2] + gy[3];
    const f32x4 t = gy * xh;
    float s2 = t[0] + t[1] + t[2] + t[3];
#pragma unroll
    for (int o = 1; o < L; o <<= 1) {
      s1 += __shfl_xor(s1, o, 64);
      s2 += __shfl_xor(s2, o, 64);
    }
    const float c1 = s1 / D, c2 = s2 / D;
    if (ok) {
      const f32x4 o = (gy - c1 - xh * c2) * rs + rv;
      ds += o;
      put((f32x4*)(dx + row * lddx + c), o);
      if (LP) store4<bf16>(dx_lp + row * lddx_lp + c, o);
    }
  }
  red[wave][lane] = dg;
  red[wave][64 + lane] = db;
  red[wave][128 + lane] = ds;
  __syncthreads();
  if (threadIdx.x < 3 * L) {
    const int which = threadIdx.x / L, cc = threadIdx.x % L;
    f32x4 acc = zero;
    for (int w = 0; w < 4; ++w)
      for (int q = 0; q < RW; ++q) acc += red[w][which * 64 + q * L + cc];
    *(f32x4*)(part + ((int64_t)which * gridDim.x + blockIdx.x) * D + cc * 4) = acc;
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
  if (ydt == VITMI_BF16X3) {
    hipLaunchKernelGGL((ln_fwd_kernel<NV, SplitX3>), grid, dim3(256), 0, s, M, D, x, ldx, gamma, beta, eps,
                       (SplitX3*)y, ldy, mean, rstd);
    VITMI_STAT((ln_fwd_kernel<NV, SplitX3>), 0, (double)M * D * (4 + 6) + 8.0 * M);
    return;
  }
  if (ydt == VITMI_BF16F8) {
    hipLaunchKernelGGL((ln_fwd_kernel<NV, SplitF8>), grid, dim3(256), 0, s, M, D, x, ldx, gamma, beta, eps,
                       (SplitF8*)y, ldy, mean, rstd);
    VITMI_STAT((ln_fwd_kernel<NV, SplitF8>), 0, (double)M * D * (4 + 4) + 8.0 * M);
    return;
  }
  if (ydt == VITMI_BF16F8W) {
    hipLaunchKernelGGL((ln_fwd_kernel<NV, SplitF8W>), grid, dim3(256), 0, s, M, D, x, ldx, gamma, beta, eps,
                       (SplitF8W*)y, ldy, mean, rstd);
    VITMI_STAT((ln_fwd_kernel<NV, SplitF8W>), 0, (double)M * D * (4 + 3) + 8.0 * M);
    return;
  }
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
  VITMI_CHECK_ARG(y_dtype == VITMI_F32 || y_dtype == VITMI_BF16 || y_dtype == VITMI_BF16X3 || y_dtype == VITMI_BF16F8 ||
                      y_dtype == VITMI_BF16F8W,
                  "layernorm_fwd: y dtype must be VITMI_F32, VITMI_BF16, VITMI_BF16X3, VITMI_BF16F8 or VITMI_BF16F8W");
  VITMI_CHECK_ARG(ldx >= D && ldy >= (y_dtype == VITMI_BF16X3 ? 3LL * D : y_dtype == VITMI_BF16F8 ? 2LL * D
                                      : y_dtype == VITMI_BF16F8W ? 3LL * D / 2 : (int64_t)D),
                  "layernorm_fwd: ldx >= D and ldy >= D (3D for VITMI_BF16X3, 2D for VITMI_BF16F8, 1.5D for "
                  "VITMI_BF16F8W) required");
  VITMI_CHECK_ARG(y_dtype != VITMI_BF16F8 || D % 64 == 0, "layernorm_fwd: VITMI_BF16F8 needs D %% 64 == 0");
  VITMI_CHECK_ARG(y_dtype != VITMI_BF16F8W || D % 128 == 0, "layernorm_fwd: VITMI_BF16F8W needs D %% 128 == 0");
  if (M == 0) return VITMI_OK;
  VITMI_CHECK_ARG(x && gamma && beta && y && mean && rstd, "layernorm_fwd: null pointer");
  hipStream_t s = (hipStream_t)stream;
#ifndef VITMI_LN_FWD_SMALL
#define VITMI_LN_FWD_SMALL 1
#endif
  if (VITMI_LN_FWD_SMALL && (D == 64 || D == 128) && y_dtype != VITMI_BF16X3 && y_dtype != VITMI_BF16F8 &&
      y_dtype != VITMI_BF16F8W) {
    const int rw = 64 / (D / 4);
    const dim3 grid((unsigned)((M + 4 * rw - 1) / (4 * rw)));
    if (D == 64) {
      if (y_dtype == VITMI_BF16)
        hipLaunchKernelGGL((ln_fwd_small_kernel<16, bf16>), grid, dim3(256), 0, s, M, x, ldx, gamma, beta, eps,
                           (bf16*)y, ldy, mean, rstd);
      else
        hipLaunchKernelGGL((ln_fwd_small_kernel<16, float>), grid, dim3(256), 0, s, M, x, ldx, gamma, beta, eps,
                           (float*)y, ldy, mean, rstd);
    } else {
      if (y_dtype == VITMI_BF16)
        hipLaunchKernelGGL((ln_fwd_small_kernel<32, bf16>), grid, dim3(256), 0, s, M, x, ldx, gamma, beta, eps,
                           (bf16*)y, ldy, mean, rstd);
      else
        hipLaunchKernelGGL((ln_fwd_small_kernel<32, float>), grid, dim3(256), 0, s, M, x, ldx, gamma, beta, eps,
                           (float*)y, ldy, mean, rstd);
    }
    VITMI_LAUNCH_CHECK("layernorm_fwd");
    return VITMI_OK;
  }
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
#ifndef VITMI_LN_BWD_SMALL
#define VITMI_LN_BWD_SMALL 1
#endif
  if (VITMI_LN_BWD_SMALL && (D == 64 || D == 128)) {
#define LNS(LL, TD, LPB)                                                                          \
  hipLaunchKernelGGL((ln_bwd_small_kernel<LL, TD, LPB>), dim3(G), dim3(256), 0, s, M, (const TD*)dy, lddy, x, ldx, \
                     mean, rstd, gamma, dres, ldres, dx, lddx, (bf16*)dx_lp, lddx_lp, part)
    const bool bf = dy_dtype == VITMI_BF16, lp = dx_lp != nullptr;
    if (D == 64) {
      if (bf) { if (lp) LNS(16, bf16, true); else LNS(16, bf16, false); }
      else { if (lp) LNS(16, float, true); else LNS(16, float, false); }
    } else {
      if (bf) { if (lp) LNS(32, bf16, true); else LNS(32, bf16, false); }
      else { if (lp) LNS(32, float, true); else LNS(32, float, false); }
    }
#undef LNS
    VITMI_LAUNCH_CHECK("layernorm_bwd");
    if (int rc = fold_rows(part, G, D, D, dgamma, s)) return rc;
    if (int rc = fold_rows(part + (int64_t)G * D, G, D, D, dbeta, s)) return rc;
    return fold_rows(part + 2LL * G * D, G, D, D, dxsum, s);
  }
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
  VITMI_LAUNCH_CHECK("layernorm_bwd");
  // the per-block partials of dgamma (rows 0..G-1), dbeta (G..2G-1), colsum(dx) (2G..3G-1)
  if (int rc = fold_rows(part, G, D, D, dgamma, s)) return rc;
  if (int rc = fold_rows(part + (int64_t)G * D, G, D, D, dbeta, s)) return rc;
  return fold_rows(part + 2LL * G * D, G, D, D, dxsum, s);
}
