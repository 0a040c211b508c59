// cvt.hip — the convolutional pieces of the reference's CvT stages, gfx950.
//
//   * ConvEmbed: layers.Conv2D(embed_dim, kernel=k, strides=s, padding='same') at
//     models/CvT(Par).py:203-212 (k7 s4, k3 s2 in the spec :66-72).  As a GEMM over patches:
//     vitmi_conv_im2col builds [B*Ho*Wo][Kp] patch rows (column order kh, kw, c = the Keras
//     kernel [kh][kw][Cin][Cout] flattened, zero-padded to Kp) with TF's asymmetric 'same'
//     padding; vitmi_conv_col2im is its adjoint (input gradient, a gather over the
//     overlapping windows: deterministic, no atomics).
//   * Projection(method='dw_bn'): layers.DepthwiseConv2D(3, strides=1, 'same', no bias) +
//     layers.BatchNormalization() in training mode (models/CvT(Par).py:92-94,104-106), applied
//     to the spatial tokens of q, k and v (:154-156).  Batch statistics over (B, H, W) per
//     channel, moving statistics updated with `momentum` (Keras 0.99).
//
// Layout: token-major rows [.., C] fp32 (NHWC), channels vectorised by 4.  The spatial tokens
// of image b are rows b*img_stride + row_off + h*W + w, so the cls row of stage 3 (row 0 of
// every image, :146-150) is skipped without a copy.  All kernels are HBM/L2-bound stencils and
// reductions: per-channel partial sums by fixed-channel threads, block-reduced in LDS, finished
// by a second tiny pass in a fixed order (deterministic).
#include "common.h"

namespace vitmi {

struct ConvGeo {
  int B, H, W, C, Ho, Wo, kh, kw, s, pt, pl;
  int64_t ldx;          // floats between input rows
  int64_t img_stride;   // input rows between images
  int64_t row_off;      // first spatial row of an image
};

__device__ __forceinline__ int64_t in_row(const ConvGeo& g, int b, int h, int w) {
  return (int64_t)b * g.img_stride + g.row_off + (int64_t)h * g.W + w;
}

// ---------------------------------------------------------------- im2col / col2im
// patches[r][j], r = (b, oh, ow), j = (i, jj, c) < K = kh*kw*C, zero for j >= K or outside.
template <typename T, int VEC>
__global__ void conv_im2col_kernel(ConvGeo g, const float* __restrict__ x, T* __restrict__ patches, int Kp) {
  const int K = g.kh * g.kw * g.C;
  const int64_t rows = (int64_t)g.B * g.Ho * g.Wo;
  const int64_t per_row = Kp / VEC;
  const int64_t total = rows * per_row;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / per_row;
    const int j = (int)(t - r * per_row) * VEC;
    const int ow = (int)(r % g.Wo);
    const int oh = (int)((r / g.Wo) % g.Ho);
    const int b = (int)(r / ((int64_t)g.Wo * g.Ho));
    float v[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) v[e] = 0.f;
    if (j < K) {
      const int c = j % g.C, tap = j / g.C;
      const int i = tap / g.kw, jj = tap % g.kw;
      const int h = oh * g.s - g.pt + i, w = ow * g.s - g.pl + jj;
      if (h >= 0 && h < g.H && w >= 0 && w < g.W) {
        const float* src = x + in_row(g, b, h, w) * g.ldx + c;
        if constexpr (VEC == 4) {
          const f32x4 q = *(const f32x4*)src;
          v[0] = q[0]; v[1] = q[1]; v[2] = q[2]; v[3] = q[3];
        } else {
          v[0] = *src;
        }
      }
    }
    T* dst = patches + r * Kp + j;
#pragma unroll
    for (int e = 0; e < VEC; ++e) dst[e] = from_f32<T>(v[e]);
  }
}

// dx[b,h,w,c] (+)= sum over the windows (oh, ow, i, jj) that read (h, w) of dpatches.
template <typename T>
__global__ void conv_col2im_kernel(ConvGeo g, const T* __restrict__ dp, int Kp, float* __restrict__ dx,
                                   int accumulate) {
  const int C4 = g.C / 4;
  const int64_t total = (int64_t)g.B * g.H * g.W * C4;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(t % C4) * 4;
    const int64_t p = t / C4;
    const int w = (int)(p % g.W), h = (int)((p / g.W) % g.H), b = (int)(p / ((int64_t)g.W * g.H));
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < g.kh; ++i) {
      const int th = h + g.pt - i;
      if (th < 0 || th % g.s) continue;
      const int oh = th / g.s;
      if (oh >= g.Ho) continue;
      for (int jj = 0; jj < g.kw; ++jj) {
        const int tw = w + g.pl - jj;
        if (tw < 0 || tw % g.s) continue;
        const int ow = tw / g.s;
        if (ow >= g.Wo) continue;
        const T* src = dp + (((int64_t)b * g.Ho + oh) * g.Wo + ow) * Kp + (i * g.kw + jj) * g.C + c;
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] += to_f32(src[e]);
      }
    }
    float* d = dx + in_row(g, b, h, w) * g.ldx + c;
    if (accumulate) acc += *(const f32x4*)d;
    *(f32x4*)d = acc;
  }
}

// ---------------------------------------------------------------- depthwise 3x3 + BatchNorm
// VITMI_DW_ROWS (default 1): the stats / dz / dx passes walk image rows with the 3x3 window in
// registers (the *_rows kernels); 0: one pixel per thread-iteration, 9 tap loads each
#ifndef VITMI_DW_ROWS
#define VITMI_DW_ROWS 1
#endif
// Thread (pixel lane pl, channel group cg) with cg = tid % C4 fixed for the whole grid-stride
// loop: 256 / C4 pixels per block iteration (C4 divides 256).  Pixel indices are 32-bit
// (n = B*H*W < 2^31, checked on the host): one (b, h, w) split per pixel, none per tap.
struct DwGeo {
  int B, H, W, C;
  int64_t ldx, x_img, x_off;   // input rows (LN output; cls row skipped through x_off)
  int64_t ldz;                 // z / dz scratch rows: dense [B*H*W][C]
};

__device__ __forceinline__ void dw_split(const DwGeo& g, uint32_t p, uint32_t& b, int& h, int& w) {
  const uint32_t hw = (uint32_t)g.H * (uint32_t)g.W;
  b = p / hw;
  const uint32_t r = p - b * hw;
  h = (int)(r / (uint32_t)g.W);
  w = (int)(r - (uint32_t)h * (uint32_t)g.W);
}

// first row of image b in a [.., ld] row buffer with images every img rows after off
__device__ __forceinline__ int64_t img_row0(uint32_t b, int64_t img, int64_t off) { return (int64_t)b * img + off; }

// z = dwconv3x3(x) (same padding) -> z scratch; per-block partial sum / sum of squares.
__global__ __launch_bounds__(256) void dw_fwd_stats_kernel(DwGeo g, const float* __restrict__ x,
                                                           const float* __restrict__ wt,  // [3][3][C]
                                                           float* __restrict__ z, float* __restrict__ part) {
  __shared__ f32x4 red[2][256];
  const int C4 = g.C / 4, cg = threadIdx.x % C4, lanes = 256 / C4, pl = threadIdx.x / C4;
  const int c = cg * 4;
  const uint32_t n = (uint32_t)g.B * g.H * g.W;
  f32x4 wv[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) wv[k] = *(const f32x4*)(wt + k * g.C + c);
  f32x4 s1 = {0.f, 0.f, 0.f, 0.f}, s2 = {0.f, 0.f, 0.f, 0.f};
  for (uint32_t p = blockIdx.x * lanes + pl; p < n; p += gridDim.x * lanes) {
    uint32_t b;
    int h, w;
    dw_split(g, p, b, h, w);
    const float* xb = x + img_row0(b, g.x_img, g.x_off) * g.ldx + c;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int hh = h + i - 1;
      if (hh < 0 || hh >= g.H) continue;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int ww = w + j - 1;
        if (ww < 0 || ww >= g.W) continue;
        acc += wv[i * 3 + j] * *(const f32x4*)(xb + (int64_t)(hh * g.W + ww) * g.ldx);
      }
    }
    *(f32x4*)(z + (int64_t)p * g.ldz + c) = acc;
    s1 += acc;
    s2 += acc * acc;
  }
  red[0][threadIdx.x] = s1;
  red[1][threadIdx.x] = s2;
  __syncthreads();
  if (pl == 0) {
    for (int l = 1; l < lanes; ++l) {
      s1 += red[0][l * C4 + cg];
      s2 += red[1][l * C4 + cg];
    }
    *(f32x4*)(part + (int64_t)blockIdx.x * 2 * g.C + c) = s1;
    *(f32x4*)(part + (int64_t)blockIdx.x * 2 * g.C + g.C + c) = s2;
  }
}

// The same pass walking image rows: thread (row b*H + h, channel group cg) runs along w with the
// 3x3 window in registers (3 new taps per pixel instead of 9, no per-pixel index divisions).
// Taps are summed in the same (i, j) order as dw_fwd_stats_kernel (out-of-image taps add 0), so z
// is identical; the per-block statistics partials follow this kernel's own fixed order.
__global__ __launch_bounds__(256) void dw_fwd_stats_rows_kernel(DwGeo g, const float* __restrict__ x,
                                                                const float* __restrict__ wt,  // [3][3][C]
                                                                float* __restrict__ z, float* __restrict__ part) {
  __shared__ f32x4 red[2][256];
  const int C4 = g.C / 4, cg = threadIdx.x % C4, lanes = 256 / C4, pl = threadIdx.x / C4;
  const int c = cg * 4;
  const uint32_t rows = (uint32_t)g.B * g.H;
  f32x4 wv[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) wv[k] = *(const f32x4*)(wt + k * g.C + c);
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  f32x4 s1 = zero, s2 = zero;
  for (uint32_t rw = blockIdx.x * lanes + pl; rw < rows; rw += gridDim.x * lanes) {
    const uint32_t b = rw / (uint32_t)g.H;
    const int h = (int)(rw - b * (uint32_t)g.H);
    const float* xb = x + img_row0(b, g.x_img, g.x_off) * g.ldx + c;
    const float* xr[3];
    bool ok[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int hh = h + i - 1;
      ok[i] = hh >= 0 && hh < g.H;
      xr[i] = xb + (int64_t)(ok[i] ? hh : 0) * g.W * g.ldx;
    }
    auto tap = [&](int i, int ww) -> f32x4 {
      return ok[i] && ww < g.W ? *(const f32x4*)(xr[i] + (int64_t)ww * g.ldx) : zero;
    };
    f32x4 L[3], M[3], R[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) { L[i] = zero; M[i] = tap(i, 0); R[i] = tap(i, 1); }
    float* zr = z + (int64_t)rw * g.W * g.ldz + c;
    for (int w = 0; w < g.W; ++w) {
      f32x4 nx[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) nx[i] = tap(i, w + 2);   // next column, in flight under the FMAs
      f32x4 acc = zero;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        if (!ok[i]) continue;
        if (w > 0) acc += wv[i * 3 + 0] * L[i];
        acc += wv[i * 3 + 1] * M[i];
        if (w + 1 < g.W) acc += wv[i * 3 + 2] * R[i];
      }
      *(f32x4*)(zr + (int64_t)w * g.ldz) = acc;
      s1 += acc;
      s2 += acc * acc;
#pragma unroll
      for (int i = 0; i < 3; ++i) { L[i] = M[i]; M[i] = R[i]; R[i] = nx[i]; }
    }
  }
  red[0][threadIdx.x] = s1;
  red[1][threadIdx.x] = s2;
  __syncthreads();
  if (pl == 0) {
    for (int l = 1; l < lanes; ++l) {
      s1 += red[0][l * C4 + cg];
      s2 += red[1][l * C4 + cg];
    }
    *(f32x4*)(part + (int64_t)blockIdx.x * 2 * g.C + c) = s1;
    *(f32x4*)(part + (int64_t)blockIdx.x * 2 * g.C + g.C + c) = s2;
  }
}

// Fixed-order fp64 sum over the G rows of column col of part[G][ld] by a 1024-thread block laid
// out as 16 columns x 64 row groups (LDS tree in a fixed order: deterministic).  Every thread
// of the block must call it; the result is valid in all threads of the column.
constexpr int RED_COLS = 16, RED_ROWS = 64;
__device__ __forceinline__ double block_colsum(const float* __restrict__ part, int G, int64_t ld, int col,
                                               bool valid, double* red) {
  const int cl = threadIdx.x % RED_COLS, rg = threadIdx.x / RED_COLS;
  double s = 0.0;
  if (valid) {
#pragma unroll 4
    for (int b = rg; b < G; b += RED_ROWS) s += part[(int64_t)b * ld + col];
  }
  red[rg * RED_COLS + cl] = s;
  __syncthreads();
  for (int st = RED_ROWS / 2; st > 0; st >>= 1) {
    if (rg < st) red[rg * RED_COLS + cl] += red[(rg + st) * RED_COLS + cl];
    __syncthreads();
  }
  const double r = red[cl];
  __syncthreads();
  return r;
}

// Fold the G block partials into mean / rstd; update the moving statistics.
__global__ __launch_bounds__(1024) void bn_finalize_kernel(const float* __restrict__ part, int G, int C, int64_t n,
                                                           float eps, float momentum, float* __restrict__ mean,
                                                           float* __restrict__ rstd, float* __restrict__ run_mean,
                                                           float* __restrict__ run_var, int training) {
  __shared__ double red[RED_ROWS * RED_COLS];
  const int c = blockIdx.x * RED_COLS + threadIdx.x % RED_COLS;
  const bool ok = c < C;
  const double s1 = block_colsum(part, G, 2 * C, c, training && ok, red);
  const double s2 = block_colsum(part, G, 2 * C, C + c, training && ok, red);
  if (threadIdx.x >= RED_COLS || !ok) return;
  if (!training) {   // inference: the moving statistics
    mean[c] = run_mean[c];
    rstd[c] = (float)(1.0 / sqrt((double)run_var[c] + (double)eps));
    return;
  }
  const double mu = s1 / (double)n;
  double var = s2 / (double)n - mu * mu;
  if (var < 0.0) var = 0.0;
  mean[c] = (float)mu;
  rstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (run_mean) run_mean[c] = momentum * run_mean[c] + (1.f - momentum) * (float)mu;
  // the moving variance takes the unbiased batch variance (Bessel's n/(n-1)), as Keras'
  // fused BatchNormalization on NHWC tensors and torch's BatchNorm2d (MS_CvT) both do
  const double var_u = n > 1 ? var * (double)n / (double)(n - 1) : var;
  if (run_var) run_var[c] = momentum * run_var[c] + (1.f - momentum) * (float)var_u;
}

// y = (z - mean) * rstd * gamma + beta  -> rows b*y_img + y_off + hw of y (out dtype)
template <typename TY>
__global__ void bn_apply_kernel(DwGeo g, const float* __restrict__ z, const float* __restrict__ mean,
                                const float* __restrict__ rstd, const float* __restrict__ gamma,
                                const float* __restrict__ beta, TY* __restrict__ y, int64_t ldy, int64_t y_img,
                                int64_t y_off) {
  const uint32_t C4 = g.C / 4, hw = (uint32_t)g.H * g.W;
  const uint32_t total = (uint32_t)g.B * hw * C4;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int c = (int)(t % C4) * 4;
    const uint32_t p = t / C4, b = p / hw;
    const f32x4 zv = *(const f32x4*)(z + (int64_t)p * g.ldz + c);
    const f32x4 o = (zv - *(const f32x4*)(mean + c)) * *(const f32x4*)(rstd + c) * *(const f32x4*)(gamma + c) +
                    *(const f32x4*)(beta + c);
    TY* d = y + (img_row0(b, y_img, y_off) + (p - b * hw)) * ldy + c;
#pragma unroll
    for (int e = 0; e < 4; ++e) d[e] = from_f32<TY>(o[e]);
  }
}

// backward statistics: sum dy and sum dy * zhat per channel (dy rows like y's).
template <typename TD>
__global__ __launch_bounds__(256) void bn_bwd_stats_kernel(DwGeo g, const TD* __restrict__ dy, int64_t lddy,
                                                           int64_t dy_img, int64_t dy_off,
                                                           const float* __restrict__ z,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ rstd,
                                                           float* __restrict__ part) {
  __shared__ f32x4 red[2][256];
  const int C4 = g.C / 4, cg = threadIdx.x % C4, lanes = 256 / C4, pl = threadIdx.x / C4;
  const int c = cg * 4;
  const uint32_t hw = (uint32_t)g.H * g.W, n = (uint32_t)g.B * hw;
  const f32x4 mu = *(const f32x4*)(mean + c), rs = *(const f32x4*)(rstd + c);
  f32x4 s1 = {0.f, 0.f, 0.f, 0.f}, s2 = {0.f, 0.f, 0.f, 0.f};
  for (uint32_t p = blockIdx.x * lanes + pl; p < n; p += gridDim.x * lanes) {
    const uint32_t b = p / hw;
    const TD* src = dy + (img_row0(b, dy_img, dy_off) + (p - b * hw)) * lddy + c;
    f32x4 d;
#pragma unroll
    for (int e = 0; e < 4; ++e) d[e] = to_f32(src[e]);
    const f32x4 zh = (*(const f32x4*)(z + (int64_t)p * g.ldz + c) - mu) * rs;
    s1 += d;
    s2 += d * zh;
  }
  red[0][threadIdx.x] = s1;
  red[1][threadIdx.x] = s2;
  __syncthreads();
  if (pl == 0) {
    for (int l = 1; l < lanes; ++l) {
      s1 += red[0][l * C4 + cg];
      s2 += red[1][l * C4 + cg];
    }
    *(f32x4*)(part + (int64_t)blockIdx.x * 2 * g.C + c) = s1;
    *(f32x4*)(part + (int64_t)blockIdx.x * 2 * g.C + g.C + c) = s2;
  }
}

// sums -> dgamma/dbeta (+=), and the per-channel constants of dz: k1 = mean(dy), k2 = mean(dy zhat)
__global__ __launch_bounds__(1024) void bn_bwd_finalize_kernel(const float* __restrict__ part, int G, int C,
                                                               int64_t n, float* __restrict__ dgamma,
                                                               float* __restrict__ dbeta, float* __restrict__ kk) {
  __shared__ double red[RED_ROWS * RED_COLS];
  const int c = blockIdx.x * RED_COLS + threadIdx.x % RED_COLS;
  const bool ok = c < C;
  const double s1 = block_colsum(part, G, 2 * C, c, ok, red);
  const double s2 = block_colsum(part, G, 2 * C, C + c, ok, red);
  if (threadIdx.x >= RED_COLS || !ok) return;
  if (dgamma) dgamma[c] += (float)s2;
  if (dbeta) dbeta[c] += (float)s1;
  kk[c] = (float)(s1 / (double)n);
  kk[C + c] = (float)(s2 / (double)n);
}

// dz = gamma * rstd * (dy - k1 - zhat * k2) -> scratch; per-block partials of
// dW[i][j][c] = sum_p dz[p][c] * x[p + (i-1, j-1)][c].
template <typename TD>
__global__ __launch_bounds__(256) void dw_bwd_dz_kernel(DwGeo g, const TD* __restrict__ dy, int64_t lddy,
                                                        int64_t dy_img, int64_t dy_off,
                                                        const float* __restrict__ z, const float* __restrict__ x,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ rstd,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ kk, float* __restrict__ dz,
                                                        float* __restrict__ part) {
  __shared__ f32x4 red[256];
  const int C4 = g.C / 4, cg = threadIdx.x % C4, lanes = 256 / C4, pl = threadIdx.x / C4;
  const int c = cg * 4;
  const uint32_t n = (uint32_t)g.B * g.H * g.W;
  const f32x4 mu = *(const f32x4*)(mean + c), rs = *(const f32x4*)(rstd + c);
  const f32x4 gr = *(const f32x4*)(gamma + c) * rs;
  const f32x4 k1 = *(const f32x4*)(kk + c), k2 = *(const f32x4*)(kk + g.C + c);
  f32x4 dw[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) dw[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (uint32_t p = blockIdx.x * lanes + pl; p < n; p += gridDim.x * lanes) {
    uint32_t b;
    int h, w;
    dw_split(g, p, b, h, w);
    const int hw_i = h * g.W + w;
    const TD* src = dy + (img_row0(b, dy_img, dy_off) + hw_i) * lddy + c;
    f32x4 d;
#pragma unroll
    for (int e = 0; e < 4; ++e) d[e] = to_f32(src[e]);
    const f32x4 zh = (*(const f32x4*)(z + (int64_t)p * g.ldz + c) - mu) * rs;
    const f32x4 dzv = gr * (d - k1 - zh * k2);
    *(f32x4*)(dz + (int64_t)p * g.ldz + c) = dzv;
    const float* xb = x + img_row0(b, g.x_img, g.x_off) * g.ldx + c;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int hh = h + i - 1;
      if (hh < 0 || hh >= g.H) continue;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int ww = w + j - 1;
        if (ww < 0 || ww >= g.W) continue;
        dw[i * 3 + j] += dzv * *(const f32x4*)(xb + (int64_t)(hh * g.W + ww) * g.ldx);
      }
    }
  }
  for (int k = 0; k < 9; ++k) {
    __syncthreads();
    red[threadIdx.x] = dw[k];
    __syncthreads();
    if (pl == 0) {
      f32x4 s = dw[k];
      for (int l = 1; l < lanes; ++l) s += red[l * C4 + cg];
      *(f32x4*)(part + ((int64_t)blockIdx.x * 9 + k) * g.C + c) = s;
    }
  }
}

// The same pass walking image rows (see dw_fwd_stats_rows_kernel): the x window slides along w,
// so each pixel loads dy, z and 3 new x taps.  dz is identical; the weight-gradient partials
// follow this kernel's fixed order.
template <typename TD>
__global__ __launch_bounds__(256) void dw_bwd_dz_rows_kernel(DwGeo g, const TD* __restrict__ dy, int64_t lddy,
                                                             int64_t dy_img, int64_t dy_off,
                                                             const float* __restrict__ z, const float* __restrict__ x,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ rstd,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ kk, float* __restrict__ dz,
                                                             float* __restrict__ part) {
  __shared__ f32x4 red[256];
  const int C4 = g.C / 4, cg = threadIdx.x % C4, lanes = 256 / C4, pl = threadIdx.x / C4;
  const int c = cg * 4;
  const uint32_t rows = (uint32_t)g.B * g.H;
  const f32x4 mu = *(const f32x4*)(mean + c), rs = *(const f32x4*)(rstd + c);
  const f32x4 gr = *(const f32x4*)(gamma + c) * rs;
  const f32x4 k1 = *(const f32x4*)(kk + c), k2 = *(const f32x4*)(kk + g.C + c);
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  f32x4 dw[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) dw[k] = zero;
  for (uint32_t rw = blockIdx.x * lanes + pl; rw < rows; rw += gridDim.x * lanes) {
    const uint32_t b = rw / (uint32_t)g.H;
    const int h = (int)(rw - b * (uint32_t)g.H);
    const float* xb = x + img_row0(b, g.x_img, g.x_off) * g.ldx + c;
    const float* xr[3];
    bool ok[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int hh = h + i - 1;
      ok[i] = hh >= 0 && hh < g.H;
      xr[i] = xb + (int64_t)(ok[i] ? hh : 0) * g.W * g.ldx;
    }
    auto tap = [&](int i, int ww) -> f32x4 {
      return ok[i] && ww < g.W ? *(const f32x4*)(xr[i] + (int64_t)ww * g.ldx) : zero;
    };
    f32x4 L[3], M[3], R[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) { L[i] = zero; M[i] = tap(i, 0); R[i] = tap(i, 1); }
    const TD* dyr = dy + (img_row0(b, dy_img, dy_off) + (int64_t)h * g.W) * lddy + c;
    const float* zr = z + (int64_t)rw * g.W * g.ldz + c;
    float* dzr = dz + (int64_t)rw * g.W * g.ldz + c;
    for (int w = 0; w < g.W; ++w) {
      f32x4 nx[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) nx[i] = tap(i, w + 2);
      f32x4 d;
      const TD* src = dyr + (int64_t)w * lddy;
#pragma unroll
      for (int e = 0; e < 4; ++e) d[e] = to_f32(src[e]);
      const f32x4 zh = (*(const f32x4*)(zr + (int64_t)w * g.ldz) - mu) * rs;
      const f32x4 dzv = gr * (d - k1 - zh * k2);
      *(f32x4*)(dzr + (int64_t)w * g.ldz) = dzv;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        if (!ok[i]) continue;
        if (w > 0) dw[i * 3 + 0] += dzv * L[i];
        dw[i * 3 + 1] += dzv * M[i];
        if (w + 1 < g.W) dw[i * 3 + 2] += dzv * R[i];
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) { L[i] = M[i]; M[i] = R[i]; R[i] = nx[i]; }
    }
  }
  for (int k = 0; k < 9; ++k) {
    __syncthreads();
    red[threadIdx.x] = dw[k];
    __syncthreads();
    if (pl == 0) {
      f32x4 s = dw[k];
      for (int l = 1; l < lanes; ++l) s += red[l * C4 + cg];
      *(f32x4*)(part + ((int64_t)blockIdx.x * 9 + k) * g.C + c) = s;
    }
  }
}

// dx[p] += sum_{i,j} w[i][j] * dz[p - (i-1, j-1)] walking image rows: thread (row, channel group)
// slides a 3x3 dz window along w (3 new loads per pixel); same (i, j) order as dw_bwd_dx_kernel,
// so dx is identical.
__global__ __launch_bounds__(256) void dw_bwd_dx_rows_kernel(DwGeo g, const float* __restrict__ dz,
                                                             const float* __restrict__ wt, float* __restrict__ dx) {
  const uint32_t C4 = g.C / 4;
  const uint32_t total = (uint32_t)g.B * g.H * C4;
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int c = (int)(t % C4) * 4;
    const uint32_t rw = t / C4;
    const uint32_t b = rw / (uint32_t)g.H;
    const int h = (int)(rw - b * (uint32_t)g.H);
    f32x4 wv[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) wv[k] = *(const f32x4*)(wt + k * g.C + c);
    // dz rows h + 1 (i = 0), h (i = 1), h - 1 (i = 2) of image b
    const float* zb = dz + (int64_t)b * g.H * g.W * g.ldz + c;
    const float* zr[3];
    bool ok[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int hh = h - i + 1;
      ok[i] = hh >= 0 && hh < g.H;
      zr[i] = zb + (int64_t)(ok[i] ? hh : 0) * g.W * g.ldz;
    }
    auto tap = [&](int i, int ww) -> f32x4 {
      return ok[i] && ww < g.W ? *(const f32x4*)(zr[i] + (int64_t)ww * g.ldz) : zero;
    };
    // window: P = dz(w - 1), Q = dz(w), S = dz(w + 1); tap j reads column w - j + 1
    f32x4 P[3], Q[3], S[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) { P[i] = zero; Q[i] = tap(i, 0); S[i] = tap(i, 1); }
    float* dr = dx + (img_row0(b, g.x_img, g.x_off) + (int64_t)h * g.W) * g.ldx + c;
    for (int w = 0; w < g.W; ++w) {
      f32x4 nx[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) nx[i] = tap(i, w + 2);
      f32x4 acc = zero;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        if (!ok[i]) continue;
        if (w + 1 < g.W) acc += wv[i * 3 + 0] * S[i];
        acc += wv[i * 3 + 1] * Q[i];
        if (w > 0) acc += wv[i * 3 + 2] * P[i];
      }
      float* d = dr + (int64_t)w * g.ldx;
      *(f32x4*)d = *(const f32x4*)d + acc;
#pragma unroll
      for (int i = 0; i < 3; ++i) { P[i] = Q[i]; Q[i] = S[i]; S[i] = nx[i]; }
    }
  }
}

// dW[k][c] += sum over blocks of the partials (fixed order)
__global__ __launch_bounds__(1024) void dw_wgrad_finalize_kernel(const float* __restrict__ part, int G, int C,
                                                                 float* __restrict__ dwt) {
  __shared__ double red[RED_ROWS * RED_COLS];
  const int e = blockIdx.x * RED_COLS + threadIdx.x % RED_COLS;
  const bool ok = e < 9 * C;
  const double s = block_colsum(part, G, 9 * C, e, ok, red);
  if (threadIdx.x < RED_COLS && ok) dwt[e] += (float)s;
}

// dx[p] += sum_{i,j} w[i][j] * dz[p - (i-1, j-1)]   (rows of dx like x's)
__global__ void dw_bwd_dx_kernel(DwGeo g, const float* __restrict__ dz, const float* __restrict__ wt,
                                 float* __restrict__ dx) {
  const uint32_t C4 = g.C / 4;
  const uint32_t total = (uint32_t)g.B * g.H * g.W * C4;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int c = (int)(t % C4) * 4;
    const uint32_t p = t / C4;
    uint32_t b;
    int h, w;
    dw_split(g, p, b, h, w);
    const float* zb = dz + ((int64_t)p - (h * g.W + w)) * g.ldz + c;   // (b, 0, 0)
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int hh = h - i + 1;
      if (hh < 0 || hh >= g.H) continue;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int ww = w - j + 1;
        if (ww < 0 || ww >= g.W) continue;
        acc += *(const f32x4*)(wt + (i * 3 + j) * g.C + c) * *(const f32x4*)(zb + (int64_t)(hh * g.W + ww) * g.ldz);
      }
    }
    float* d = dx + (img_row0(b, g.x_img, g.x_off) + h * g.W + w) * g.ldx + c;
    *(f32x4*)d = *(const f32x4*)d + acc;
  }
}

static unsigned grid_of(int64_t work, int per_block = 256, int cap = 4096) {
  int64_t gsz = (work + per_block - 1) / per_block;
  if (gsz > cap) gsz = cap;
  return (unsigned)(gsz < 1 ? 1 : gsz);
}

static int dw_blocks(int64_t n, int C) {
  const int lanes = 256 / (C / 4);
  int64_t gsz = (n + lanes * 8 - 1) / (lanes * 8);   // >= 8 pixels per thread
  if (gsz > 1024) gsz = 1024;
  return (int)(gsz < 1 ? 1 : gsz);
}

static bool dw_channels_ok(int C) { return C >= 4 && C % 4 == 0 && 1024 % C == 0; }

// TF 'same': Ho = ceil(H / s), pad_total = max((Ho - 1) s + k - H, 0), pad_before = total / 2
static void same_pad(int H, int k, int s, int& Ho, int& pt) {
  Ho = (H + s - 1) / s;
  int tot = (Ho - 1) * s + k - H;
  if (tot < 0) tot = 0;
  pt = tot / 2;
}

}  // namespace vitmi

using namespace vitmi;

extern "C" int vitmi_conv_same_geometry(int H, int W, int kh, int kw, int s, int* Ho, int* Wo, int* pad_top,
                                        int* pad_left) {
  VITMI_CHECK_ARG(H > 0 && W > 0 && kh > 0 && kw > 0 && s > 0, "conv_same_geometry: bad sizes");
  int ho, wo, pt, pl;
  same_pad(H, kh, s, ho, pt);
  same_pad(W, kw, s, wo, pl);
  if (Ho) *Ho = ho;
  if (Wo) *Wo = wo;
  if (pad_top) *pad_top = pt;
  if (pad_left) *pad_left = pl;
  return VITMI_OK;
}

static int make_geo(ConvGeo& g, int B, int H, int W, int C, int kh, int kw, int s, int pt, int pl, int Ho, int Wo,
                    int64_t ldx, int64_t img_stride, int64_t row_off) {
  VITMI_CHECK_ARG(B > 0 && H > 0 && W > 0 && C > 0 && kh > 0 && kw > 0 && s > 0, "conv: bad sizes");
  VITMI_CHECK_ARG(pt >= 0 && pl >= 0 && pt < kh && pl < kw && Ho > 0 && Wo > 0, "conv: bad padding / output size");
  VITMI_CHECK_ARG((Ho - 1) * s - pt < H && (Wo - 1) * s - pl < W, "conv: output window outside the input");
  VITMI_CHECK_ARG(ldx >= C && img_stride >= (int64_t)H * W + row_off && row_off >= 0, "conv: bad row layout");
  g.B = B; g.H = H; g.W = W; g.C = C; g.kh = kh; g.kw = kw; g.s = s;
  g.Ho = Ho; g.Wo = Wo; g.pt = pt; g.pl = pl;
  g.ldx = ldx; g.img_stride = img_stride; g.row_off = row_off;
  return VITMI_OK;
}

extern "C" int vitmi_conv_im2col(int dtype, int B, int H, int W, int C, int kh, int kw, int s, int pad_top,
                                 int pad_left, int Ho, int Wo, const float* x, int64_t ldx, int64_t img_stride,
                                 int64_t row_off, void* patches, int Kp, vitmi_stream_t stream) {
  ConvGeo g;
  if (int rc = make_geo(g, B, H, W, C, kh, kw, s, pad_top, pad_left, Ho, Wo, ldx, img_stride, row_off)) return rc;
  VITMI_CHECK_ARG(x && patches, "conv_im2col: null pointer");
  VITMI_CHECK_ARG(Kp >= kh * kw * C, "conv_im2col: Kp < kh*kw*C");
  VITMI_CHECK_ARG(dtype == VITMI_BF16 || dtype == VITMI_F32, "conv_im2col: bad dtype");
  const bool vec = C % 4 == 0 && Kp % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)x % 16) == 0;
  const int64_t work = (int64_t)B * g.Ho * g.Wo * Kp / (vec ? 4 : 1);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VITMI_BF16) {
    if (vec) hipLaunchKernelGGL((conv_im2col_kernel<bf16, 4>), dim3(grid_of(work)), dim3(256), 0, st, g, x, (bf16*)patches, Kp);
    else hipLaunchKernelGGL((conv_im2col_kernel<bf16, 1>), dim3(grid_of(work)), dim3(256), 0, st, g, x, (bf16*)patches, Kp);
  } else {
    if (vec) hipLaunchKernelGGL((conv_im2col_kernel<float, 4>), dim3(grid_of(work)), dim3(256), 0, st, g, x, (float*)patches, Kp);
    else hipLaunchKernelGGL((conv_im2col_kernel<float, 1>), dim3(grid_of(work)), dim3(256), 0, st, g, x, (float*)patches, Kp);
  }
  VITMI_LAUNCH_CHECK("conv_im2col");
  return VITMI_OK;
}

extern "C" int vitmi_conv_col2im(int dtype, int B, int H, int W, int C, int kh, int kw, int s, int pad_top,
                                 int pad_left, int Ho, int Wo, const void* dpatches, int Kp, float* dx, int64_t ldx,
                                 int64_t img_stride, int64_t row_off, int accumulate, vitmi_stream_t stream) {
  ConvGeo g;
  if (int rc = make_geo(g, B, H, W, C, kh, kw, s, pad_top, pad_left, Ho, Wo, ldx, img_stride, row_off)) return rc;
  VITMI_CHECK_ARG(dpatches && dx, "conv_col2im: null pointer");
  VITMI_CHECK_ARG(C % 4 == 0 && ldx % 4 == 0 && Kp >= kh * kw * C, "conv_col2im: C %% 4 == 0 required");
  const int64_t work = (int64_t)B * H * W * (C / 4);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VITMI_BF16)
    hipLaunchKernelGGL(conv_col2im_kernel<bf16>, dim3(grid_of(work)), dim3(256), 0, st, g, (const bf16*)dpatches, Kp,
                       dx, accumulate);
  else
    hipLaunchKernelGGL(conv_col2im_kernel<float>, dim3(grid_of(work)), dim3(256), 0, st, g, (const float*)dpatches,
                       Kp, dx, accumulate);
  VITMI_LAUNCH_CHECK("conv_col2im");
  return VITMI_OK;
}

static int make_dw(DwGeo& g, int B, int H, int W, int C, int64_t ldx, int64_t x_img, int64_t x_off) {
  VITMI_CHECK_ARG(B > 0 && H > 0 && W > 0 && (int64_t)B * H * W * (C / 4) < (1LL << 31), "dwconv: bad sizes");
  VITMI_CHECK_ARG(dw_channels_ok(C), "dwconv: C must be a multiple of 4 dividing 1024 (got %d)", C);
  VITMI_CHECK_ARG(ldx % 4 == 0 && ldx >= C && x_img >= (int64_t)H * W + x_off && x_off >= 0, "dwconv: bad row layout");
  g.B = B; g.H = H; g.W = W; g.C = C; g.ldx = ldx; g.x_img = x_img; g.x_off = x_off; g.ldz = C;
  return VITMI_OK;
}

extern "C" size_t vitmi_dwconv_bn_workspace_size(int B, int H, int W, int C) {
  const int64_t n = (int64_t)B * H * W;
  const int G = dw_blocks(n, C);
  // partials (max of the stats pass and the 9-tap weight-grad pass) + dz scratch + k1/k2
  return (size_t)G * 9 * C * sizeof(float) + (size_t)n * C * sizeof(float) + 2 * C * sizeof(float);
}

extern "C" int vitmi_dwconv_bn_fwd(int B, int H, int W, int C, const float* x, int64_t ldx, int64_t x_img,
                                   int64_t x_off, const float* wt, const float* gamma, const float* beta,
                                   float eps, float momentum, int training, float* run_mean, float* run_var,
                                   float* z, float* mean, float* rstd, void* y, int y_dtype, int64_t ldy,
                                   int64_t y_img, int64_t y_off, void* workspace, size_t ws_bytes,
                                   vitmi_stream_t stream) {
  DwGeo g;
  if (int rc = make_dw(g, B, H, W, C, ldx, x_img, x_off)) return rc;
  VITMI_CHECK_ARG(x && wt && gamma && beta && z && mean && rstd && y, "dwconv_bn_fwd: null pointer");
  VITMI_CHECK_ARG(workspace && ws_bytes >= vitmi_dwconv_bn_workspace_size(B, H, W, C), "dwconv_bn_fwd: workspace");
  VITMI_CHECK_ARG(ldy % 4 == 0 && y_img >= (int64_t)H * W + y_off, "dwconv_bn_fwd: bad output layout");
  VITMI_CHECK_ARG(training || (run_mean && run_var), "dwconv_bn_fwd: inference needs the moving statistics");
  hipStream_t st = (hipStream_t)stream;
  const int64_t n = (int64_t)B * H * W;
  float* part = (float*)workspace;
#if VITMI_DW_ROWS
  // row-walking stats pass: one thread per (image row, channel group), at most dw_blocks blocks
  // (the workspace's partial rows)
  int G = (int)(((int64_t)B * H * (C / 4) + 255) / 256);
  if (G > dw_blocks(n, C)) G = dw_blocks(n, C);
  hipLaunchKernelGGL(dw_fwd_stats_rows_kernel, dim3(G), dim3(256), 0, st, g, x, wt, z, part);
#else
  const int G = dw_blocks(n, C);
  hipLaunchKernelGGL(dw_fwd_stats_kernel, dim3(G), dim3(256), 0, st, g, x, wt, z, part);
#endif
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + RED_COLS - 1) / RED_COLS), dim3(1024), 0, st, (const float*)part, G, C, n, eps,
                     momentum, mean, rstd, run_mean, run_var, training);
  const int64_t work = n * (C / 4);
  if (y_dtype == VITMI_BF16)
    hipLaunchKernelGGL(bn_apply_kernel<bf16>, dim3(grid_of(work)), dim3(256), 0, st, g, (const float*)z,
                       (const float*)mean, (const float*)rstd, gamma, beta, (bf16*)y, ldy, y_img, y_off);
  else
    hipLaunchKernelGGL(bn_apply_kernel<float>, dim3(grid_of(work)), dim3(256), 0, st, g, (const float*)z,
                       (const float*)mean, (const float*)rstd, gamma, beta, (float*)y, ldy, y_img, y_off);
  VITMI_LAUNCH_CHECK("dwconv_bn_fwd");
  return VITMI_OK;
}

extern "C" int vitmi_dwconv_bn_bwd(int B, int H, int W, int C, const void* dy, int dy_dtype, int64_t lddy,
                                   int64_t dy_img, int64_t dy_off, const float* x, int64_t ldx, int64_t x_img,
                                   int64_t x_off, const float* wt, const float* gamma, const float* z,
                                   const float* mean, const float* rstd, float* dx, float* dwt, float* dgamma,
                                   float* dbeta, void* workspace, size_t ws_bytes, vitmi_stream_t stream) {
  DwGeo g;
  if (int rc = make_dw(g, B, H, W, C, ldx, x_img, x_off)) return rc;
  VITMI_CHECK_ARG(dy && x && wt && gamma && z && mean && rstd && dx && dwt, "dwconv_bn_bwd: null pointer");
  VITMI_CHECK_ARG(workspace && ws_bytes >= vitmi_dwconv_bn_workspace_size(B, H, W, C), "dwconv_bn_bwd: workspace");
  VITMI_CHECK_ARG(lddy % 4 == 0 && dy_img >= (int64_t)H * W + dy_off, "dwconv_bn_bwd: bad dy layout");
  hipStream_t st = (hipStream_t)stream;
  const int64_t n = (int64_t)B * H * W;
  const int G = dw_blocks(n, C);
  float* part = (float*)workspace;
  float* dz = part + (size_t)G * 9 * C;
  float* kk = dz + (size_t)n * C;
  if (dy_dtype == VITMI_BF16) {
    hipLaunchKernelGGL(bn_bwd_stats_kernel<bf16>, dim3(G), dim3(256), 0, st, g, (const bf16*)dy, lddy, dy_img, dy_off,
                       z, mean, rstd, part);
  } else {
    hipLaunchKernelGGL(bn_bwd_stats_kernel<float>, dim3(G), dim3(256), 0, st, g, (const float*)dy, lddy, dy_img,
                       dy_off, z, mean, rstd, part);
  }
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + RED_COLS - 1) / RED_COLS), dim3(1024), 0, st, (const float*)part, G, C, n,
                     dgamma, dbeta, kk);
#if VITMI_DW_ROWS
  int Gw = (int)(((int64_t)B * H * (C / 4) + 255) / 256);
  if (Gw > G) Gw = G;
  if (dy_dtype == VITMI_BF16)
    hipLaunchKernelGGL(dw_bwd_dz_rows_kernel<bf16>, dim3(Gw), dim3(256), 0, st, g, (const bf16*)dy, lddy, dy_img, dy_off,
                       z, x, mean, rstd, gamma, (const float*)kk, dz, part);
  else
    hipLaunchKernelGGL(dw_bwd_dz_rows_kernel<float>, dim3(Gw), dim3(256), 0, st, g, (const float*)dy, lddy, dy_img,
                       dy_off, z, x, mean, rstd, gamma, (const float*)kk, dz, part);
  hipLaunchKernelGGL(dw_wgrad_finalize_kernel, dim3((9 * C + RED_COLS - 1) / RED_COLS), dim3(1024), 0, st, (const float*)part, Gw, C,
                     dwt);
  hipLaunchKernelGGL(dw_bwd_dx_rows_kernel, dim3(grid_of((int64_t)B * H * (C / 4))), dim3(256), 0, st, g, (const float*)dz,
                     wt, dx);
#else
  if (dy_dtype == VITMI_BF16)
    hipLaunchKernelGGL(dw_bwd_dz_kernel<bf16>, dim3(G), dim3(256), 0, st, g, (const bf16*)dy, lddy, dy_img, dy_off, z,
                       x, mean, rstd, gamma, (const float*)kk, dz, part);
  else
    hipLaunchKernelGGL(dw_bwd_dz_kernel<float>, dim3(G), dim3(256), 0, st, g, (const float*)dy, lddy, dy_img, dy_off,
                       z, x, mean, rstd, gamma, (const float*)kk, dz, part);
  hipLaunchKernelGGL(dw_wgrad_finalize_kernel, dim3((9 * C + RED_COLS - 1) / RED_COLS), dim3(1024), 0, st, (const float*)part, G, C,
                     dwt);
  hipLaunchKernelGGL(dw_bwd_dx_kernel, dim3(grid_of(n * (C / 4))), dim3(256), 0, st, g, (const float*)dz, wt, dx);
#endif
  VITMI_LAUNCH_CHECK("dwconv_bn_bwd");
  return VITMI_OK;
}

// ---------------------------------------------------------------- 'avg' projection
// AveragePooling2D(pool 3, stride 1, padding 'same') (models/CvT(Par).py:95-96,107-108): the
// mean over the in-bounds taps (TF 'same' pooling excludes the padding from the count); with
// count_pad the divisor is always 9 (torch AvgPool2d(3, 1, 1), MS_CvT old_codes/MS_CvT.py:145-153).
__device__ __forceinline__ float inb3(int i, int n) { return (float)(3 - (i == 0) - (i == n - 1)); }

template <typename TY>
__global__ void avgpool3_fwd_kernel(DwGeo g, const float* __restrict__ x, TY* __restrict__ y, int64_t ldy,
                                    int64_t y_img, int64_t y_off, int count_pad) {
  const uint32_t C4 = g.C / 4, hw = (uint32_t)g.H * g.W;
  const uint32_t total = (uint32_t)g.B * hw * C4;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int c = (int)(t % C4) * 4;
    uint32_t b;
    int h, w;
    dw_split(g, t / C4, b, h, w);
    const float* xb = x + img_row0(b, g.x_img, g.x_off) * g.ldx + c;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = -1; i <= 1; ++i) {
      const int hh = h + i;
      if (hh < 0 || hh >= g.H) continue;
#pragma unroll
      for (int j = -1; j <= 1; ++j) {
        const int ww = w + j;
        if (ww < 0 || ww >= g.W) continue;
        acc += *(const f32x4*)(xb + (int64_t)(hh * g.W + ww) * g.ldx);
      }
    }
    acc *= count_pad ? 1.f / 9.f : 1.f / (inb3(h, g.H) * inb3(w, g.W));
    TY* d = y + (img_row0(b, y_img, y_off) + h * g.W + w) * ldy + c;
#pragma unroll
    for (int e = 0; e < 4; ++e) d[e] = from_f32<TY>(acc[e]);
  }
}

// dx[p] += sum over the windows q containing p of dy[q] / count(q)
template <typename TD>
__global__ void avgpool3_bwd_kernel(DwGeo g, const TD* __restrict__ dy, int64_t lddy, int64_t dy_img,
                                    int64_t dy_off, float* __restrict__ dx, int count_pad) {
  const uint32_t C4 = g.C / 4, hw = (uint32_t)g.H * g.W;
  const uint32_t total = (uint32_t)g.B * hw * C4;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int c = (int)(t % C4) * 4;
    uint32_t b;
    int h, w;
    dw_split(g, t / C4, b, h, w);
    const TD* db = dy + img_row0(b, dy_img, dy_off) * lddy + c;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = -1; i <= 1; ++i) {
      const int hh = h + i;
      if (hh < 0 || hh >= g.H) continue;
#pragma unroll
      for (int j = -1; j <= 1; ++j) {
        const int ww = w + j;
        if (ww < 0 || ww >= g.W) continue;
        const TD* s = db + (int64_t)(hh * g.W + ww) * lddy;
        const float r = count_pad ? 1.f / 9.f : 1.f / (inb3(hh, g.H) * inb3(ww, g.W));
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] += to_f32(s[e]) * r;
      }
    }
    float* d = dx + (img_row0(b, g.x_img, g.x_off) + h * g.W + w) * g.ldx + c;
    *(f32x4*)d = *(const f32x4*)d + acc;
  }
}

extern "C" int vitmi_avgpool3_fwd(int B, int H, int W, int C, const float* x, int64_t ldx, int64_t x_img,
                                  int64_t x_off, void* y, int y_dtype, int64_t ldy, int64_t y_img, int64_t y_off,
                                  int count_pad, vitmi_stream_t stream) {
  DwGeo g;
  if (int rc = make_dw(g, B, H, W, C, ldx, x_img, x_off)) return rc;
  VITMI_CHECK_ARG(x && y, "avgpool3_fwd: null pointer");
  VITMI_CHECK_ARG(ldy % 4 == 0 && ldy >= C && y_img >= (int64_t)H * W + y_off && y_off >= 0,
                  "avgpool3_fwd: bad output layout");
  VITMI_CHECK_ARG(y_dtype == VITMI_BF16 || y_dtype == VITMI_F32, "avgpool3_fwd: bad dtype");
  hipStream_t st = (hipStream_t)stream;
  const int64_t work = (int64_t)B * H * W * (C / 4);
  if (y_dtype == VITMI_BF16)
    hipLaunchKernelGGL(avgpool3_fwd_kernel<bf16>, dim3(grid_of(work)), dim3(256), 0, st, g, x, (bf16*)y, ldy, y_img,
                       y_off, count_pad);
  else
    hipLaunchKernelGGL(avgpool3_fwd_kernel<float>, dim3(grid_of(work)), dim3(256), 0, st, g, x, (float*)y, ldy, y_img,
                       y_off, count_pad);
  VITMI_LAUNCH_CHECK("avgpool3_fwd");
  return VITMI_OK;
}

extern "C" int vitmi_avgpool3_bwd(int B, int H, int W, int C, const void* dy, int dy_dtype, int64_t lddy,
                                  int64_t dy_img, int64_t dy_off, float* dx, int64_t ldx, int64_t x_img,
                                  int64_t x_off, int count_pad, vitmi_stream_t stream) {
  DwGeo g;
  if (int rc = make_dw(g, B, H, W, C, ldx, x_img, x_off)) return rc;
  VITMI_CHECK_ARG(dy && dx, "avgpool3_bwd: null pointer");
  VITMI_CHECK_ARG(lddy % 4 == 0 && lddy >= C && dy_img >= (int64_t)H * W + dy_off && dy_off >= 0,
                  "avgpool3_bwd: bad dy layout");
  VITMI_CHECK_ARG(dy_dtype == VITMI_BF16 || dy_dtype == VITMI_F32, "avgpool3_bwd: bad dtype");
  hipStream_t st = (hipStream_t)stream;
  const int64_t work = (int64_t)B * H * W * (C / 4);
  if (dy_dtype == VITMI_BF16)
    hipLaunchKernelGGL(avgpool3_bwd_kernel<bf16>, dim3(grid_of(work)), dim3(256), 0, st, g, (const bf16*)dy, lddy,
                       dy_img, dy_off, dx, count_pad);
  else
    hipLaunchKernelGGL(avgpool3_bwd_kernel<float>, dim3(grid_of(work)), dim3(256), 0, st, g, (const float*)dy, lddy,
                       dy_img, dy_off, dx, count_pad);
  VITMI_LAUNCH_CHECK("avgpool3_bwd");
  return VITMI_OK;
}
