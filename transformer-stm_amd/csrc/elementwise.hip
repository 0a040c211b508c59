// elementwise.hip — the HBM-bound glue of the ViT path: patch im2col, token
// assembly (cls + pos-embed), bias-gradient column sums, the classifier head,
// the loss, and the fp32 -> bf16 weight cast.  All loads/stores are 16-byte
// vectors where the layout allows (cdna_hip_programming.md Guideline 13).
#include "common.h"

namespace vitmi {

// ------------------------------------------------------------ patch im2col
// patches[(b*np + ph*G + pw)][c*P*P + kh*P + kw] = img[b][c][ph*P+kh][pw*P+kw]
// one block per patch row (b, ph, pw), one thread per 4 consecutive kw (P % 4 == 0, S % 4 ==
// 0, K / 4 <= 1024): the row's indices are block-uniform, the column split is small 32-bit
// arithmetic (a grid-stride loop with 64-bit divisions per element ran 68 us at ViT-B bs 256)
template <typename T>
__global__ __launch_bounds__(1024) void im2col_kernel(const float* __restrict__ img, T* __restrict__ out, int B,
                                                      int C, int S, int P) {
  const int G = S / P, np = G * G, K = C * P * P;
  const int row = blockIdx.x;                        // b * np + ph * G + pw
  const int b = row / np, pidx = row - b * np;
  const int ph = pidx / G, pw = pidx - ph * G;
  const int col = threadIdx.x * 4;
  if (col >= K) return;
  const int c = col / (P * P), r = col - c * P * P, kh = r / P, kw = r - kh * P;
  const f32x4 v = *(const f32x4*)(img + (((int64_t)b * C + c) * S + ph * P + kh) * S + pw * P + kw);
  T* o = out + (int64_t)row * K + col;
  if constexpr (sizeof(T) == 2) {
    bf16x4 w;
    w[0] = (bf16)v[0]; w[1] = (bf16)v[1]; w[2] = (bf16)v[2]; w[3] = (bf16)v[3];
    *(bf16x4*)o = w;
  } else {
    *(f32x4*)o = v;
  }
}

// ------------------------------------------------------------ token assembly
__global__ void tokens_assemble_kernel(int B, int np, int D, const float* __restrict__ tok,
                                       const float* __restrict__ cls, const float* __restrict__ pos,
                                       float* __restrict__ x) {
  const int N = np + 1, D4 = D / 4;
  const int64_t total = (int64_t)B * N * D4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int d = (int)(i % D4) * 4;
    const int64_t bn = i / D4;
    const int n = (int)(bn % N);
    const int b = (int)(bn / N);
    f32x4 v = n == 0 ? (cls ? *(const f32x4*)(cls + d) : f32x4{0.f, 0.f, 0.f, 0.f})
                     : *(const f32x4*)(tok + ((int64_t)b * np + n - 1) * D + d);
    if (pos) v += *(const f32x4*)(pos + (int64_t)n * D + d);
    *(f32x4*)(x + bn * D + d) = v;
  }
}

__global__ void tokens_split_bwd_kernel(int B, int np, int D, const float* __restrict__ dx,
                                        float* __restrict__ dtok, bf16* __restrict__ dtok_lp) {
  const int N = np + 1, D4 = D / 4;
  const int64_t total = (int64_t)B * np * D4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int d = (int)(i % D4) * 4;
    const int64_t r = i / D4;  // b*np + p
    const int b = (int)(r / np), p = (int)(r % np);
    const f32x4 v = *(const f32x4*)(dx + ((int64_t)b * N + p + 1) * D + d);
    if (dtok) *(f32x4*)(dtok + r * D + d) = v;
    if (dtok_lp) {
      bf16x4 w;
      w[0] = (bf16)v[0]; w[1] = (bf16)v[1]; w[2] = (bf16)v[2]; w[3] = (bf16)v[3];
      *(bf16x4*)(dtok_lp + r * D + d) = w;
    }
  }
}

// dpos[n][d] += sum_b dx[b][n][d];  dcls[d] += sum_b dx[b][0][d]
__global__ void tokens_pos_bwd_kernel(int B, int N, int D, const float* __restrict__ dx,
                                      float* __restrict__ dcls, float* __restrict__ dpos) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * D) return;
  const int n = (int)(i / D), d = (int)(i % D);
  float s = 0.f;
  // 8 loads in flight per thread (the dependent one-at-a-time loop was latency-bound: 98 us for
  // 155 MB at ViT-B bs 256); the sum order stays b = 0, 1, ...
  const float* p = dx + (int64_t)n * D + d;
  const int64_t st = (int64_t)N * D;
  int b = 0;
  for (; b + 8 <= B; b += 8) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = p[(int64_t)(b + j) * st];
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j];
  }
  for (; b < B; ++b) s += p[(int64_t)b * st];
  if (dpos) dpos[i] += s;
  if (dcls && n == 0) dcls[d] += s;
}

// ------------------------------------------------------------ bias gradient
// partial[z][n] = sum over the rows of chunk z of dy[m][n].  256 threads = 4 row groups x
// 64 lanes, 8 columns per lane (one 16-byte load of bf16 / two of fp32 per row).  A wave covers
// 2^lshift lanes x 8 columns of a row and 64 >> lshift rows at a time (lshift = 6 unless N < 512:
// at N = 64 a one-row wave left 56 lanes idle).  Fixed summation order.
template <typename T>
__global__ __launch_bounds__(256) void colsum8_kernel(int64_t M, int64_t N, const T* __restrict__ dy,
                                                      int64_t ldy, float* __restrict__ part,
                                                      int64_t rows_per, int lshift) {
  __shared__ f32x4 red[4][64][2];
  const int lane = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int R = 64 >> lshift, j = lane & ((1 << lshift) - 1), r = lane >> lshift;
  const int64_t c = ((int64_t)blockIdx.x * 64 + j) * 8;
  const int64_t m0 = (int64_t)blockIdx.y * rows_per;
  const int64_t m1 = m0 + rows_per < M ? m0 + rows_per : M;
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
  if (c < N) {
#pragma unroll 4
    for (int64_t m = m0 + rg * R + r; m < m1; m += 4 * R) {
      const T* p = dy + m * ldy + c;
      if constexpr (sizeof(T) == 2) {
        const bf16x8 v = *(const bf16x8*)p;
        a0 += f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
        a1 += f32x4{(float)v[4], (float)v[5], (float)v[6], (float)v[7]};
      } else {
        a0 += *(const f32x4*)p;
        a1 += *(const f32x4*)(p + 4);
      }
    }
  }
  red[rg][lane][0] = a0;
  red[rg][lane][1] = a1;
  __syncthreads();
  if (rg == 0 && r == 0 && c < N) {
    f32x4 s0 = red[0][lane][0] + red[1][lane][0] + red[2][lane][0] + red[3][lane][0];
    f32x4 s1 = red[0][lane][1] + red[1][lane][1] + red[2][lane][1] + red[3][lane][1];
    for (int q = 1; q < R; ++q) {
      const int l2 = (q << lshift) + j;
      s0 += red[0][l2][0] + red[1][l2][0] + red[2][l2][0] + red[3][l2][0];
      s1 += red[0][l2][1] + red[1][l2][1] + red[2][l2][1] + red[3][l2][1];
    }
    float* o = part + (int64_t)blockIdx.y * N + c;
    *(f32x4*)o = s0;
    *(f32x4*)(o + 4) = s1;
  }
}

// generic (any N / alignment) variant: one thread per column
template <typename T>
__global__ void colsum_kernel(int64_t M, int64_t N, const T* __restrict__ dy, int64_t ldy,
                              float* __restrict__ part, int64_t rows_per) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const int64_t m0 = (int64_t)blockIdx.y * rows_per;
  const int64_t m1 = m0 + rows_per < M ? m0 + rows_per : M;
  float s = 0.f;
  for (int64_t m = m0; m < m1; ++m) s += to_f32(dy[m * ldy + n]);
  part[(int64_t)blockIdx.y * N + n] = s;
}

// ------------------------------------------------------------ partial-sum folds
// out[c] += sum_r part[r * ld + c] for the per-block partial rows that the LayerNorm backward
// (dgamma, dbeta and the fused bias-gradient column sums) and the fused column sums of the
// DGELU dgrad / attention backward leave behind.  One launch folds up to FOLD_MAX such jobs
// (blockIdx.y = job): each fold is a few MB and runs at the ~5 us floor of a dependent launch,
// so a backward that queues its folds (vitmi_fold_begin / _end) pays that floor once per block
// instead of four times.  Fixed summation order (row groups, then the 64 group sums in order):
// deterministic, no atomics.
struct FoldJob {
  const float* part;
  int64_t rows, cols, ld;
  float* out;
};
constexpr int FOLD_MAX = 16;
struct FoldBatch {
  FoldJob j[FOLD_MAX];
};

#ifndef VITMI_FOLD_UNROLL
#define VITMI_FOLD_UNROLL 8
#endif
__global__ __launch_bounds__(1024) void fold_kernel(FoldBatch b) {
  __shared__ float red[64][17];
  const FoldJob J = b.j[blockIdx.y];
  if ((int64_t)blockIdx.x * 16 >= J.cols) return;              // block-uniform
  const int c = threadIdx.x & 15, gi = threadIdx.x >> 4;
  const int64_t col = (int64_t)blockIdx.x * 16 + c;
  float a = 0.f;
  if (col < J.cols) {
#pragma unroll VITMI_FOLD_UNROLL
    for (int64_t r = gi; r < J.rows; r += 64) a += J.part[r * J.ld + col];
  }
  red[gi][c] = a;
  __syncthreads();
  if (threadIdx.x < 16 && col < J.cols) {
    float t = 0.f;
    for (int k = 0; k < 64; ++k) t += red[k][c];
    J.out[col] += t;
  }
}

namespace {
thread_local FoldBatch t_batch;
thread_local int t_njobs = 0;
thread_local bool t_defer = false;
thread_local hipStream_t t_stream = nullptr;
// streams that ran folds since vitmi_fold_begin (vitmi_fold_end orders its stream after them)
constexpr int FOLD_STREAMS = 8;
thread_local hipStream_t t_fold_streams[FOLD_STREAMS];
thread_local int t_nfold_streams = 0;
thread_local hipEvent_t t_fold_events[FOLD_STREAMS] = {};

// A stream past the table's FOLD_STREAMS could not be ordered before vitmi_fold_end's stream (the
// gradient read, or the workspace released, before that fold ran): refuse it instead.
int note_fold_stream(hipStream_t s) {
  for (int i = 0; i < t_nfold_streams; ++i)
    if (t_fold_streams[i] == s) return VITMI_OK;
  if (t_nfold_streams == FOLD_STREAMS)
    return fail(VITMI_ERR_UNSUPPORTED, "fold: more than %d streams ran deferred folds between vitmi_fold_begin "
                "and vitmi_fold_end", FOLD_STREAMS);
  t_fold_streams[t_nfold_streams++] = s;
  return VITMI_OK;
}

int launch_folds(const FoldBatch& b, int n, hipStream_t s) {
  if (n == 0) return VITMI_OK;
  int64_t bx = 1;
  double by = 0;
  for (int i = 0; i < n; ++i) {
    const int64_t x = (b.j[i].cols + 15) / 16;
    bx = x > bx ? x : bx;
    by += 4.0 * (b.j[i].rows + 2) * b.j[i].cols;
  }
  hipLaunchKernelGGL(fold_kernel, dim3((unsigned)bx, (unsigned)n), dim3(1024), 0, s, b);
  VITMI_LAUNCH_CHECK("fold");
  VITMI_STAT(fold_kernel, 0, by);
  return VITMI_OK;
}

int flush_folds() {
  const int n = t_njobs;
  t_njobs = 0;
  if (n > 0)
    if (int rc = note_fold_stream(t_stream)) return rc;
  return launch_folds(t_batch, n, t_stream);
}
}  // namespace

int fold_rows(const float* part, int64_t rows, int64_t cols, int64_t ld, float* out, hipStream_t s) {
  if (out == nullptr || rows <= 0 || cols <= 0) return VITMI_OK;
  const FoldJob job{part, rows, cols, ld, out};
  if (!t_defer) {
    FoldBatch b;
    b.j[0] = job;
    return launch_folds(b, 1, s);
  }
  // two queued folds into overlapping outputs would race in one launch (+= from two blocks; a tied
  // LayerNorm's dgamma receives both LN backwards' partials): launch the queue first
  bool overlap = false;
  for (int i = 0; i < t_njobs; ++i)
    overlap |= t_batch.j[i].out < out + cols && out < t_batch.j[i].out + t_batch.j[i].cols;
  if (t_njobs > 0 && (t_stream != s || t_njobs == FOLD_MAX || overlap))
    if (int rc = flush_folds()) return rc;
  t_stream = s;
  t_batch.j[t_njobs++] = job;
  return VITMI_OK;
}

int launch_colsum_finish(int64_t N, int Z, const float* part, float* db, hipStream_t s) {
  return fold_rows(part, Z, N, N, db, s);
}

// number of row chunks: enough blocks to fill the chip (~1024) for the vector kernel
static int colsum_splits(int64_t M, int64_t N) {
  const int64_t colblocks = (N + 511) / 512;
  int64_t z = 1024 / (colblocks < 1 ? 1 : colblocks);
  const int64_t zmax = (M + 31) / 32;   // >= 32 rows per chunk
  if (z > zmax) z = zmax;
  if (z > 256) z = 256;
  return (int)(z < 1 ? 1 : z);
}

// ------------------------------------------------------------ head + loss
// logits[b][c] = y[b] . w[c] + bias[c]; one wave per (b, c)
__global__ void head_fwd_kernel(int B, int D, int C, const float* __restrict__ y, int64_t ldy,
                                const float* __restrict__ w, const float* __restrict__ bias,
                                float* __restrict__ logits) {
  const int wv = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (wv >= B * C) return;
  const int b = wv / C, c = wv % C;
  float s = 0.f;
  for (int d = lane; d < D; d += 64) s += y[(int64_t)b * ldy + d] * w[(int64_t)c * D + d];
  s = wave_sum(s);
  if (lane == 0) logits[wv] = s + (bias ? bias[c] : 0.f);
}

// dy[b][d] = sum_c dl[b][c] w[c][d]
__global__ void head_bwd_dy_kernel(int B, int D, int C, const float* __restrict__ dl,
                                   const float* __restrict__ w, float* __restrict__ dy) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * D) return;
  const int b = (int)(i / D), d = (int)(i % D);
  float s = 0.f;
  for (int c = 0; c < C; ++c) s += dl[b * C + c] * w[(int64_t)c * D + d];
  dy[i] = s;
}

// dw[c][d] += sum_b dl[b][c] y[b][d];  db[c] += sum_b dl[b][c]
// grid (ceil(D/64), C), 1024 threads: 16 waves split the batch rows (wave w: b = w, w+16, ...),
// lane = column d; the 16 wave sums fold in order (deterministic).  One thread per (c, d) looping
// over the whole batch was latency-bound (73 us at B = 256, D = 768).
__global__ __launch_bounds__(1024) void head_bwd_dw_kernel(int B, int D, int C, const float* __restrict__ dl,
                                                           const float* __restrict__ y, int64_t ldy,
                                                           float* __restrict__ dw, float* __restrict__ db) {
  __shared__ float red[2][16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.y, d = blockIdx.x * 64 + lane;
  float s = 0.f, t = 0.f;
  for (int b = w; b < B; b += 16) {
    const float g = dl[(int64_t)b * C + c];
    if (d < D) s += g * y[(int64_t)b * ldy + d];
    t += g;
  }
  red[0][w][lane] = s;
  red[1][w][lane] = t;
  __syncthreads();
  if (w == 0) {
    float a = 0.f, e = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      a += red[0][k][lane];
      e += red[1][k][lane];
    }
    if (d < D) dw[(int64_t)c * D + d] += a;
    if (db && blockIdx.x == 0 && lane == 0) db[c] += e;
  }
}

// mean-reduced loss and its gradient; one block of 256 threads
__global__ void loss_kernel(int kind, int B, int C, const float* __restrict__ logits,
                            const void* __restrict__ target, float* __restrict__ loss,
                            float* __restrict__ dl) {
  __shared__ float red[256];
  float acc = 0.f;
  const float invB = 1.f / B;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const float* z = logits + (int64_t)b * C;
    if (kind == VITMI_LOSS_CE) {
      const int64_t t = ((const int64_t*)target)[b];
      float mx = -INFINITY;
      for (int c = 0; c < C; ++c) mx = fmaxf(mx, z[c]);
      float se = 0.f;
      for (int c = 0; c < C; ++c) se += expf(z[c] - mx);
      const float lse = mx + logf(se);
      acc += lse - z[t];
      if (dl)
        for (int c = 0; c < C; ++c) dl[(int64_t)b * C + c] = (expf(z[c] - lse) - (c == t ? 1.f : 0.f)) * invB;
    } else {  // MSE over all outputs (Keras mean_squared_error, C == 1 for the reference)
      const float* t = (const float*)target + (int64_t)b * C;
      for (int c = 0; c < C; ++c) {
        const float d = z[c] - t[c];
        acc += d * d / C;
        if (dl) dl[(int64_t)b * C + c] = 2.f * d * invB / C;
      }
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0 && loss) loss[0] = red[0] * invB;
}

__global__ void cast_kernel(int64_t n, const float* __restrict__ src, bf16* __restrict__ dst) {
  const int64_t n8 = n / 8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8;
       i += (int64_t)gridDim.x * blockDim.x) {
    const f32x4 a = *(const f32x4*)(src + i * 8), b = *(const f32x4*)(src + i * 8 + 4);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] = (bf16)a[j];
      o[4 + j] = (bf16)b[j];
    }
    *(bf16x8*)(dst + i * 8) = o;
  }
  const int64_t t = n8 * 8 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) dst[t] = (bf16)src[t];
}

__global__ void cast_up_kernel(int64_t n, const bf16* __restrict__ src, float* __restrict__ dst) {
  const int64_t n8 = n / 8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8;
       i += (int64_t)gridDim.x * blockDim.x) {
    const bf16x8 v = *(const bf16x8*)(src + i * 8);
    f32x4 a, b;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[j] = (float)v[j];
      b[j] = (float)v[4 + j];
    }
    *(f32x4*)(dst + i * 8) = a;
    *(f32x4*)(dst + i * 8 + 4) = b;
  }
  const int64_t t = n8 * 8 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) dst[t] = (float)src[t];
}

// y[r][c] = x[r][c] * keep(seed, site, r, c) / (1 - p): the dropout mask applied to a
// gradient in the backward (the forward fuses it into the GEMM epilogues).  4 columns per
// thread; N % 4 == 0.
template <typename TO>
__global__ void dropout_apply_kernel(int64_t M, int64_t N, const float* __restrict__ x, int64_t ldx,
                                     TO* __restrict__ y, int64_t ldy, uint32_t seed, uint32_t site,
                                     uint32_t thresh, float scale) {
  const int64_t n4 = N / 4, total = M * n4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / n4, c = (i - r * n4) * 4;
    const uint32_t rk = drop_row_key(seed, site, (uint32_t)r);
    const f32x4 v = *(const f32x4*)(x + r * ldx + c);
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = drop_hash(rk, (uint32_t)(c + e)) >= thresh ? v[e] * scale : 0.f;
    if constexpr (sizeof(TO) == 4) {
      *(f32x4*)(y + r * ldy + c) = o;
    } else {
      bf16x4 b;
#pragma unroll
      for (int e = 0; e < 4; ++e) b[e] = (bf16)o[e];
      *(bf16x4*)(y + r * ldy + c) = b;
    }
  }
}

static unsigned grid_for(int64_t work, int per_block = 256) {
  int64_t g = (work + per_block - 1) / per_block;
  if (g > 8192) g = 8192;
  return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace vitmi

using namespace vitmi;

extern "C" int vitmi_patch_im2col(int dtype, int B, int C, int S, int P, const float* img,
                                  void* patches, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(P > 0 && S % P == 0 && P % 4 == 0, "im2col: need S %% P == 0 and P %% 4 == 0");
  VITMI_CHECK_ARG(img && patches, "im2col: null pointer");
  const int K = C * P * P;
  const int64_t rows = (int64_t)B * (S / P) * (S / P);
  VITMI_CHECK_ARG(K / 4 <= 1024 && rows < 0x7fffffff, "im2col: C*P*P must be <= 4096");
  if (rows == 0) return VITMI_OK;
  hipStream_t s = (hipStream_t)stream;
  const dim3 block((unsigned)((K / 4 + 63) / 64 * 64));
  if (dtype == VITMI_BF16)
    hipLaunchKernelGGL(im2col_kernel<bf16>, dim3((unsigned)rows), block, 0, s, img, (bf16*)patches, B, C, S, P);
  else
    hipLaunchKernelGGL(im2col_kernel<float>, dim3((unsigned)rows), block, 0, s, img, (float*)patches, B, C, S, P);
  VITMI_LAUNCH_CHECK("im2col");
  return VITMI_OK;
}

extern "C" int vitmi_tokens_assemble(int B, int np, int D, const float* tok, const float* cls,
                                     const float* pos, float* x, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(D % 4 == 0 && tok && x, "tokens_assemble: bad arguments");
  const int64_t work = (int64_t)B * (np + 1) * D / 4;
  hipLaunchKernelGGL(tokens_assemble_kernel, dim3(grid_for(work)), dim3(256), 0, (hipStream_t)stream,
                     B, np, D, tok, cls, pos, x);
  VITMI_LAUNCH_CHECK("tokens_assemble");
  return VITMI_OK;
}

extern "C" int vitmi_tokens_assemble_bwd(int B, int np, int D, const float* dx, float* dtok,
                                         void* dtok_lp, float* dcls, float* dpos,
                                         vitmi_stream_t stream) {
  VITMI_CHECK_ARG(D % 4 == 0 && dx, "tokens_assemble_bwd: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  if (dtok || dtok_lp) {
    const int64_t work = (int64_t)B * np * D / 4;
    hipLaunchKernelGGL(tokens_split_bwd_kernel, dim3(grid_for(work)), dim3(256), 0, s, B, np, D, dx,
                       dtok, (bf16*)dtok_lp);
  }
  if (dcls || dpos) {
    const int64_t work = (int64_t)(np + 1) * D;
    hipLaunchKernelGGL(tokens_pos_bwd_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s, B,
                       np + 1, D, dx, dcls, dpos);
  }
  VITMI_LAUNCH_CHECK("tokens_assemble_bwd");
  return VITMI_OK;
}

extern "C" size_t vitmi_bias_grad_workspace_size(int64_t M, int64_t N) {
  return (size_t)colsum_splits(M, N) * N * sizeof(float);
}

extern "C" int vitmi_bias_grad(int dtype, int64_t M, int64_t N, const void* dy, int64_t ldy,
                               float* db, void* workspace, size_t ws_bytes, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(dy && db, "bias_grad: null pointer");
  VITMI_CHECK_ARG(workspace && ws_bytes >= vitmi_bias_grad_workspace_size(M, N), "bias_grad: workspace too small");
  if (M == 0 || N == 0) return VITMI_OK;
  hipStream_t s = (hipStream_t)stream;
  const int Z = colsum_splits(M, N);
  const int64_t rows_per = (M + Z - 1) / Z;
  const bool vec = (N % 8 == 0) && (ldy % 8 == 0) && ((uintptr_t)dy % 16 == 0);
  if (vec) {
    dim3 grid((unsigned)((N + 511) / 512), Z);
    int lshift = 6;   // lanes per row: the smallest power of two >= N / 8, at most 64
    while (lshift > 0 && (int64_t)8 << (lshift - 1) >= N) --lshift;
    if (dtype == VITMI_BF16) {
      hipLaunchKernelGGL(colsum8_kernel<bf16>, grid, dim3(256), 0, s, M, N, (const bf16*)dy, ldy,
                         (float*)workspace, rows_per, lshift);
      VITMI_STAT(colsum8_kernel<bf16>, 0, (double)M * N * 2);
    } else {
      hipLaunchKernelGGL(colsum8_kernel<float>, grid, dim3(256), 0, s, M, N, (const float*)dy, ldy,
                         (float*)workspace, rows_per, lshift);
      VITMI_STAT(colsum8_kernel<float>, 0, (double)M * N * 4);
    }
  } else {
    dim3 grid((unsigned)((N + 255) / 256), Z);
    if (dtype == VITMI_BF16)
      hipLaunchKernelGGL(colsum_kernel<bf16>, grid, dim3(256), 0, s, M, N, (const bf16*)dy, ldy,
                         (float*)workspace, rows_per);
    else
      hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(256), 0, s, M, N, (const float*)dy, ldy,
                         (float*)workspace, rows_per);
  }
  VITMI_LAUNCH_CHECK("bias_grad");
  return fold_rows((const float*)workspace, Z, N, N, db, s);
}

extern "C" int vitmi_head_fwd(int B, int D, int C, const float* y, int64_t ldy, const float* w,
                              const float* b, float* logits, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(y && w && logits && B > 0 && C > 0, "head_fwd: bad arguments");
  const int waves = B * C;
  hipLaunchKernelGGL(head_fwd_kernel, dim3((waves + 3) / 4), dim3(256), 0, (hipStream_t)stream, B, D, C,
                     y, ldy, w, b, logits);
  VITMI_LAUNCH_CHECK("head_fwd");
  return VITMI_OK;
}

extern "C" int vitmi_head_bwd(int B, int D, int C, const float* dlogits, const float* y, int64_t ldy,
                              const float* w, float* dy, float* dw, float* db,
                              vitmi_stream_t stream) {
  VITMI_CHECK_ARG(dlogits && y && w && dy && dw, "head_bwd: bad arguments");
  VITMI_CHECK_ARG(C <= 65535, "head_bwd: at most 65535 classes");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(head_bwd_dy_kernel, dim3((unsigned)(((int64_t)B * D + 255) / 256)), dim3(256), 0, s,
                     B, D, C, dlogits, w, dy);
  hipLaunchKernelGGL(head_bwd_dw_kernel, dim3((unsigned)((D + 63) / 64), (unsigned)C), dim3(1024), 0, s,
                     B, D, C, dlogits, y, ldy, dw, db);
  VITMI_LAUNCH_CHECK("head_bwd");
  return VITMI_OK;
}

extern "C" int vitmi_loss_fwd_bwd(int kind, int B, int C, const float* logits, const void* target,
                                  float* loss, float* dlogits, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(kind == VITMI_LOSS_CE || kind == VITMI_LOSS_MSE, "loss: bad kind %d", kind);
  VITMI_CHECK_ARG(logits && target && (loss || dlogits) && B > 0 && C > 0, "loss: bad arguments");
  hipLaunchKernelGGL(loss_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, kind, B, C, logits, target,
                     loss, dlogits);
  VITMI_LAUNCH_CHECK("loss");
  return VITMI_OK;
}

extern "C" int vitmi_cast_f32_bf16(int64_t n, const float* src, void* dst, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(src && dst, "cast: null pointer");
  VITMI_CHECK_ARG(((uintptr_t)src % 16) == 0 && ((uintptr_t)dst % 16) == 0, "cast: 16-byte alignment required");
  if (n == 0) return VITMI_OK;
  hipLaunchKernelGGL(cast_kernel, dim3(grid_for(n / 8 + 1)), dim3(256), 0, (hipStream_t)stream, n, src,
                     (bf16*)dst);
  VITMI_STAT(cast_kernel, 0, 6.0 * n);
  VITMI_LAUNCH_CHECK("cast");
  return VITMI_OK;
}

extern "C" int vitmi_cast_bf16_f32(int64_t n, const void* src, float* dst, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(src && dst, "cast_bf16_f32: null pointer");
  VITMI_CHECK_ARG(((uintptr_t)src % 16) == 0 && ((uintptr_t)dst % 16) == 0,
                  "cast_bf16_f32: 16-byte alignment required");
  if (n == 0) return VITMI_OK;
  hipLaunchKernelGGL(cast_up_kernel, dim3(grid_for(n / 8 + 1)), dim3(256), 0, (hipStream_t)stream, n,
                     (const bf16*)src, dst);
  VITMI_LAUNCH_CHECK("cast_bf16_f32");
  return VITMI_OK;
}

extern "C" int vitmi_dropout_apply(int64_t M, int64_t N, const float* x, int64_t ldx, void* y,
                                   int y_dtype, int64_t ldy, uint32_t seed, uint32_t site,
                                   uint32_t thresh, float scale, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(x && y, "dropout_apply: null pointer");
  VITMI_CHECK_ARG(y_dtype == VITMI_F32 || y_dtype == VITMI_BF16, "dropout_apply: bad dtype %d", y_dtype);
  VITMI_CHECK_ARG(N % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && ldx >= N && ldy >= N,
                  "dropout_apply: N and leading dims must be multiples of 4");
  VITMI_CHECK_ARG(((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 8) == 0, "dropout_apply: alignment");
  if (M == 0 || N == 0) return VITMI_OK;
  const unsigned grid = grid_for(M * N / 4);
  if (y_dtype == VITMI_F32)
    hipLaunchKernelGGL(dropout_apply_kernel<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream, M, N, x, ldx,
                       (float*)y, ldy, seed, site, thresh, scale);
  else
    hipLaunchKernelGGL(dropout_apply_kernel<bf16>, dim3(grid), dim3(256), 0, (hipStream_t)stream, M, N, x, ldx,
                       (bf16*)y, ldy, seed, site, thresh, scale);
  VITMI_LAUNCH_CHECK("dropout_apply");
  return VITMI_OK;
}

extern "C" uint32_t vitmi_dropout_hash(uint32_t seed, uint32_t site, uint32_t row, uint32_t col) {
  return drop_hash(drop_row_key(seed, site, row), col);
}

extern "C" int vitmi_fold_begin(void) {
  t_defer = true;
  t_nfold_streams = 0;
  return VITMI_OK;
}

extern "C" int vitmi_fold_end(vitmi_stream_t stream) {
  t_defer = false;
  // the queued folds run on the stream their producers ran on; `stream` then waits for each such
  // stream other than itself, so the gradients are final in `stream` order
  if (int rc = flush_folds()) return rc;
  const hipStream_t s = (hipStream_t)stream;
  for (int i = 0; i < t_nfold_streams; ++i) {
    if (t_fold_streams[i] == s) continue;
    if (!t_fold_events[i]) VITMI_HIP_CHECK(hipEventCreateWithFlags(&t_fold_events[i], hipEventDisableTiming), "fold_end");
    VITMI_HIP_CHECK(hipEventRecord(t_fold_events[i], t_fold_streams[i]), "fold_end");
    VITMI_HIP_CHECK(hipStreamWaitEvent(s, t_fold_events[i], 0), "fold_end");
  }
  t_nfold_streams = 0;
  return VITMI_OK;
}
