// dense.hip — the small fp32 Dense layers of the reference's multi-input head, gfx950.
//
//   Proc_Dense_1/2 = layers.Dense(256, activation='relu') on the 5 standardised process
//   parameters (models/CvT(Par).py:343-344).  [B x 5] -> [B x 256] -> [B x 256]: 17 MFLOP per
//   256-image batch, far below one MFMA tile's worth of work per CU, so these are plain fp32 FMA
//   kernels (exact fp32 products, fixed summation order -> deterministic), one thread per output
//   element.  The GEMM-shaped image path never comes here.
//
//   forward : y = act(x W^T + b)                  x [M][ldx], W [N][K], y [M][ldy]
//   backward: g = dy * act'(y);  dx = g W (optional),  dW += g^T x,  db += colsum(g)
#include "common.h"

namespace vitmi {

__device__ __forceinline__ float act_grad(float dy, float y, int act) { return (act == 1 && y <= 0.f) ? 0.f : dy; }

__global__ void dense_fwd_kernel(int M, int N, int K, const float* __restrict__ x, int64_t ldx,
                                 const float* __restrict__ w, const float* __restrict__ b, float* __restrict__ y,
                                 int64_t ldy, int act) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)M * N) return;
  const int m = (int)(t / N), n = (int)(t % N);
  const float* xr = x + (int64_t)m * ldx;
  const float* wr = w + (int64_t)n * K;
  float acc = b ? b[n] : 0.f;
  for (int k = 0; k < K; ++k) acc = fmaf(xr[k], wr[k], acc);
  if (act == 1) acc = fmaxf(acc, 0.f);
  y[(int64_t)m * ldy + n] = acc;
}

// dx[m][k] = sum_n g[m][n] W[n][k]
__global__ void dense_bwd_dx_kernel(int M, int N, int K, const float* __restrict__ dy, int64_t lddy,
                                    const float* __restrict__ y, int64_t ldy, const float* __restrict__ w,
                                    float* __restrict__ dx, int64_t lddx, int act) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)M * K) return;
  const int m = (int)(t / K), k = (int)(t % K);
  float acc = 0.f;
  for (int n = 0; n < N; ++n)
    acc = fmaf(act_grad(dy[(int64_t)m * lddy + n], y[(int64_t)m * ldy + n], act), w[(int64_t)n * K + k], acc);
  dx[(int64_t)m * lddx + k] = acc;
}

// dW[n][k] += sum_m g[m][n] x[m][k];  db[n] += sum_m g[m][n]  (the k == 0 thread)
__global__ void dense_bwd_dw_kernel(int M, int N, int K, const float* __restrict__ dy, int64_t lddy,
                                    const float* __restrict__ y, int64_t ldy, const float* __restrict__ x,
                                    int64_t ldx, float* __restrict__ dw, float* __restrict__ db, int act) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)N * K) return;
  const int n = (int)(t / K), k = (int)(t % K);
  float acc = 0.f, accb = 0.f;
  for (int m = 0; m < M; ++m) {
    const float g = act_grad(dy[(int64_t)m * lddy + n], y[(int64_t)m * ldy + n], act);
    acc = fmaf(g, x[(int64_t)m * ldx + k], acc);
    accb += g;
  }
  dw[t] += acc;
  if (db && k == 0) db[n] += accb;
}

static unsigned blocks_for(int64_t work) { return (unsigned)((work + 255) / 256); }

}  // namespace vitmi

using namespace vitmi;

extern "C" int vitmi_dense_f32_fwd(int M, int N, int K, const float* x, int64_t ldx, const float* w,
                                   const float* b, float* y, int64_t ldy, int act, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(M > 0 && N > 0 && K > 0 && (int64_t)M * N < (1LL << 31), "dense_f32_fwd: bad sizes");
  VITMI_CHECK_ARG(x && w && y && ldx >= K && ldy >= N, "dense_f32_fwd: bad operands");
  VITMI_CHECK_ARG(act == 0 || act == 1, "dense_f32_fwd: act must be 0 (linear) or 1 (relu)");
  hipLaunchKernelGGL(dense_fwd_kernel, dim3(blocks_for((int64_t)M * N)), dim3(256), 0, (hipStream_t)stream, M, N, K, x,
                     ldx, w, b, y, ldy, act);
  VITMI_LAUNCH_CHECK("dense_f32_fwd");
  return VITMI_OK;
}

extern "C" int vitmi_dense_f32_bwd(int M, int N, int K, const float* dy, int64_t lddy, const float* y, int64_t ldy,
                                   const float* x, int64_t ldx, const float* w, float* dx, int64_t lddx, float* dw,
                                   float* db, int act, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(M > 0 && N > 0 && K > 0 && (int64_t)N * K < (1LL << 31) && (int64_t)M * K < (1LL << 31),
                  "dense_f32_bwd: bad sizes");
  VITMI_CHECK_ARG(dy && y && x && w && dw && lddy >= N && ldy >= N && ldx >= K, "dense_f32_bwd: bad operands");
  VITMI_CHECK_ARG(act == 0 || act == 1, "dense_f32_bwd: act must be 0 (linear) or 1 (relu)");
  hipStream_t st = (hipStream_t)stream;
  if (dx) {
    VITMI_CHECK_ARG(lddx >= K, "dense_f32_bwd: bad dx stride");
    hipLaunchKernelGGL(dense_bwd_dx_kernel, dim3(blocks_for((int64_t)M * K)), dim3(256), 0, st, M, N, K, dy, lddy, y,
                       ldy, w, dx, lddx, act);
  }
  hipLaunchKernelGGL(dense_bwd_dw_kernel, dim3(blocks_for((int64_t)N * K)), dim3(256), 0, st, M, N, K, dy, lddy, y,
                     ldy, x, ldx, dw, db, act);
  VITMI_LAUNCH_CHECK("dense_f32_bwd");
  return VITMI_OK;
}
