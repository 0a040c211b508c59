// optim.hip — the reference's optimizer step, fused, gfx950.
//
// model.compile(optimizer=keras.optimizers.Adam(learning_rate=1e-3)) (models/CvT(Par).py:458-460)
// with Keras' Adam update (beta_1 0.9, beta_2 0.999, epsilon 1e-7; the "epsilon hat" form: eps
// is added to sqrt(v) WITHOUT bias correction, the bias corrections are folded into the step):
//
//   m <- m + (g - m)(1 - b1);   v <- v + (g^2 - v)(1 - b2)
//   p <- p - alpha m / (sqrt(v) + eps),   alpha = lr sqrt(1 - b2^t) / (1 - b1^t)  (host, fp32)
//
// One launch over a ParamArena's flat fp32 buffers (all parameters, gradients, m, v at the same
// offsets); optionally writes the bf16 operand shadow of the updated parameters in the same pass
// (what the next forward's GEMMs read), so no separate cast pass is needed.  HBM-bound:
// 16 B read + 12 B written per parameter (+2 B with the shadow).  Every operation is an
// explicitly rounded IEEE fp32 op in the order above (no FMA contraction), so the result is
// bit-identical to a numpy float32 evaluation of the same formula (oracle/optim_ref.py).
#include "common.h"

namespace vitmi {

struct AdamArgs {
  float alpha, one_m_b1, one_m_b2, eps, grad_scale;
};

__device__ __forceinline__ void adam1(const AdamArgs& a, float& p, float g, float& m, float& v) {
  // HIP's __f*_rn are plain operators (and __fsqrt_rn is the native approximation): the file is
  // built with -ffp-contract=off (Makefile) so a*b+c stays two roundings; sqrtf and / are
  // correctly rounded in HIP by default
  if (a.grad_scale != 1.f) g = __fmul_rn(g, a.grad_scale);
  m = __fadd_rn(m, __fmul_rn(__fsub_rn(g, m), a.one_m_b1));
  v = __fadd_rn(v, __fmul_rn(__fsub_rn(__fmul_rn(g, g), v), a.one_m_b2));
  const float den = __fadd_rn(sqrtf(v), a.eps);
  p = __fsub_rn(p, __fdiv_rn(__fmul_rn(m, a.alpha), den));
}

// VITMI_ADAM_NT: streaming (non-temporal) loads and stores, two 16-B groups per thread in flight:
// 573-595 -> 504-526 us per ViT-B step (tools/ln_bench.py, same box; gpurun_out r04_ln A/B)
#ifndef VITMI_ADAM_NT
#define VITMI_ADAM_NT 1
#endif
template <typename V>
__device__ __forceinline__ V ld_s(const V* q) {
  if constexpr (VITMI_ADAM_NT) return __builtin_nontemporal_load(q);
  else return *q;
}
template <typename V>
__device__ __forceinline__ void st_s(V* q, V x) {
  if constexpr (VITMI_ADAM_NT) __builtin_nontemporal_store(x, q);
  else *q = x;
}

template <bool LP>
__global__ __launch_bounds__(256) void adam_kernel(int64_t n, float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   bf16* __restrict__ lp, AdamArgs a) {
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  constexpr int U = VITMI_ADAM_NT ? 2 : 1;
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < n4; i0 += U * stride) {
    f32x4 pv[U], gv[U], mv[U], vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (u == 0 || i < n4) {
        pv[u] = ld_s((const f32x4*)p + i);
        gv[u] = ld_s((const f32x4*)g + i);
        mv[u] = ld_s((const f32x4*)m + i);
        vv[u] = ld_s((const f32x4*)v + i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (u > 0 && i >= n4) break;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float pe = pv[u][e], me = mv[u][e], ve = vv[u][e];
        adam1(a, pe, gv[u][e], me, ve);
        pv[u][e] = pe;
        mv[u][e] = me;
        vv[u][e] = ve;
      }
      st_s((f32x4*)p + i, pv[u]);
      st_s((f32x4*)m + i, mv[u]);
      st_s((f32x4*)v + i, vv[u]);
      if constexpr (LP) {
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = from_f32<bf16>(pv[u][e]);
        ((bf16x4*)lp)[i] = o;
      }
    }
  }
  // tail (n % 4) by the first threads
  const int64_t t = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n && t < n4 * 4 + 4) {
    float pe = p[t], me = m[t], ve = v[t];
    adam1(a, pe, g[t], me, ve);
    p[t] = pe;
    m[t] = me;
    v[t] = ve;
    if constexpr (LP) lp[t] = from_f32<bf16>(pe);
  }
}

}  // namespace vitmi

using namespace vitmi;

extern "C" int vitmi_adam_step(int64_t n, float* p, const float* g, float* m, float* v, void* p_lp, float alpha,
                               double beta_1, double beta_2, float epsilon, float grad_scale, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(n >= 0, "adam_step: n < 0");
  if (n == 0) return VITMI_OK;
  VITMI_CHECK_ARG(p && g && m && v, "adam_step: null pointer");
  VITMI_CHECK_ARG(((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16 == 0,
                  "adam_step: fp32 buffers must be 16-byte aligned");
  VITMI_CHECK_ARG(!p_lp || (uintptr_t)p_lp % 8 == 0, "adam_step: bf16 shadow must be 8-byte aligned");
  VITMI_CHECK_ARG(beta_1 >= 0.0 && beta_1 < 1.0 && beta_2 >= 0.0 && beta_2 < 1.0 && epsilon >= 0.f,
                  "adam_step: bad hyper-parameters");
  // (1 - beta) in double then rounded once, as Keras does with its Python-float hyper-parameters
  AdamArgs a{alpha, (float)(1.0 - beta_1), (float)(1.0 - beta_2), epsilon, grad_scale};
  const int64_t work = (n / 4) > 0 ? (n / 4) : 1;
  int64_t blocks = (work + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (p_lp)
    hipLaunchKernelGGL(adam_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, n, p, g, m, v,
                       (bf16*)p_lp, a);
  else
    hipLaunchKernelGGL(adam_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, n, p, g, m, v,
                       (bf16*)nullptr, a);
  VITMI_LAUNCH_CHECK("adam_step");
  // p, g, m, v read; p, m, v (+ the bf16 shadow) written
  if (p_lp) VITMI_STAT(adam_kernel<true>, 0, (double)n * 30);
  else VITMI_STAT(adam_kernel<false>, 0, (double)n * 28);
  return VITMI_OK;
}
