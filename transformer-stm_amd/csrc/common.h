// Shared device/host helpers for the gfx950 (CDNA4) kernels of libvitmi.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include "../../include/vitmi.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

namespace vitmi {

// ---------------------------------------------------------------- host side
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);

#define VITMI_CHECK_ARG(cond, ...)                                   \
  do {                                                               \
    if (!(cond)) return ::vitmi::fail(VITMI_ERR_INVALID, __VA_ARGS__); \
  } while (0)

#define VITMI_HIP_CHECK(call, what)                                           \
  do {                                                                        \
    hipError_t e_ = (call);                                                   \
    if (e_ != hipSuccess)                                                     \
      return ::vitmi::fail(VITMI_ERR_HIP, "%s: %s", what, hipGetErrorString(e_)); \
  } while (0)

#define VITMI_LAUNCH_CHECK(what)                                              \
  do {                                                                        \
    hipError_t e_ = hipGetLastError();                                        \
    if (e_ != hipSuccess)                                                     \
      return ::vitmi::fail(VITMI_ERR_HIP, "%s: %s", what, hipGetErrorString(e_)); \
  } while (0)

// ---------------------------------------------------------------- conversions
__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }

// ---------------------------------------------------------------- e4m3 (the bf16f8 knob)
// VITMI_BF16F8 operands (the precision knob's cheaper form): x = hi + lo, hi = bf16(x); the row
// carries hi (bf16) and two OCP e4m3 parts, hi8 = e4m3(hi) and lo8 = e4m3(lo * 2^9), so the two
// correction products hi.lo + lo.hi run as ONE block-scaled fp8 product (the GEMM's fp8 K-steps,
// scale 2^-9 on the weight operand).  lo = x - hi is exact in fp32, at most half a bf16 ulp:
// |lo| <= 2^(e-8) for 2^e <= |x| < 2^(e+1), so lo8 = lo * 2^9 <= 2^(e+1) <= 2|x|.  The fixed scales
// bound where the corrections hold (tools/precision_emulate_fp8.py): e4m3 saturates at
// +-448, so lo8 can clip once |x| > 224 and hi8 once |x| > 448, and past that the product falls back
// to roughly plain-bf16 accuracy; at the small end hi8 is subnormal below |x| = 2^-6 and lo8 below
// |lo| = 2^-15, where those terms lose relative precision (but weigh < 2^-6 of a unit operand).
// tests/test_gpu_f8.py bounds the GEMM error inside the range (|x| up to ~200) and shows the
// fallback to bf16 accuracy past it.
// The e4m3 part (2K bytes after the K bf16 of hi) interleaves per 64 k: block j = [hi8 of k
// 64j..64j+63 | lo8 of the same k] for an A operand, [lo8 | hi8] for a weight, so one 128-B GEMM
// K-step pairs hi8.lo8 and lo8.hi8 of the same 64 k, and a producer's 64-column tile leaves as
// whole 128-B lines (K % 64 == 0).
__host__ __device__ constexpr int64_t f8_off(int64_t c) { return (c >> 6) * 128 + (c & 63); }
constexpr float F8_LO_SCALE = 512.f;
constexpr int F8_E8M0_ONE = 127, F8_E8M0_LO = 127 - 9;   // E8M0 scales 1 and 2^-9
// four floats -> four OCP e4m3 bytes (RNE; saturated to +-448 first: the conversion itself would
// give NaN past the range), little-endian in one dword
__device__ __forceinline__ uint32_t e4m3x4(float a, float b, float c, float d) {
  a = __builtin_amdgcn_fmed3f(a, 448.f, -448.f);
  b = __builtin_amdgcn_fmed3f(b, 448.f, -448.f);
  c = __builtin_amdgcn_fmed3f(c, 448.f, -448.f);
  d = __builtin_amdgcn_fmed3f(d, 448.f, -448.f);
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (uint32_t)v;
}
// hi (bf16), hi8 and lo8 (dwords of 4 e4m3) of four fp32 values
__device__ __forceinline__ void split_f8(f32x4 v, bf16x4& hi, uint32_t& hi8, uint32_t& lo8) {
  f32x4 h, l;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    hi[e] = (bf16)v[e];
    h[e] = (float)hi[e];
    l[e] = (v[e] - h[e]) * F8_LO_SCALE;
  }
  hi8 = e4m3x4(h[0], h[1], h[2], h[3]);
  lo8 = e4m3x4(l[0], l[1], l[2], l[3]);
}

// exact-erf GELU (tf.nn.gelu default, models/CvT(Par).py:254) and its derivative
__device__ __forceinline__ float gelu_f(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}
__device__ __forceinline__ float gelu_grad_f(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// ---------------------------------------------------------------- dropout mask
// Keep-mask of dropout (layers.Dropout, models/CvT(Par).py:189,255,257; Keras rate 0.1 in
// training): a counter hash of (seed, site, row, col) built from murmur3's 32-bit finaliser,
// keep iff hash >= thresh with thresh = round(p * 2^32).  Kept elements are scaled by
// 1/(1-p).  The mask is regenerated wherever it is needed (forward epilogue, backward copy)
// and never stored; oracle/vit_ref.py restates the same function bit for bit.
__host__ __device__ inline uint32_t fmix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}
__host__ __device__ inline uint32_t drop_row_key(uint32_t seed, uint32_t site, uint32_t row) {
  return fmix32(seed ^ (site * 0x9E3779B1u) ^ fmix32(row + 0x7F4A7C15u));
}
__host__ __device__ inline uint32_t drop_hash(uint32_t row_key, uint32_t col) {
  return fmix32(row_key ^ (col * 0x85EBCA77u));
}

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---------------------------------------------------------------- buffer resources
// A raw buffer descriptor: loads past `bytes` return 0 (the hardware range check),
// which is how ragged M/N/reduction edges are zero-filled without branches.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ uint32_t clamp_bytes(int64_t b) {
  return b <= 0 ? 0u : (b > 0x7fffffff ? 0x7fffffffu : (uint32_t)b);
}

// Algorithmic work of one kernel launch (flops = 2 x MACs of its dense contractions, bytes =
// the HBM bytes its operands must move at least once), accumulated per kernel while
// vitmi_stats_enable(1) is on (abi.cpp): bench.py joins it with a rocprofv3 kernel trace of
// the same run to report per-kernel TFLOP/s and GB/s.  Off (one branch) otherwise.
extern bool g_stats_on;
void stat_record(const void* kernel, double flops, double bytes);
#define VITMI_STAT(kernel, flops, bytes)                                                     \
  do {                                                                                      \
    if (::vitmi::g_stats_on) ::vitmi::stat_record((const void*)(kernel), (double)(flops), (double)(bytes)); \
  } while (0)

// db[n] += sum_z part[z][n] in a fixed order (elementwise.hip)
int launch_colsum_finish(int64_t N, int Z, const float* part, float* db, hipStream_t s);
// out[c] += sum_r part[r * ld + c] (fixed order), launched now or, between vitmi_fold_begin and
// vitmi_fold_end on this thread, queued and launched with the other queued folds (elementwise.hip)
int fold_rows(const float* part, int64_t rows, int64_t cols, int64_t ld, float* out, hipStream_t s);

}  // namespace vitmi
