// split.hip — operands of the precision knob (ViTConfig dtype "bf16x3").
//
// The reference computes in fp32 (Keras' default floatx; models/CvT(Par).py), and the north
// star asks for logits within 1e-3 of it.  Plain bf16 operands miss that at ViT-B depth 12
// (tools/precision_emulate.py: the weights, the LayerNorm outputs, the attention output and the
// GELU output each cost 0.5-1.8e-3 of logits error).  The knob keeps the bf16 MFMA and carries
// each of those operands as two bf16 terms, x = hi + lo with hi = bf16(x), lo = bf16(x - hi)
// (relative residual 2^-16).  A product then needs three bf16 products, hi.hi + hi.lo + lo.hi
// (lo.lo is below fp32 rounding), and the GEMM kernels do them unchanged as ONE GEMM over
// K' = 3K: the A operand's rows are laid out [hi | hi | lo] and the weight's [hi | lo | hi].
//
// The weights (and the patch-embedding im2col rows) are split here; the activation operands come
// split from their producers (LayerNorm, attention, the fc1 epilogue).  An HBM-bound stream:
// 16-B loads, 8-B stores, 4 columns per thread.
//
// The knob's cheaper form (dtype "bf16f8", VITMI_BF16F8): hi stays bf16 and the two correction
// products run as ONE block-scaled e4m3 product over 2K, so each row carries [hi | hi8 | lo8]
// (A operand) or [hi | lo8 | hi8] (weight), hi8 = e4m3(hi), lo8 = e4m3((x - hi) * 2^9) (common.h
// split_f8): 2K-equivalent MFMA work instead of 3K (tools/precision_emulate_fp8.py: logits
// 1.8-2.3e-4 at ViT-B depth 12, measured 2.2e-4).
#include "common.h"

namespace vitmi {

__device__ __forceinline__ void split4(f32x4 v, bf16x4& hi, bf16x4& lo) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    hi[e] = (bf16)v[e];
    lo[e] = (bf16)(v[e] - (float)hi[e]);
  }
}

// dst row r = pattern 0: [hi | hi | lo], pattern 1: [hi | lo | hi]; copy (optional) = hi
__global__ __launch_bounds__(256) void split3_kernel(int64_t rows, int64_t K, const float* __restrict__ src,
                                                     int64_t ld_src, bf16* __restrict__ dst, int64_t ld_dst,
                                                     int pattern, bf16* __restrict__ copy, int64_t ld_copy) {
  const int64_t K4 = K / 4, total = rows * K4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / K4, c = (i - r * K4) * 4;
    bf16x4 hi, lo;
    split4(*(const f32x4*)(src + r * ld_src + c), hi, lo);
    bf16* d = dst + r * ld_dst + c;
    *(bf16x4*)d = hi;
    *(bf16x4*)(d + K) = pattern == 0 ? hi : lo;
    *(bf16x4*)(d + 2 * K) = pattern == 0 ? lo : hi;
    if (copy) *(bf16x4*)(copy + r * ld_copy + c) = hi;
  }
}

// VITMI_BF16F8 rows (common.h split_f8, f8_off): [hi (K bf16) | e4m3 part (2K bytes)], the e4m3
// part in 64-k blocks [hi8 | lo8] (pattern 0, A operand) or [lo8 | hi8] (pattern 1, weights);
// ld_dst in bf16 units
__global__ __launch_bounds__(256) void split_f8_kernel(int64_t rows, int64_t K, const float* __restrict__ src,
                                                       int64_t ld_src, bf16* __restrict__ dst, int64_t ld_dst,
                                                       int pattern, bf16* __restrict__ copy, int64_t ld_copy) {
  const int64_t K4 = K / 4, total = rows * K4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / K4, c = (i - r * K4) * 4;
    bf16x4 hi;
    uint32_t hi8, lo8;
    split_f8(*(const f32x4*)(src + r * ld_src + c), hi, hi8, lo8);
    bf16* d = dst + r * ld_dst;
    *(bf16x4*)(d + c) = hi;
    if (pattern >= 2) {   // VITMI_BF16F8W: one byte per k, hi8 (A) or lo8 (weight)
      *(uint32_t*)((uint8_t*)(d + K) + c) = pattern == 2 ? hi8 : lo8;
    } else {
      uint8_t* f8 = (uint8_t*)(d + K) + f8_off(c);   // (common.h: 64-k blocks, [first | second])
      *(uint32_t*)f8 = pattern == 0 ? hi8 : lo8;
      *(uint32_t*)(f8 + 64) = pattern == 0 ? lo8 : hi8;
    }
    if (copy) *(bf16x4*)(copy + r * ld_copy + c) = hi;
  }
}

// Several dense weights ([rows][K] fp32 -> [rows][2K] pattern-1 rows) in one launch: the
// bf16f8 knob splits a block's four GEMM weights per forward (one launch instead of four)
struct SplitBatch {
  const float* src[8];
  bf16* dst[8];
  int64_t K[8];
  int64_t start[9];   // prefix sums of rows * K / 4 (thread items)
  int pat[8];         // 1: VITMI_BF16F8 weight rows [hi | lo8, hi8 blocks]; 3: VITMI_BF16F8W [hi | lo8]
  int n;
};
__global__ __launch_bounds__(256) void split_f8_batch_kernel(SplitBatch b) {
  const int64_t total = b.start[b.n];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int j = 0;
    while (j + 1 < b.n && i >= b.start[j + 1]) ++j;
    const int64_t K = b.K[j], K4 = K / 4, li = i - b.start[j];
    const int64_t r = li / K4, c = (li - r * K4) * 4;
    bf16x4 hi;
    uint32_t hi8, lo8;
    split_f8(*(const f32x4*)(b.src[j] + r * K + c), hi, hi8, lo8);
    if (b.pat[j] == 3) {
      bf16* d = b.dst[j] + r * (K + K / 2);
      *(bf16x4*)(d + c) = hi;
      *(uint32_t*)((uint8_t*)(d + K) + c) = lo8;
      continue;
    }
    bf16* d = b.dst[j] + r * 2 * K;
    *(bf16x4*)(d + c) = hi;
    uint8_t* f8 = (uint8_t*)(d + K) + f8_off(c);
    *(uint32_t*)f8 = lo8;
    *(uint32_t*)(f8 + 64) = hi8;
  }
}

static unsigned grid_of(int64_t items) {
  int64_t b = (items + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

}  // namespace vitmi

using namespace vitmi;

extern "C" int vitmi_split_bf16x3(int64_t rows, int64_t K, const float* src, int64_t ld_src, void* dst,
                                  int64_t ld_dst, int pattern, void* hi_copy, int64_t ld_copy, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(rows >= 0 && K > 0 && K % 4 == 0, "split_bf16x3: K must be a positive multiple of 4");
  VITMI_CHECK_ARG(pattern == 0 || pattern == 1, "split_bf16x3: pattern must be 0 ([hi|hi|lo]) or 1 ([hi|lo|hi])");
  VITMI_CHECK_ARG(ld_src >= K && ld_src % 4 == 0 && ld_dst >= 3 * K && ld_dst % 4 == 0,
                  "split_bf16x3: strides must be multiples of 4, ld_src >= K, ld_dst >= 3K");
  VITMI_CHECK_ARG(!hi_copy || (ld_copy >= K && ld_copy % 4 == 0), "split_bf16x3: bad ld_copy");
  if (rows == 0) return VITMI_OK;
  VITMI_CHECK_ARG(src && dst, "split_bf16x3: null pointer");
  VITMI_CHECK_ARG(((uintptr_t)src % 16) == 0 && ((uintptr_t)dst % 8) == 0 && ((uintptr_t)hi_copy % 8) == 0,
                  "split_bf16x3: src 16-byte, dst/copy 8-byte alignment required");
  hipLaunchKernelGGL(split3_kernel, dim3(grid_of(rows * K / 4)), dim3(256), 0, (hipStream_t)stream, rows, K, src,
                     ld_src, (bf16*)dst, ld_dst, pattern, (bf16*)hi_copy, ld_copy);
  VITMI_LAUNCH_CHECK("split_bf16x3");
  VITMI_STAT(split3_kernel, 0, (double)rows * K * (4 + 6 + (hi_copy ? 2 : 0)));
  return VITMI_OK;
}

extern "C" int vitmi_split_bf16f8_weights_mixed(int n, const float* const* srcs, void* const* dsts,
                                                const int64_t* rows, const int64_t* K, const int* patterns,
                                                vitmi_stream_t stream) {
  VITMI_CHECK_ARG(n >= 1 && n <= 8 && srcs && dsts && rows && K, "split_bf16f8_weights: 1..8 weights");
  SplitBatch b{};
  b.n = n;
  for (int j = 0; j < n; ++j) {
    b.pat[j] = patterns ? patterns[j] : 1;
    VITMI_CHECK_ARG(b.pat[j] == 1 || b.pat[j] == 3, "split_bf16f8_weights: weight %d: pattern must be 1 or 3", j);
    VITMI_CHECK_ARG(rows[j] > 0 && K[j] > 0 && K[j] % (b.pat[j] == 3 ? 128 : 64) == 0,
                    "split_bf16f8_weights: weight %d: K %% %d and rows", j, b.pat[j] == 3 ? 128 : 64);
    VITMI_CHECK_ARG(srcs[j] && dsts[j] && ((uintptr_t)srcs[j] % 16) == 0 && ((uintptr_t)dsts[j] % 16) == 0,
                    "split_bf16f8_weights: weight %d: null or unaligned pointer", j);
    b.src[j] = srcs[j];
    b.dst[j] = (bf16*)dsts[j];
    b.K[j] = K[j];
    b.start[j + 1] = b.start[j] + rows[j] * K[j] / 4;
  }
  hipLaunchKernelGGL(split_f8_batch_kernel, dim3(grid_of(b.start[n])), dim3(256), 0, (hipStream_t)stream, b);
  VITMI_LAUNCH_CHECK("split_bf16f8_weights");
  VITMI_STAT(split_f8_batch_kernel, 0, (double)b.start[n] * 4 * 8);
  return VITMI_OK;
}

extern "C" int vitmi_split_bf16f8_weights(int n, const float* const* srcs, void* const* dsts, const int64_t* rows,
                                          const int64_t* K, vitmi_stream_t stream) {
  return vitmi_split_bf16f8_weights_mixed(n, srcs, dsts, rows, K, nullptr, stream);
}

extern "C" int vitmi_split_bf16f8(int64_t rows, int64_t K, const float* src, int64_t ld_src, void* dst,
                                  int64_t ld_dst, int pattern, void* hi_copy, int64_t ld_copy, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(pattern >= 0 && pattern <= 3, "split_bf16f8: pattern must be 0 (A: [hi|hi8|lo8]), 1 (W: "
                  "[hi|lo8|hi8]), 2 (A: [hi|hi8]) or 3 (W: [hi|lo8])");
  VITMI_CHECK_ARG(rows >= 0 && K > 0 && K % (pattern >= 2 ? 128 : 64) == 0,
                  "split_bf16f8: K must be a positive multiple of %d", pattern >= 2 ? 128 : 64);
  VITMI_CHECK_ARG(ld_src >= K && ld_src % 4 == 0 && ld_dst >= (pattern >= 2 ? K + K / 2 : 2 * K) && ld_dst % 4 == 0,
                  "split_bf16f8: strides must be multiples of 4, ld_src >= K, ld_dst >= 2K (1.5K for patterns 2 / 3; "
                  "bf16 units)");
  VITMI_CHECK_ARG(!hi_copy || (ld_copy >= K && ld_copy % 4 == 0), "split_bf16f8: bad ld_copy");
  if (rows == 0) return VITMI_OK;
  VITMI_CHECK_ARG(src && dst, "split_bf16f8: null pointer");
  VITMI_CHECK_ARG(((uintptr_t)src % 16) == 0 && ((uintptr_t)dst % 8) == 0 && ((uintptr_t)hi_copy % 8) == 0,
                  "split_bf16f8: src 16-byte, dst/copy 8-byte alignment required");
  hipLaunchKernelGGL(split_f8_kernel, dim3(grid_of(rows * K / 4)), dim3(256), 0, (hipStream_t)stream, rows, K, src,
                     ld_src, (bf16*)dst, ld_dst, pattern, (bf16*)hi_copy, ld_copy);
  VITMI_LAUNCH_CHECK("split_bf16f8");
  VITMI_STAT(split_f8_kernel, 0, (double)rows * K * (4 + 4 + (hi_copy ? 2 : 0)));
  return VITMI_OK;
}
