// sls.hip — the reference's SLS image preprocessing on the GPU, gfx950.
//
// models/CvT(Par).py:414-428 per layer image: cv2.imread (BGR uint8 340x345) ->
// cv2.resize(img, (128, 128)) (INTER_LINEAR) -> cv2.cvtColor(BGR2GRAY) -> / 255.0.
// The reference runs this per image on the host inside its data loading; here the decoded
// uint8 frames are uploaded in chunks and ONE launch per chunk produces the fp32 model inputs,
// which stay resident in HBM for the whole training run (40,000 layers x 64 KiB = 2.6 GB).
//
// Bit-level semantics (OpenCV 4.x 8-bit fixed point, restated in oracle/sls_ref.py):
//   horizontal: H[c] = src[y][x0][c] * a0 + src[y][x1][c] * a1            (Q11 weights, exact int)
//   vertical:   v = ((((H0 >> 4) * b0) >> 16) + (((H1 >> 4) * b1) >> 16) + 2) >> 2, saturated to u8
//   gray:       (B*1868 + G*9617 + R*4899 + 2^13) >> 14
//   output:     (float)(gray / 255.0)   (fp64 division rounded once, numpy's float64 then Keras' cast)
// The axis tables (source offsets + Q11 weights) come from vitmi_sls_resize_table (host).
//
// One thread per output pixel; the source is read through L2 (adjacent output pixels share
// source rows), 12 B of useful reads + 4 B written per pixel: an HBM-bound gather.
#include "common.h"

#include <cmath>

namespace vitmi {

__global__ __launch_bounds__(256) void sls_preprocess_kernel(int n, int H, int W, const uint8_t* __restrict__ src,
                                                             int64_t img_bytes, int64_t row_bytes, int bgr, int Ho,
                                                             int Wo, const int* __restrict__ xofs,
                                                             const short* __restrict__ xw,
                                                             const int* __restrict__ yofs,
                                                             const short* __restrict__ yw, float* __restrict__ out) {
  const int64_t total = (int64_t)n * Ho * Wo;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(t % Wo);
    const int y = (int)((t / Wo) % Ho);
    const int64_t img = t / ((int64_t)Wo * Ho);
    const int sx0 = xofs[x], sx1 = min(sx0 + 1, W - 1);
    const int sy0 = yofs[y], sy1 = min(sy0 + 1, H - 1);
    const int a0 = xw[2 * x], a1 = xw[2 * x + 1], b0 = yw[2 * y], b1 = yw[2 * y + 1];
    const uint8_t* base = src + img * img_bytes;
    const uint8_t* r0 = base + (int64_t)sy0 * row_bytes;
    const uint8_t* r1 = base + (int64_t)sy1 * row_bytes;
    int ch[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int h0 = r0[sx0 * 3 + c] * a0 + r0[sx1 * 3 + c] * a1;
      const int h1 = r1[sx0 * 3 + c] * a0 + r1[sx1 * 3 + c] * a1;
      int v = ((((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16) + 2) >> 2;
      ch[c] = v < 0 ? 0 : (v > 255 ? 255 : v);
    }
    const int B = bgr ? ch[0] : ch[2], G = ch[1], R = bgr ? ch[2] : ch[0];
    const int gray = (B * 1868 + G * 9617 + R * 4899 + (1 << 13)) >> 14;
    out[t] = (float)((double)gray / 255.0);
  }
}

}  // namespace vitmi

using namespace vitmi;

// cv2 INTER_LINEAR axis table: ofs[d] = first source index, w[2d], w[2d+1] = Q11 weights.
extern "C" int vitmi_sls_resize_table(int ssize, int dsize, int* ofs, short* w) {
  VITMI_CHECK_ARG(ssize > 0 && dsize > 0 && ofs && w, "sls_resize_table: bad arguments");
  const double inv_scale = (double)dsize / ssize;
  const double scale = 1.0 / inv_scale;
  for (int d = 0; d < dsize; ++d) {
    float f = (float)((d + 0.5) * scale - 0.5);
    int s = (int)std::floor(f);
    f -= (float)s;
    if (s < 0) {
      f = 0.f;
      s = 0;
    }
    if (s >= ssize - 1) {
      f = 0.f;
      s = ssize - 1;
    }
    const float c0 = 1.f - f, c1 = f;
    ofs[d] = s;
    w[2 * d] = (short)std::lrint(c0 * 2048.f);
    w[2 * d + 1] = (short)std::lrint(c1 * 2048.f);
  }
  return VITMI_OK;
}

extern "C" int vitmi_sls_preprocess(int n, int H, int W, const void* src, int64_t img_bytes, int64_t row_bytes,
                                    int bgr, int Ho, int Wo, const int* xofs, const short* xw, const int* yofs,
                                    const short* yw, float* out, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(n >= 0 && H > 0 && W > 0 && Ho > 0 && Wo > 0, "sls_preprocess: bad sizes");
  if (n == 0) return VITMI_OK;
  VITMI_CHECK_ARG(src && xofs && xw && yofs && yw && out, "sls_preprocess: null pointer");
  VITMI_CHECK_ARG(row_bytes >= 3LL * W && img_bytes >= row_bytes * H, "sls_preprocess: bad source layout");
  const int64_t total = (int64_t)n * Ho * Wo;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(sls_preprocess_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, n, H, W,
                     (const uint8_t*)src, img_bytes, row_bytes, bgr, Ho, Wo, xofs, xw, yofs, yw, out);
  VITMI_LAUNCH_CHECK("sls_preprocess");
  return VITMI_OK;
}

// Batch assembly from the HBM-resident dataset: dst[i] = src[idx[i]] for rows of row_bytes
// (images, process parameters, labels), 16-byte vectorised when the row size allows.
namespace vitmi {
// an index outside [0, n_src) yields a zero row (never an out-of-bounds read)
__global__ void gather_rows_kernel(int64_t n, int64_t row_words, const uint4* __restrict__ src, int64_t n_src,
                                   const int64_t* __restrict__ idx, uint4* __restrict__ dst) {
  const int64_t total = n * row_words;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / row_words, w = t - r * row_words;
    const int64_t i = idx[r];
    dst[t] = (i >= 0 && i < n_src) ? src[i * row_words + w] : make_uint4(0, 0, 0, 0);
  }
}
__global__ void gather_rows_b_kernel(int64_t n, int64_t row_bytes, const uint8_t* __restrict__ src, int64_t n_src,
                                     const int64_t* __restrict__ idx, uint8_t* __restrict__ dst) {
  const int64_t total = n * row_bytes;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / row_bytes, b = t - r * row_bytes;
    const int64_t i = idx[r];
    dst[t] = (i >= 0 && i < n_src) ? src[i * row_bytes + b] : (uint8_t)0;
  }
}
}  // namespace vitmi

extern "C" int vitmi_gather_rows(int64_t n, int64_t row_bytes, const void* src, int64_t n_src, const int64_t* idx,
                                 void* dst, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(n >= 0 && row_bytes > 0, "gather_rows: bad sizes");
  if (n == 0) return VITMI_OK;
  VITMI_CHECK_ARG(src && idx && dst, "gather_rows: null pointer");
  const bool vec = row_bytes % 16 == 0 && (uintptr_t)src % 16 == 0 && (uintptr_t)dst % 16 == 0;
  const int64_t total = vec ? n * (row_bytes / 16) : n * row_bytes;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  if (vec)
    hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, n, row_bytes / 16,
                       (const uint4*)src, n_src, idx, (uint4*)dst);
  else
    hipLaunchKernelGGL(gather_rows_b_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, n, row_bytes,
                       (const uint8_t*)src, n_src, idx, (uint8_t*)dst);
  VITMI_LAUNCH_CHECK("gather_rows");
  return VITMI_OK;
}
