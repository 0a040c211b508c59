// PROTOTYPE (tools/, not the product): a 2-blocks-per-CU bf16 GEMM main loop for gfx950, to
// measure against gemm256 before any integration.  C[M,N] = A[M,K] B[N,K]^T (both k-major),
// bf16 out + fp32 bias.  Tile 256 x 128, BK = 32, 4 waves (2 x 2, 128 x 64 outputs each, the
// same per-wave tile and C^T accumulator layout as gemm256), NSTAGE-deep LDS-DMA ring, ONE raw
// barrier per K-step; two such workgroups per CU (<= 80 KiB LDS each) so one block's epilogue
// and barrier stalls overlap the other block's MFMAs on every SIMD.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

namespace {
constexpr int BM = 256, BN = 128, BK = 32, NW = 4;
constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
constexpr int EPI_PITCH = 144, EPI_SCR = 16 * EPI_PITCH;
constexpr int DMA_PER_STAGE = STAGE / 1024 / NW;   // 6 per wave

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint32_t clampb(int64_t b) { return b <= 0 ? 0u : (b > 0x7fffffff ? 0x7fffffffu : (uint32_t)b); }
// 64-B rows: chunk' = chunk ^ 3*row[3]  (ds_read_b128 of 16 consecutive rows x one chunk per
// lane group: conflict-free, see the bank table in MI355X_MICROARCH.md §LDS)
__device__ __forceinline__ int swz(int row) { return 3 * ((row >> 3) & 1); }
__device__ __forceinline__ void barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int R>
__device__ __forceinline__ void stage_k(char* lds, __amdgpu_buffer_rsrc_t rs, int64_t ld, int64_t k0, int wave,
                                        int lane) {
  constexpr int PIECES = R * 64 / 1024;
  static_assert(PIECES % NW == 0, "pieces per wave");
#pragma unroll
  for (int j = 0; j < PIECES / NW; ++j) {
    const int p = wave + NW * j;
    const int r = p * 16 + (lane >> 2);
    const int c = (lane & 3) ^ swz(r);
    const uint32_t voff = (uint32_t)((int64_t)r * ld * 2 + k0 * 2 + c * 16);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(void, lds + p * 1024), 16, voff, 0, 0, 0);
  }
}

__device__ __forceinline__ void gelu4(f32x4 x, f32x4& a, f32x4& gp) {
  f32x4 ax, u, e;
#pragma unroll
  for (int i = 0; i < 4; ++i) ax[i] = fabsf(x[i]);
  const f32x4 d = ax * (0.3275911f * 0.70710678118654752f) + 1.0f;
  // u = -t = 1 / -d (the sign rides on v_rcp's source modifier).  In u every coefficient of the
  // -0.5-scaled polynomial is positive and each Horner step is the exact negation of the one in
  // t, so q = -0.5 P(t) bit for bit and 0.5 erf = 0.5 + q e is a plain FMA: no negated operand
  // for the compiler to materialise with a v_xor per element
#pragma unroll
  for (int i = 0; i < 4; ++i) u[i] = __builtin_amdgcn_rcpf(-d[i]);
  // exp(-x^2/2) = exp2(-(x k)^2), k = sqrt(log2(e) / 2): a packed multiply by an SGPR constant and
  // a packed square, the minus sign on v_exp's source modifier (a literal factor after the square
  // cannot be packed: it took two scalar multiplies per pair)
  const f32x4 xk = x * 0.84932180028801907f;
  const f32x4 y = xk * xk;
#pragma unroll
  for (int i = 0; i < 4; ++i) e[i] = __builtin_amdgcn_exp2f(-y[i]);
  f32x4 q = u * (0.5f * 1.061405429f) + (0.5f * 1.453152027f);
  q = q * u + (0.5f * 1.421413741f);
  q = q * u + (0.5f * 0.284496736f);
  q = q * u + (0.5f * 0.254829592f);
  q = q * u;
  f32x4 h = q * e + 0.5f;                                  // 0.5 erf(|x| / sqrt 2)
#pragma unroll
  for (int i = 0; i < 4; ++i) h[i] = __builtin_copysignf(h[i], x[i]);
  const f32x4 cdf = h + 0.5f;
  a = x * cdf;
  gp = (x * 0.39894228040143268f) * e + cdf;               // Phi(x) + x phi(x)
}


template <int NSTAGE, bool GELU>
__global__ __launch_bounds__(256, 2) void gemm2b_nt(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                     bf16* __restrict__ C, bf16* __restrict__ aux,
                                                     const float* __restrict__ bias, int M, int N, int K,
                                                     int tiles_n) {
  __shared__ __attribute__((aligned(16))) char smem[NSTAGE * STAGE];
  static_assert(NSTAGE * STAGE >= NW * EPI_SCR, "epilogue image reuses the ring");
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware tile order: blocks dealt round-robin over 8 XCDs; each XCD walks a contiguous
  // range of row-major tiles (consecutive tiles share the A row panel in that XCD's L2)
  const int total = gridDim.x, i = blockIdx.x;
  const int x = i & 7, slot = i >> 3, per = total >> 3, rem = total & 7;
  const int tile = (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + slot;
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(A + m0 * K, clampb((int64_t)(M - m0) * K * 2));
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(B + n0 * K, clampb((int64_t)(N - n0) * K * 2));
  const int nk = K / BK;

  auto issue = [&](int t) {
    char* s = smem + (t % NSTAGE) * STAGE;
    stage_k<BM>(s, ra, K, (int64_t)t * BK, wave, lane);
    stage_k<BN>(s + A_BYTES, rb, K, (int64_t)t * BK, wave, lane);
  };
  const int l15 = lane & 15, lg = lane >> 4;
  const int fofs = l15 * 64 + ((lg ^ swz(l15)) << 4);
  f32x4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int t = 0; t < NSTAGE - 1; ++t)
    if (t < nk) issue(t);
  for (int t = 0; t < nk; ++t) {
    // own DMAs of stage t done (NSTAGE-2 younger stages may stay in flight), then everyone's
    if (t + NSTAGE - 2 < nk) {
      if constexpr (NSTAGE == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if constexpr (NSTAGE == 4) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    barrier();
    if (t + NSTAGE - 1 < nk) issue(t + NSTAGE - 1);
    const char* sa = smem + (t % NSTAGE) * STAGE;
    const char* sb = sa + A_BYTES;
    bf16x8 bfr[4], afr[8];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) bfr[nt] = *(const bf16x8*)(sb + (wn * 64 + nt * 16) * 64 + fofs);
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) afr[mt] = *(const bf16x8*)(sa + (wm * 128 + mt * 16) * 64 + fofs);
#pragma unroll
    for (int mt = 0; mt < 8; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[nt], afr[mt], acc[mt][nt], 0, 0, 0);
  }
  // epilogue: bias, bf16, through a per-wave 16-row image (whole 128-B lines out)
  barrier();
  char* scr = smem + wave * EPI_SCR;
  const int lr = lane & 15, lc4 = 4 * (lane >> 4), rr = lane >> 3, cc = lane & 7;
  f32x4 bv[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) bv[nt] = bias ? *(const f32x4*)(bias + n0 + wn * 64 + nt * 16 + lc4) : f32x4{0, 0, 0, 0};
  const __amdgpu_buffer_rsrc_t rc = make_rsrc(C + m0 * N + n0, clampb((int64_t)(M - m0) * N * 2 - n0 * 2));
  const __amdgpu_buffer_rsrc_t ru = make_rsrc(aux + m0 * N + n0, GELU ? clampb((int64_t)(M - m0) * N * 2 - n0 * 2) : 0u);
  auto flush = [&](__amdgpu_buffer_rsrc_t r, int mi) {
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const u32x4 d = *(const u32x4*)(scr + (8 * j + rr) * EPI_PITCH + cc * 16);
      const uint32_t vo = (uint32_t)(((int64_t)(wm * 128 + mi * 16 + 8 * j + rr) * N + wn * 64 + cc * 8) * 2);
      __builtin_amdgcn_raw_buffer_store_b128(d, r, vo, 0, 0);
    }
    asm volatile("" ::: "memory");
  };
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    bf16x4 us[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      f32x4 v = acc[mi][nt] + bv[nt];
      if constexpr (GELU) {
        f32x4 a4, g4;
        gelu4(v, a4, g4);
        v = a4;
#pragma unroll
        for (int e = 0; e < 4; ++e) us[nt][e] = (bf16)g4[e];
      }
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (bf16)v[e];
      *(bf16x4*)(scr + lr * EPI_PITCH + (nt * 16 + lc4) * 2) = o;
    }
    flush(rc, mi);
    if constexpr (GELU) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) *(bf16x4*)(scr + lr * EPI_PITCH + (nt * 16 + lc4) * 2) = us[nt];
      flush(ru, mi);
    }
  }
}
}  // namespace

template <bool G>
static void launch(int nstage, dim3 grid, hipStream_t s, const bf16* A, const bf16* B, bf16* C, bf16* aux,
                   const float* bias, int M, int N, int K, int tiles_n) {
  if (nstage == 2)
    hipLaunchKernelGGL((gemm2b_nt<2, G>), grid, dim3(256), 0, s, A, B, C, aux, bias, M, N, K, tiles_n);
  else if (nstage == 4)
    hipLaunchKernelGGL((gemm2b_nt<4, G>), grid, dim3(256), 0, s, A, B, C, aux, bias, M, N, K, tiles_n);
  else
    hipLaunchKernelGGL((gemm2b_nt<3, G>), grid, dim3(256), 0, s, A, B, C, aux, bias, M, N, K, tiles_n);
}

// aux != NULL: C = gelu(acc + bias), aux = gelu'(acc + bias) (the fc1 epilogue of gemm256)
extern "C" int proto_gemm_nt(int nstage, int M, int N, int K, const void* A, const void* B, void* C, void* aux,
                             const float* bias, void* stream) {
  if (M % BM || N % BN || K % BK || K / BK < 2) return 1;
  const int tiles_n = N / BN, tiles = (M / BM) * tiles_n;
  hipStream_t s = (hipStream_t)stream;
  if (aux)
    launch<true>(nstage, dim3(tiles), s, (const bf16*)A, (const bf16*)B, (bf16*)C, (bf16*)aux, bias, M, N, K, tiles_n);
  else
    launch<false>(nstage, dim3(tiles), s, (const bf16*)A, (const bf16*)B, (bf16*)C, nullptr, bias, M, N, K, tiles_n);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
