// gemm.hip — LDS-tiled MFMA GEMM for gfx950 with fused epilogues.
//
// C[M,N] = sum_k A(m,k) B(k,n); each operand is either k-major (rows of k, the
// nn.Linear weight / activation layout) or m/n-major (the transposed operands of
// the backward).  Tiles are staged global->LDS with `buffer_load ... lds`
// (LDS-DMA, 16 B per lane, no VGPR round trip); the buffer range check zero-fills
// ragged edges.  The LDS images are XOR-swizzled on the SOURCE address so the
// fragment reads are bank-conflict free:
//   k-major  [R][BK]: chunk' = chunk ^ ((row >> 1) & 7)       read by ds_read_b128
//   mn-major [BK][R]: chunk' = chunk ^ (2*(k&3) + 8*((k>>3)&1)) read by ds_read_b64_tr_b16
// (tools/lds_bank_check.py enumerates every access of both images.)
//
// MFMA: v_mfma_f32_16x16x32_bf16 for bf16 operands, v_mfma_f32_16x16x4_f32 for
// fp32 (exact fp32 products).  For fp32 each lane reads 8 consecutive k and the
// j-th MFMA consumes element j from every lane group: both operands use the same
// k permutation, so the sum is unchanged.
#include <atomic>
#include "common.h"
#include <stdlib.h>
#include <type_traits>

// Opens every inline-asm buffer store that takes SGPR operands (descriptor, soffset): under SGPR
// pressure hipcc rematerialises such operands with v_readlane right before the statement, and a
// VALU write of an SGPR needs 5 wait states before a VMEM instruction reads it.  hipcc pads that
// hazard for its own instructions only, not for the text of an asm statement; without the pad the
// store reads the stale soffset and lands on another row group (seen on the GELU-dropout and
// residual epilogues).
#define VMEM_SGPR_GUARD "s_nop 4\n\t"
// cache-policy modifiers of the epilogue's output stores (empty: the default policy)
// (VITMI_ST_MASK bits: 1 = gelu' aux, 2 = bf16 C, 4 = fp32 C / residual output, 8 = split-K
// partial slabs; the bit's stores carry the non-temporal hint)
#ifndef VITMI_ST_MASK
#define VITMI_ST_MASK 3
#endif
#if VITMI_ST_MASK & 1
#define VITMI_ST_AUX " nt"
#else
#define VITMI_ST_AUX ""
#endif
#if VITMI_ST_MASK & 2
#define VITMI_ST_C16 " nt"
#else
#define VITMI_ST_C16 ""
#endif
#if VITMI_ST_MASK & 4
#define VITMI_ST_C32 " nt"
#else
#define VITMI_ST_C32 ""
#endif
#if VITMI_ST_MASK & 8
#define VITMI_ST_PART " nt"
#else
#define VITMI_ST_PART ""
#endif

namespace vitmi {

template <typename T> struct TT;
template <> struct TT<bf16> { static constexpr int BK = 64, ES = 2; };
template <> struct TT<float> { static constexpr int BK = 32, ES = 4; };

struct GemmArgs {
  const void* A;
  const void* B;
  void* C;
  int64_t M, N, K;
  int64_t lda, ldb, ldc;
  const float* bias;
  void* aux;
  int64_t ldaux;
  const float* residual;
  int64_t ldr;
  int64_t k_per_split;   // reduction range of one blockIdx.z (multiple of BK)
  int64_t split_stride;  // elements between split partial slabs (EPI_PARTIAL)
  int tiles_n;           // number of BN tiles along N
  // gemm256 tail split (stream-K-like): units [0, t_full) are whole tiles; the remaining
  // tiles are split into nsplit K-ranges of ksplit K-steps each, written as fp32 partials
  // to tail_ws ([unit - t_full][256][256]) and finished by gemm_tail_fixup_kernel.
  int t_full;
  int nsplit;
  int ksplit;
  float* tail_ws;
  size_t tail_ws_bytes;
  // gemm256 split-K folded into the persistent unit space (EPI_PARTIAL): unit = z*ntiles +
  // tile, slab z covers K-steps [z*kz_steps, (z+1)*kz_steps).  Consecutive units share one
  // K-range, so the contiguous unit range of an XCD re-reads its A/B panels from that
  // XCD's L2 (a gridDim.z split scatters them over all XCDs).
  int kz;          // 1 = no folded split
  int kz_steps;
  int ntiles;
  // dropout of the *_DROP epilogues (see drop_hash in common.h)
  uint32_t drop_seed, drop_site, drop_thresh;
  float drop_scale;
  // gemm256 DGELU epilogue: column sums of the output (the bias gradient of the layer whose
  // input gradient this is), one fp32 row per 128-row half tile: colsum[(2*tm + wm)*N + col]
  float* colsum;
  unsigned long long* stamps;        // DIAGNOSTIC build only (VITMI_GEMM_STAMPS)
  int aux_tiled;                     // gelu' in the tile-native layout (VITMI_EPI_AUX_TILED)
  // VITMI_BF16F8 operands (gemm256<..., F8>): K-steps >= k8 (absolute, 64-bf16 = 128-B steps) are
  // the rows' e4m3 parts, multiplied by the block-scaled fp8 MFMA; the steps before are bf16
  int k8;
  // grouped weight gradients (gemm256_kernel<false, false, EPI_PARTIAL, float, false, true>): up to
  // GRP_MAX problems over one reduction length K, each with its own operands and partial slabs;
  // the folded split-K unit space runs over their concatenated tiles (problem p owns tiles
  // [tile0, tile0 + tiles)); slab z of problem p at C + z * M * N (fp32, row pitch N)
  struct Prob {
    const void* A;
    const void* B;
    float* C;
    int64_t M, N, lda, ldb;
    int tiles_n, tile0;
  } grp[4];
  int ngrp;
};
constexpr int GRP_MAX = 4;

// Element (row, col) of a tile-native gelu' buffer (VITMI_EPI_AUX_TILED; bf16 elements): 256x256
// tiles in row-major tile order, each 128 KiB laid out as gemm256's epilogue registers hold it --
// [wave (wm*4 + wn)][row group mi][column pair][lane][16 B], lane = (row & 15) + 16 * ((col >> 2) & 3)
// -- so the BIAS_GELU epilogue stores and the DGELU epilogue loads whole KiB per instruction
// straight from / into the accumulator layout.
__device__ __forceinline__ int64_t aux_at(const GemmArgs& g, int64_t row, int64_t col) {
  if (!g.aux_tiled) return row * g.ldaux + col;
  const int64_t tile = (row >> 8) * ((g.N + 255) >> 8) + (col >> 8);
  const int r = (int)(row & 255), c = (int)(col & 255);
  const int wave = (r >> 7) * 4 + (c >> 6), mi = (r >> 4) & 7, ni = (c >> 4) & 3;
  const int lane = (r & 15) + 16 * ((c >> 2) & 3);
  return tile * 65536 + (((wave * 8 + mi) * 2 + (ni >> 1)) * 1024 + lane * 16 + (ni & 1) * 8) / 2 + (c & 3);
}

// (tile-row, tile-col) of tile index tl: row-major over the tiles_n tile columns (a persistent
// block walks consecutive tiles, so an XCD's concurrent tiles share A row panels in its L2;
// grouped column-major orders measured 0.5-1 % slower end to end)
// row panels per tile group (0: row-major tiles).  C3 step 7292-7314 -> 7335-7350 img/s over
// three rounds (GM 5 and 7 as row-major; fc1 + GELU 308-313 -> 299-304 µs, DGELU 297-302 -> 288;
// profiles/r06_gm*)
#ifndef VITMI_TILE_GM
#define VITMI_TILE_GM 6
#endif
__device__ __forceinline__ void tile_rc(const GemmArgs& g, int tl, int& tm, int& tn) {
  if constexpr (VITMI_TILE_GM > 1) {
    // groups of GM row panels walked column by column: an XCD's 32 concurrent tiles span GM row
    // panels x 32/GM column panels instead of ~3 x all of them, and the next ones reuse the
    // same GM row panels from its L2
    const int tiles_m = (int)((g.M + 255) >> 8);
    const int per = VITMI_TILE_GM * g.tiles_n;
    const int grp = tl / per, r = tl - grp * per;
    const int m0 = grp * VITMI_TILE_GM;
    const int gm = tiles_m - m0 < VITMI_TILE_GM ? tiles_m - m0 : VITMI_TILE_GM;
    tn = r / gm;
    tm = m0 + (r - tn * gm);
  } else {
    tm = tl / g.tiles_n;
    tn = tl - tm * g.tiles_n;
  }
}

// internal epilogues: split-K partial slab, and GELU / residual with a fused dropout
// EPI_GELU_X3: BIAS_GELU with the activation written split, [hi | hi | lo] (VITMI_EPI_SPLIT_X3)
// EPI_GELU_F8: BIAS_GELU with the activation written as VITMI_BF16F8 A-operand rows (VITMI_EPI_SPLIT_F8)
enum { EPI_PARTIAL = 100, EPI_GELU_DROP = 101, EPI_RESIDUAL_DROP = 102, EPI_GELU_X3 = 103, EPI_GELU_F8 = 104 };
// the public epilogue an internal one extends, and whether it drops
template <int EPI> struct EpiOf {
  static constexpr int base = EPI == EPI_GELU_DROP || EPI == EPI_GELU_X3 || EPI == EPI_GELU_F8 ? VITMI_EPI_BIAS_GELU
                              : EPI == EPI_RESIDUAL_DROP ? VITMI_EPI_RESIDUAL : EPI;
  static constexpr bool drop = EPI == EPI_GELU_DROP || EPI == EPI_RESIDUAL_DROP;
};
static inline int epi_base(int epi) {
  return epi == EPI_GELU_DROP || epi == EPI_GELU_X3 || epi == EPI_GELU_F8 ? VITMI_EPI_BIAS_GELU
         : epi == EPI_RESIDUAL_DROP ? VITMI_EPI_RESIDUAL : epi;
}
// dropout factor (0 or 1/(1-p)) of output element (row, col)
__device__ __forceinline__ float drop_factor(const GemmArgs& g, int64_t row, int64_t col) {
  return drop_hash(drop_row_key(g.drop_seed, g.drop_site, (uint32_t)row), (uint32_t)col) >= g.drop_thresh
             ? g.drop_scale : 0.f;
}

__device__ __forceinline__ int swz_k(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int swz_mn(int k) { return 2 * (k & 3) + 8 * ((k >> 3) & 1); }

// Fragment of one 16x16xK32 MFMA step for one lane.
template <typename T> struct Frag;
template <> struct Frag<bf16> { bf16x8 v; };
template <> struct Frag<float> { f32x4 lo, hi; };

// ---- tile staging ---------------------------------------------------------
// Stage an R x BK tile (rows = m or n) of a k-major matrix into LDS image [R][BK].
template <typename T, int R, int NWAVES>
__device__ __forceinline__ void stage_kmajor(char* lds, __amdgpu_buffer_rsrc_t rs, int64_t ld,
                                             int64_t k0, int wave, int lane) {
  constexpr int ES = TT<T>::ES, BK = TT<T>::BK;
  constexpr int RB = BK * ES;            // 128 bytes per row
  constexpr int PIECES = R * RB / 1024;  // 1 KiB per wave instruction
  static_assert(RB == 128, "k-major rows must be 128 B");
#pragma unroll
  for (int p = wave; p < PIECES; p += NWAVES) {
    const int r = p * 8 + (lane >> 3);
    const int c = (lane & 7) ^ swz_k(r);
    const uint32_t voff = (uint32_t)(r * ld * ES + k0 * ES + c * 16);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(void, lds + p * 1024), 16, voff, 0, 0, 0);
  }
}

// Stage a BK x R tile (rows = k) of an m/n-major matrix into LDS image [BK][R].
template <typename T, int R, int NWAVES>
__device__ __forceinline__ void stage_mnmajor(char* lds, __amdgpu_buffer_rsrc_t rs, int64_t ld,
                                              int64_t krow0, int wave, int lane) {
  constexpr int ES = TT<T>::ES, BK = TT<T>::BK;
  constexpr int RB = R * ES;
  constexpr int CPR = RB / 16;        // chunks per row
  constexpr int RPP = 64 / CPR;       // rows per 1 KiB piece
  constexpr int PIECES = BK * RB / 1024;
  static_assert(CPR >= 16 && CPR <= 64, "m/n-major rows must be 256..1024 B");
#pragma unroll
  for (int p = wave; p < PIECES; p += NWAVES) {
    const int r = p * RPP + lane / CPR;
    const int c = (lane % CPR) ^ swz_mn(r);
    const uint32_t voff = (uint32_t)((krow0 + r) * ld * ES + c * 16);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(void, lds + p * 1024), 16, voff, 0, 0, 0);
  }
}

// ---- fragment reads -------------------------------------------------------
template <typename T, bool KMAJ, int R>
struct FragReader;

template <int R>
struct FragReader<bf16, true, R> {
  static __device__ __forceinline__ Frag<bf16> read(const char* lds, int row0, int kk, int lane) {
    const int row = row0 + (lane & 15);
    const int c = ((kk >> 3) + (lane >> 4)) ^ swz_k(row);
    Frag<bf16> f;
    f.v = *(const bf16x8*)(lds + row * 128 + c * 16);
    return f;
  }
};

template <int R>
struct FragReader<float, true, R> {
  static __device__ __forceinline__ Frag<float> read(const char* lds, int row0, int kk, int lane) {
    const int row = row0 + (lane & 15);
    const int c0 = (kk >> 2) + 2 * (lane >> 4);
    const int s = swz_k(row);
    Frag<float> f;
    f.lo = *(const f32x4*)(lds + row * 128 + ((c0) ^ s) * 16);
    f.hi = *(const f32x4*)(lds + row * 128 + ((c0 + 1) ^ s) * 16);
    return f;
  }
};

template <int R>
struct FragReader<bf16, false, R> {
  // image [BK][R] bf16, rows of R*2 bytes; lane gets col row0+(lane&15), k = kk+8g+j
  static __device__ __forceinline__ Frag<bf16> read(const char* lds, int row0, int kk, int lane) {
    constexpr int RB = R * 2;
    const int t = lane & 15, g = lane >> 4, q = t >> 2, p = t & 3;
    const int chunk = (row0 >> 3) + (p >> 1);
    Frag<bf16> f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int kr = kk + 8 * g + 4 * i + q;
      const int addr = kr * RB + ((chunk ^ swz_mn(kr)) * 16) + (p & 1) * 8;
      s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, lds + addr));
      bf16x4 b = __builtin_bit_cast(bf16x4, v);
      f.v[4 * i + 0] = b[0];
      f.v[4 * i + 1] = b[1];
      f.v[4 * i + 2] = b[2];
      f.v[4 * i + 3] = b[3];
    }
    return f;
  }
};

template <int R>
struct FragReader<float, false, R> {
  static __device__ __forceinline__ Frag<float> read(const char* lds, int row0, int kk, int lane) {
    constexpr int RB = R * 4;
    const int col = row0 + (lane & 15), g = lane >> 4;
    const int cb = col * 4;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kr = kk + 8 * g + j;
      v[j] = *(const float*)(lds + kr * RB + (((cb >> 4) ^ swz_mn(kr)) << 4) + (cb & 15));
    }
    Frag<float> f;
    f.lo = f32x4{v[0], v[1], v[2], v[3]};
    f.hi = f32x4{v[4], v[5], v[6], v[7]};
    return f;
  }
};

__device__ __forceinline__ f32x4 mma(const Frag<bf16>& a, const Frag<bf16>& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, c, 0, 0, 0);
}
// One block-scaled fp8 MFMA over a 128-B K-step (VITMI_BF16F8): the two bf16 fragments of the
// step (ks = 0, 1) ARE its 32 e4m3 bytes per lane.  Their k order (chunks lg and 4 + lg of the
// 128-B row) differs from the instruction's (32 consecutive k per lane group), but A and B use the
// same one and the scales are uniform, so the dot product is the same.  Scale 2^-9 on the first
// operand (the weight side: exactly one factor of each product is a lo8 = lo * 2^9), 1 on the other.
typedef int i32x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x4 mma8(const Frag<bf16>& a0, const Frag<bf16>& a1, const Frag<bf16>& b0,
                                      const Frag<bf16>& b1, f32x4 c) {
  const i32x8 a = __builtin_bit_cast(i32x8, __builtin_shufflevector(a0.v, a1.v, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11,
                                                                    12, 13, 14, 15));
  const i32x8 b = __builtin_bit_cast(i32x8, __builtin_shufflevector(b0.v, b1.v, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11,
                                                                    12, 13, 14, 15));
#ifdef VITMI_F6_TIMING   // DIAGNOSTIC: the same bytes read as e2m3 (MX FP6 rate); results meaningless
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 2, 2, 0, F8_E8M0_LO, 0, F8_E8M0_ONE);
#else
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, F8_E8M0_LO, 0, F8_E8M0_ONE);
#endif
}
__device__ __forceinline__ f32x4 mma(const Frag<float>& a, const Frag<float>& b, f32x4 c) {
#pragma unroll
  for (int j = 0; j < 4; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo[j], b.lo[j], c, 0, 0, 0);
#pragma unroll
  for (int j = 0; j < 4; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi[j], b.hi[j], c, 0, 0, 0);
  return c;
}

// ---- epilogue ----------------------------------------------------------------
template <typename T, typename TC, int EPI>
__device__ __forceinline__ void epi_store(const GemmArgs& g, int64_t row, int64_t col, float acc,
                                          float biasv) {
  if constexpr (EPI == EPI_GELU_DROP) {
    const float u = acc + biasv, f = drop_factor(g, row, col);
    ((T*)g.aux)[aux_at(g, row, col)] = from_f32<T>(gelu_grad_f(u) * f);
    ((TC*)g.C)[row * g.ldc + col] = from_f32<TC>(gelu_f(u) * f);
  } else if constexpr (EPI == EPI_RESIDUAL_DROP) {
    ((float*)g.C)[row * g.ldc + col] = g.residual[row * g.ldr + col] + (acc + biasv) * drop_factor(g, row, col);
  } else if constexpr (EPI == EPI_PARTIAL) {
    ((float*)g.C)[blockIdx.z * g.split_stride + row * g.ldc + col] = acc;
  } else if constexpr (EPI == VITMI_EPI_STORE) {
    ((TC*)g.C)[row * g.ldc + col] = from_f32<TC>(acc + biasv);
  } else if constexpr (EPI == VITMI_EPI_BIAS_GELU) {
    const float u = acc + biasv;
    ((T*)g.aux)[aux_at(g, row, col)] = from_f32<T>(gelu_grad_f(u));
    ((TC*)g.C)[row * g.ldc + col] = from_f32<TC>(gelu_f(u));
  } else if constexpr (EPI == EPI_GELU_X3) {
    const float u = acc + biasv, a = gelu_f(u);
    const bf16 hi = (bf16)a;
    bf16* c = (bf16*)g.C + row * g.ldc + col;
    ((T*)g.aux)[aux_at(g, row, col)] = from_f32<T>(gelu_grad_f(u));
    c[0] = hi;
    c[g.N] = hi;
    c[2 * g.N] = (bf16)(a - (float)hi);
  } else if constexpr (EPI == VITMI_EPI_RESIDUAL) {
    ((float*)g.C)[row * g.ldc + col] = g.residual[row * g.ldr + col] + acc + biasv;
  } else if constexpr (EPI == VITMI_EPI_DGELU) {
    const float gp = to_f32(((const T*)g.aux)[aux_at(g, row, col)]);
    ((TC*)g.C)[row * g.ldc + col] = from_f32<TC>(acc * gp);
  } else if constexpr (EPI == VITMI_EPI_ACCUM) {
    ((float*)g.C)[row * g.ldc + col] += acc;
  }
}

// ---- the kernel ------------------------------------------------------------
template <typename T, bool AK, bool BKM, int EPI, typename TC, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(WM* WN * 64) void gemm_kernel(GemmArgs g) {
  constexpr int ES = TT<T>::ES, BK = TT<T>::BK;
  constexpr int NW = WM * WN;
  constexpr int A_BYTES = BM * BK * ES, B_BYTES = BN * BK * ES;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  // bf16 outputs of the store / GELU / DGELU epilogues: MFMA operands swapped (C^T in the
  // accumulator, as in gemm256), so a lane owns 4 consecutive columns of one row and stores them
  // as one 8-byte vector instead of four 2-byte scalars (the CvT's K = 64 stage-1 MLP GEMMs)
  constexpr bool SWP = std::is_same<T, bf16>::value && std::is_same<TC, bf16>::value &&
                       (EPI == VITMI_EPI_STORE || EPI == VITMI_EPI_BIAS_GELU || EPI == VITMI_EPI_DGELU);
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN, wn = wave % WN;

  const int tile = blockIdx.x;
  const int tm_i = tile / g.tiles_n, tn_i = tile % g.tiles_n;
  const int64_t m0 = (int64_t)tm_i * BM, n0 = (int64_t)tn_i * BN;
  const int64_t kb = (int64_t)blockIdx.z * g.k_per_split;
  const int64_t ke = min(g.K, kb + g.k_per_split);
  const int nk = (int)((ke - kb + BK - 1) / BK);

  // buffer descriptors rebased at this block's panel (range check = zero fill)
  __amdgpu_buffer_rsrc_t ra, rb;
  if (AK) {
    const char* base = (const char*)g.A + m0 * g.lda * ES;
    ra = make_rsrc(base, clamp_bytes((g.M - m0) * g.lda * ES));
  } else {
    const char* base = (const char*)g.A + (kb * g.lda + m0) * ES;
    ra = make_rsrc(base, clamp_bytes(((g.K - kb) * g.lda - m0) * ES));
  }
  if (BKM) {
    const char* base = (const char*)g.B + n0 * g.ldb * ES;
    rb = make_rsrc(base, clamp_bytes((g.N - n0) * g.ldb * ES));
  } else {
    const char* base = (const char*)g.B + (kb * g.ldb + n0) * ES;
    rb = make_rsrc(base, clamp_bytes(((g.K - kb) * g.ldb - n0) * ES));
  }

  auto stage = [&](int t, int buf) {
    char* sa = smem + buf * STAGE;
    char* sb = sa + A_BYTES;
    if (AK) stage_kmajor<T, BM, NW>(sa, ra, g.lda, kb + (int64_t)t * BK, wave, lane);
    else stage_mnmajor<T, BM, NW>(sa, ra, g.lda, (int64_t)t * BK, wave, lane);
    if (BKM) stage_kmajor<T, BN, NW>(sb, rb, g.ldb, kb + (int64_t)t * BK, wave, lane);
    else stage_mnmajor<T, BN, NW>(sb, rb, g.ldb, (int64_t)t * BK, wave, lane);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    if (t + 1 < nk) stage(t + 1, buf ^ 1);
    const char* sa = smem + buf * STAGE;
    const char* sb = sa + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      Frag<T> af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = FragReader<T, AK, BM>::read(sa, wm * (BM / WM) + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = FragReader<T, BKM, BN>::read(sb, wn * (BN / WN) + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = SWP ? mma(bfr[j], af[i], acc[i][j]) : mma(af[i], bfr[j], acc[i][j]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  if constexpr (SWP) {
    // C^T layout: row = lane & 15, columns 4 * (lane >> 4) + 0..3
    const int rl = lane & 15, cq = 4 * (lane >> 4);
    const bool vst = (g.ldc & 3) == 0 && ((uintptr_t)g.C & 7) == 0;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int64_t col0 = n0 + wn * (BN / WN) + j * 16 + cq;
      if (col0 >= g.N) continue;
      float bv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[e] = (g.bias && EPI != VITMI_EPI_DGELU && col0 + e < g.N) ? g.bias[col0 + e] : 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int64_t row = m0 + wm * (BM / WM) + i * 16 + rl;
        if (row >= g.M) continue;
        if (vst && col0 + 4 <= g.N) {
          bf16x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float v = acc[i][j][e];
            if constexpr (EPI == VITMI_EPI_STORE) {
              o[e] = (bf16)(v + bv[e]);
            } else if constexpr (EPI == VITMI_EPI_BIAS_GELU) {
              const float u = v + bv[e];
              ((T*)g.aux)[aux_at(g, row, col0 + e)] = from_f32<T>(gelu_grad_f(u));
              o[e] = (bf16)gelu_f(u);
            } else {   // DGELU
              o[e] = (bf16)(v * to_f32(((const T*)g.aux)[aux_at(g, row, col0 + e)]));
            }
          }
          *(bf16x4*)((bf16*)g.C + row * g.ldc + col0) = o;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (col0 + e < g.N) epi_store<T, TC, EPI>(g, row, col0 + e, acc[i][j][e], bv[e]);
        }
      }
    }
    return;
  }

  // epilogue: C layout of 16x16 MFMA: col = lane&15, row = 4*(lane>>4) + i
  const int cl = lane & 15, rg = 4 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int64_t col = n0 + wn * (BN / WN) + j * 16 + cl;
    if (col >= g.N) continue;
    const float bv = (g.bias && EPI != EPI_PARTIAL && EPI != VITMI_EPI_ACCUM &&
                      EPI != VITMI_EPI_DGELU) ? g.bias[col] : 0.f;   // (the *_DROP ones have bias)
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm * (BM / WM) + i * 16 + rg + r;
        if (row < g.M) epi_store<T, TC, EPI>(g, row, col, acc[i][j][r], bv);
      }
    }
  }
}

// =============================================================================
// gemm256: the bf16 workhorse.  256x256 block tile, BK = 64, 8 waves (2 along M x
// 4 along N, 128x64 outputs each), one block per CU (LDS 136 KiB).
//
// Each operand tile is held as two 16 KiB "half" sub-images so that one wave
// quadrant (64 rows x 32 cols x K64 = 16 MFMAs) needs exactly one A half and one
// B half.  A half h holds tile rows {128*w + 64*h + i}, B half h holds tile cols
// {64*w + 32*h + i}.  A K-tile runs in 4 phases over the quadrants
//   p0 (A0,B0)  p1 (A0,B1)  p2 (A1,B1)  p3 (A1,B0)
// (A fragments re-used p0->p1 and p2->p3, B p1->p2), and each phase issues ONE
// half-tile of the NEXT K-tile by LDS-DMA in the same order A0,B0,A1,B1 — so the
// only waits are a counted `s_waitcnt vmcnt(2)` after p0 and `vmcnt(4)` after p3;
// DMA stays in flight across the raw `s_barrier`s (cdna_hip_programming.md §5
// "Pipelining across barriers", 8-phase template T3/T4/T5).
// Block ids are remapped so consecutive tiles of one XCD share an A row panel.
// =============================================================================
// row groups per load batch of the loading epilogues (fp32 residual+accum; DGELU loads all 8)
#ifndef VITMI_EPI_RB_BF16
#define VITMI_EPI_RB_BF16 8
#endif
#ifndef VITMI_EPI_RB_F32
#define VITMI_EPI_RB_F32 4
#endif
namespace g256 {
// raw s_barrier that the compiler may not move memory operations across; DMA (vmcnt)
// stays in flight (a __syncthreads() would drain it).
__device__ __forceinline__ void barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
constexpr int BM = 256, BN = 256, BK = 64, NWAVES = 8;
constexpr int HALF = 16384;                 // bytes per half sub-image
constexpr int STAGE = 4 * HALF;             // A0 A1 B0 B1
// epilogue staging image per wave: 16 rows x 64 bf16 at a 144-B pitch (36 dwords: the 16 rows
// of a ds_write_b64 lane group start on distinct even banks, conflict free)
constexpr int EPI_PITCH = 144;
constexpr int EPI_SCR = 16 * EPI_PITCH;

// tile line of sub-image line i in half h: A (blocks of 64 per wave-row), B (blocks of 32)
template <bool IS_A>
__device__ __forceinline__ int line_of(int i, int h) {
  return IS_A ? ((i >> 6) << 7) + (h << 6) + (i & 63) : ((i >> 5) << 6) + (h << 5) + (i & 31);
}

// Issue the LDS-DMA of one half sub-image (16 pieces of 1 KiB, 2 per wave).
template <bool IS_A, bool KMAJ>
__device__ __forceinline__ void stage_half(char* sub, __amdgpu_buffer_rsrc_t rs, int64_t ld,
                                           int64_t k0, int krow0, int h, int wave, int lane) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int p = wave + NWAVES * j;
    uint32_t voff;
    if (KMAJ) {  // image [128 lines][64 k], 128-B rows
      const int i = p * 8 + (lane >> 3);
      const int c = (lane & 7) ^ swz_k(i);
      voff = (uint32_t)((int64_t)line_of<IS_A>(i, h) * ld * 2 + k0 * 2 + c * 16);
    } else {     // image [64 k][128 lines], 256-B rows
      const int r = p * 4 + (lane >> 4);
      const int c = (lane & 15) ^ swz_mn(r);
      voff = (uint32_t)((int64_t)(krow0 + r) * ld * 2 + (int64_t)line_of<IS_A>(c * 8, h) * 2);
    }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(void, sub + p * 1024), 16, voff, 0, 0, 0);
  }
}
}  // namespace g256

// GELU and gelu' of a fragment's four columns, erf by Abramowitz-Stegun 7.1.26 (|error| <=
// 1.5e-7: one exp, one rcp, 5 FMAs; used only where the result is rounded to bf16, the fp32
// path keeps erff).  Written on f32x4 so that everything but the rcp / exp / |x| / sign steps
// issues as packed v_pk_* pairs, the two independent halves of every step alternating (a packed
// result consumed by the very next instruction costs an s_nop): 12 VALU per element instead of
// 16 (the fc1 epilogue is VALU-bound; fc1 + GELU 334 -> 328 us at 14).  0.5*erf comes directly
// from coefficients pre-scaled by 0.5 (exact), the sign by copysign (v_bfi).
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

// Persistent variant: gridDim.x blocks (<= one per CU) walk the tiles; blocks with equal
// blockIdx.x % 8 (one XCD under round-robin dispatch) take consecutive tiles of one
// contiguous range, so the XCD's concurrent tiles share A row panels in its L2.  The last
// K-step of a tile prefetches K-step 0 of the block's next tile, so that DMA overlaps the
// epilogue.  MFMA operands are swapped (B first): the 16x16 accumulator then holds C^T,
// i.e. every lane owns 4 consecutive output COLUMNS of one row -> 8/16-byte vector stores
// straight from registers.
//
// The staggered ("ping-pong") K-loop.  A workgroup's waves w and w+4 share a SIMD.
// Waves 4..7 run one barrier behind waves 0..3, and every phase is
//     load section:  ds_read this phase's fragments, issue one half-tile LDS-DMA of the
//                    next K-step, counted vmcnt;
//     s_barrier;  compute section: lgkmcnt(0), 16 MFMAs;  s_barrier
// so in every barrier interval one wave of each SIMD is in its MFMA section while its
// partner is in its load section: the matrix pipe stays busy and the LDS reads of one
// wave hide under the partner's MFMAs (cdna_hip_programming.md §5, "The 256² 8-phase
// template"; MI355X_MICROARCH.md "Two waves per SIMD").
// Step s (buffer b = s&1) reads A0,B0 @P0, B1 @P1, A1 @P2, nothing @P3 (B0 stays in
// registers).  Each half is refilled two phases after its last read (the WAR rule once the
// reads were retired by an lgkmcnt before the reading phase's compute section): P0 DMAs
// B1(s+1), P1 A1(s+1) into b^1, P2 A0(s+2), P3 B0(s+2) into b, so four half-tiles (8
// LDS-DMA instructions per wave) are always in flight and each lands ~5 phases before it
// is read.  The stream of steps runs across tile boundaries (the next tile's steps 0/1).
// Waits: vmcnt(8) at P0 retires B1(s), at P1 A1(s), at P3 A0(s+1),B0(s+1); each sits
// before a barrier that the later reader passes, with one barrier of slack for the
// staggered group.
template <bool AK, bool BKM, int EPI, typename TC, bool F8 = false, bool GRP = false>
__global__ __launch_bounds__(512) void gemm256_kernel(GemmArgs g, int nwg) {
  using namespace g256;
  // two DMA stages + the bias of the current and the next tile (fp32, double-buffered) + one
  // per-wave image of a 16-row group of the output, through which bf16 epilogue stores leave
  // as whole 128-B lines
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + 2048 + NWAVES * EPI_SCR];
  constexpr int EB = EpiOf<EPI>::base;         // public epilogue (the *_DROP ones extend one)
  constexpr bool DROP = EpiOf<EPI>::drop;
  constexpr bool HAS_BIAS = EB == VITMI_EPI_STORE || EB == VITMI_EPI_BIAS_GELU || EB == VITMI_EPI_RESIDUAL;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;

  // tile range of this block's XCD group, and the block's stride inside it
  const int G = gridDim.x;
  const int xcd = blockIdx.x & 7, jx = blockIdx.x >> 3;
  const int gq = G >> 3, gr = G & 7;
  const int nbx = gq + (xcd < gr ? 1 : 0);              // blocks in this group
  // Each XCD group owns a contiguous range of the whole tiles AND an equal share of the
  // tail-split units (work-balanced; consecutive whole tiles share A panels in the XCD's
  // L2).  Sequence index i of a block runs jx, jx + nbx, ... over [0, nf + ns).
  const int ns_all = nwg - g.t_full;
  const int q1 = g.t_full >> 3, r1 = g.t_full & 7;
  const int f_b = xcd < r1 ? xcd * (q1 + 1) : r1 * (q1 + 1) + (xcd - r1) * q1;
  const int nf = q1 + (xcd < r1 ? 1 : 0);
  const int q2 = ns_all >> 3, r2 = ns_all & 7;
  const int s_b = xcd < r2 ? xcd * (q2 + 1) : r2 * (q2 + 1) + (xcd - r2) * q2;
  const int nseq = nf + q2 + (xcd < r2 ? 1 : 0);
  auto unit_at = [&](int i) { return i < nf ? f_b + i : g.t_full + s_b + (i - nf); };

  const int64_t kb = (int64_t)blockIdx.z * g.k_per_split;
  const int64_t ke = min(g.K, kb + g.k_per_split);
  const int nk = (int)((ke - kb + BK - 1) / BK);
  if (nk <= 0) return;

  // Operand descriptors with the unit's first k (kb + ks0 K-steps) baked into the base, so
  // the DMA issue only needs the unit-relative K-step.
  // (GRP: problem p's operands; otherwise g's)
  auto rsrc_a = [&](int64_t m0, int ks0, [[maybe_unused]] int p = 0) {
    const int64_t k = kb + (int64_t)ks0 * BK;
    const char* A = (const char*)(GRP ? g.grp[p].A : g.A);
    const int64_t lda = GRP ? g.grp[p].lda : g.lda, M = GRP ? g.grp[p].M : g.M;
    return AK ? make_rsrc(A + (m0 * lda + k) * 2, clamp_bytes((M - m0) * lda * 2 - k * 2))
              : make_rsrc(A + (k * lda + m0) * 2, clamp_bytes(((g.K - k) * lda - m0) * 2));
  };
  auto rsrc_b = [&](int64_t n0, int ks0, [[maybe_unused]] int p = 0) {
    const int64_t k = kb + (int64_t)ks0 * BK;
    const char* B = (const char*)(GRP ? g.grp[p].B : g.B);
    const int64_t ldb = GRP ? g.grp[p].ldb : g.ldb, N = GRP ? g.grp[p].N : g.N;
    return BKM ? make_rsrc(B + (n0 * ldb + k) * 2, clamp_bytes((N - n0) * ldb * 2 - k * 2))
               : make_rsrc(B + (k * ldb + n0) * 2, clamp_bytes(((g.K - k) * ldb - n0) * 2));
  };
  // unit u -> tile origin, first K-step and K-step count
  auto unit_of = [&](int u, int64_t& m0_, int64_t& n0_, int& ks0_, int& nk_, int& z_, [[maybe_unused]] int& p_) {
    int tl = u;
    ks0_ = 0;
    nk_ = nk;
    z_ = 0;
    if (EPI == EPI_PARTIAL && g.kz > 1) {
      z_ = u / g.ntiles;
      tl = u - z_ * g.ntiles;
      ks0_ = z_ * g.kz_steps;
      nk_ = min(g.kz_steps, nk - ks0_);
    } else if (u >= g.t_full) {
      const int v = u - g.t_full;
      tl = g.t_full + v / g.nsplit;
      ks0_ = (v % g.nsplit) * g.ksplit;
      nk_ = min(g.ksplit, nk - ks0_);
    }
    int tm_, tn_;
    if constexpr (GRP) {
      // the problem whose tile range holds tl (wave-uniform)
      int p = 0;
#pragma unroll
      for (int q = 1; q < GRP_MAX; ++q)
        if (q < g.ngrp && tl >= g.grp[q].tile0) p = q;
      p_ = p;
      tl -= g.grp[p].tile0;
      tm_ = tl / g.grp[p].tiles_n;
      tn_ = tl - tm_ * g.grp[p].tiles_n;
    } else {
      tile_rc(g, tl, tm_, tn_);
    }
    m0_ = (int64_t)tm_ * BM;
    n0_ = (int64_t)tn_ * BN;
  };
  auto sub = [&](int buf, int which) -> char* { return smem + buf * STAGE + which * HALF; };
  // issue half `which` (0=A0 1=B0 2=A1 3=B1) of K-step t into buffer buf
  // (la, lb: the row pitches of the unit the descriptors belong to; g's unless GRP)
  auto issue = [&](__amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, int t, int buf, int which,
                   int64_t la, int64_t lb) {
    const int64_t k0 = (int64_t)t * BK;   // relative to the descriptor's k
    const int krow0 = t * BK;
    if (which == 0) stage_half<true, AK>(sub(buf, 0), ra, la, k0, krow0, 0, wave, lane);
    if (which == 1) stage_half<false, BKM>(sub(buf, 2), rb, lb, k0, krow0, 0, wave, lane);
    if (which == 2) stage_half<true, AK>(sub(buf, 1), ra, la, k0, krow0, 1, wave, lane);
    if (which == 3) stage_half<false, BKM>(sub(buf, 3), rb, lb, k0, krow0, 1, wave, lane);
  };

  // Fragment registers, double-buffered so each phase's ds_reads overlap the previous
  // phase's MFMAs: A sets X/Y (A0 halves in X, A1 in Y); B sets 0/1 alternate per K-step
  // (B0 of a K-step is read once, used by p0 AND p3; B1 lives in the other set).
  Frag<bf16> ax[4][2], ay[4][2], b0[2][2], b1[2][2];
  f32x4 acc[8][4];
  // Lane-constant LDS offsets (the swizzles depend only on the lane, not on the fragment):
  //  k-major image [128][64]: frag (tile j, ks) at line w*TW + 16j + l15, chunk (4ks+g)^s,
  //    s = (l15>>1)&7  -> offset kofs[ks] + (w*TW + 16j)*128
  //  m/n-major image [64][128] (transposed reads): lane (t=l&15, g, q=t>>2, p=t&3) reads
  //    k-row ks*32 + 8g + 4i + q, chunk ((w*TW/8 + 2j + (p>>1)) ^ (2q + 8(g&1))) ->
  //    offset mofs[j] + (ks*32 + 4i)*256
  const int l15 = lane & 15, lg = lane >> 4, lq = l15 >> 2, lp = l15 & 3;
  int kofs[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) kofs[ks] = l15 * 128 + (((4 * ks + lg) ^ ((l15 >> 1) & 7)) << 4);
  auto mofs = [&](int cw, int j) {
    return (8 * lg + lq) * 256 + (((cw + 2 * j + (lp >> 1)) ^ (2 * lq + 8 * (lg & 1))) << 4) + (lp & 1) * 8;
  };
  int amofs[4], bmofs[2];
#pragma unroll
  for (int j = 0; j < 4; ++j) amofs[j] = mofs(wm * 8, j);
#pragma unroll
  for (int j = 0; j < 2; ++j) bmofs[j] = mofs(wn * 4, j);
  auto tr_read = [&](const char* p, int ofs) -> bf16x8 {
    bf16x8 f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, p + ofs + i * 1024));
      bf16x4 b = __builtin_bit_cast(bf16x4, v);
      f[4 * i + 0] = b[0]; f[4 * i + 1] = b[1]; f[4 * i + 2] = b[2]; f[4 * i + 3] = b[3];
    }
    return f;
  };
#define RD_A(DST, BUF, H)                                                                       \
  do {                                                                                          \
    const char* s_ = sub(BUF, H);                                                               \
    _Pragma("unroll") for (int mt = 0; mt < 4; ++mt)                                            \
    _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) {                                          \
      if constexpr (AK) DST[mt][ks].v = *(const bf16x8*)(s_ + kofs[ks] + (wm * 64 + 16 * mt) * 128); \
      else DST[mt][ks].v = tr_read(s_ + ks * 32 * 256, amofs[mt]);                              \
    }                                                                                           \
  } while (0)
#define RD_B(DST, BUF, H)                                                                       \
  do {                                                                                          \
    const char* s_ = sub(BUF, 2 + H);                                                           \
    _Pragma("unroll") for (int nt = 0; nt < 2; ++nt)                                            \
    _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) {                                          \
      if constexpr (BKM) DST[nt][ks].v = *(const bf16x8*)(s_ + kofs[ks] + (wn * 32 + 16 * nt) * 128); \
      else DST[nt][ks].v = tr_read(s_ + ks * 32 * 256, bmofs[nt]);                              \
    }                                                                                           \
  } while (0)
// In a unit's first K-step (FIRST) the ks = 0 MFMA of every accumulator starts from an inline
// zero C operand instead of an accumulator cleared by 128 v_mov per wave and tile
#define MMA4(MH, NH, AS, BS)                                                                    \
  do {                                                                                          \
    __builtin_amdgcn_s_setprio(1);                                                              \
    _Pragma("unroll") for (int mt = 0; mt < 4; ++mt)                                            \
    _Pragma("unroll") for (int nt = 0; nt < 2; ++nt)                                            \
    _Pragma("unroll") for (int ks = 0; ks < 2; ++ks)                                            \
      acc[MH * 4 + mt][NH * 2 + nt] = mma(BS[nt][ks], AS[mt][ks],                               \
          FIRST && ks == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[MH * 4 + mt][NH * 2 + nt]);         \
    __builtin_amdgcn_s_setprio(0);                                                              \
  } while (0)
// the fp8 K-steps of a VITMI_BF16F8 GEMM: one scaled MFMA per (mt, nt) over the step's 128 bytes
#define MMA4F8(MH, NH, AS, BS)                                                                  \
  do {                                                                                          \
    __builtin_amdgcn_s_setprio(1);                                                              \
    _Pragma("unroll") for (int mt = 0; mt < 4; ++mt)                                            \
    _Pragma("unroll") for (int nt = 0; nt < 2; ++nt)                                            \
      acc[MH * 4 + mt][NH * 2 + nt] = mma8(BS[nt][0], BS[nt][1], AS[mt][0], AS[mt][1],           \
          FIRST ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[MH * 4 + mt][NH * 2 + nt]);                   \
    __builtin_amdgcn_s_setprio(0);                                                              \
  } while (0)

  int it = jx;
  if (it >= nseq) return;
  int tile = unit_at(it);   // work unit (a whole tile, or a K-range of a tail tile)
  int64_t m0, n0;
  int ks0, nku, zs, pc = 0;
  unit_of(tile, m0, n0, ks0, nku, zs, pc);
  __amdgpu_buffer_rsrc_t ra = rsrc_a(m0, ks0, pc), rb = rsrc_b(n0, ks0, pc);
  int64_t la = GRP ? g.grp[pc].lda : g.lda, lb = GRP ? g.grp[pc].ldb : g.ldb;
  int buf = 0;
  // steps 0 and 1 of the first unit in the loop's issue order (nk >= 2 is a precondition)
  issue(ra, rb, 0, 0, 0, la, lb); issue(ra, rb, 0, 0, 1, la, lb); issue(ra, rb, 0, 0, 3, la, lb);
  issue(ra, rb, 0, 0, 2, la, lb);
  issue(ra, rb, 1, 1, 0, la, lb); issue(ra, rb, 1, 1, 1, la, lb);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");      // A0(0), B0(0) landed
  barrier();
  if (wm) barrier();                                     // waves 4..7 one barrier behind

  const int lc4 = 4 * (lane >> 4), lr = lane & 15;
  const __amdgpu_buffer_rsrc_t rbias = make_rsrc(g.bias, g.bias ? clamp_bytes(g.N * 4) : 0u);
  int tpar = 0;   // bias buffer of the current tile
  // vector-memory ops the previous unit's epilogue issued (0: none yet).  Those are younger
  // than the half-tiles the first K-step waits for, so its counts may grow by that many.
  int ep_ops = 0;
#ifdef VITMI_GEMM_STAMPS
  // [block][iter][wave-half][8]: K-loop start, epilogue start, epilogue end (s_memtime), then
  // s_memrealtime (100 MHz) at the same three points: the in-kernel clock of each K-loop
  int st_it = 0;
  auto stamp = [&](int k) {
    if (g.stamps && lane == 0 && (wave == 0 || wave == 4) && st_it < 16) {
      unsigned long long* p_ = g.stamps + ((blockIdx.x * 16 + st_it) * 2 + (wave >> 2)) * 8;
      p_[k] = __builtin_amdgcn_s_memtime();
      p_[3 + k] = __builtin_amdgcn_s_memrealtime();
    }
  };
#else
  auto stamp = [&](int) {};
#endif
  for (;;) {
    stamp(0);
    if constexpr (HAS_BIAS) {
      // bias[n0 .. n0+256) -> LDS by ONE LDS-DMA instruction of wave 0 (64 lanes x 16 B; the
      // range check zero-fills columns >= N and a null bias).  It is older than every DMA the
      // K-loop waits for, so it only makes those counted waits stricter; the epilogue reads it
      // many barriers later.
      if (wave == 0)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rbias, LDS_PTR(void, smem + 2 * STAGE + tpar * 1024), 16,
                                                 (uint32_t)(n0 * 4 + lane * 16), 0, 0, 0);
    }
    const int itn = it + nbx;
    const bool has_next = itn < nseq;
    const int next = has_next ? unit_at(itn) : 0;
    int64_t m0n = 0, n0n = 0;
    int ks0n = 0, nkn = 0, zsn = 0, pn = 0;
    if (has_next) unit_of(next, m0n, n0n, ks0n, nkn, zsn, pn);
    const __amdgpu_buffer_rsrc_t ran = rsrc_a(m0n, ks0n, pn), rbn = rsrc_b(n0n, ks0n, pn);
    const int64_t lan = GRP ? g.grp[pn].lda : g.lda, lbn = GRP ? g.grp[pn].ldb : g.ldb;

      // vmcnt counts of the first step after an epilogue that issued S vector-memory ops:
      // 8 + S (capped at the counter's 63): S = 16 (bf16 store), 32 (GELU, fp32 store, split
      // partials), 48 (DGELU), 64 (residual / accumulate).  An op issued after the awaited DMA
      // stays outstanding while it does (in-order completion), so 8 + S is the loosest exact wait.
#define WAITV(N) asm volatile("s_waitcnt vmcnt(%0)" :: "i"(N) : "memory")
#define WAITF() do { if (fst >= 55) WAITV(63); else if (fst == 48) WAITV(56); else if (fst == 32) WAITV(40); \
                     else if (fst == 16) WAITV(24); else WAITV(8); } while (0)
#define COMPUTE(MH, NH, AS, BS)                                                                 \
      do {                                                                                      \
        barrier();                                                                              \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                      \
        if constexpr (F8STEP) MMA4F8(MH, NH, AS, BS);                                           \
        else MMA4(MH, NH, AS, BS);                                                              \
        barrier();                                                                              \
      } while (0)
      // one K-step; FIRST (step 0 of the unit, peeled) starts the accumulators from zero
      // STEADY: t + 2 < nku is known (both prefetched steps belong to this unit), so the
      // descriptor / step selects below fold away (≈ 40 scalar instructions per K-step)
      auto kstep = [&](auto first_tag, auto steady_tag, auto f8_tag, const int t) {
        constexpr bool FIRST = decltype(first_tag)::value;
        constexpr bool STEADY = decltype(steady_tag)::value;
        constexpr bool F8STEP = decltype(f8_tag)::value;   // an e4m3 K-step (VITMI_BF16F8)
        // step t+1 (B1, A1 still to issue, buffer buf^1) and step t+2 (A0, B0, buffer buf)
        const bool in1 = STEADY || t + 1 < nku, in2 = STEADY || t + 2 < nku;
        const bool h1 = in1 || has_next, h2 = in2 || has_next;
        const __amdgpu_buffer_rsrc_t a1 = in1 ? ra : ran, b1r = in1 ? rb : rbn;
        const __amdgpu_buffer_rsrc_t a2 = in2 ? ra : ran, b2r = in2 ? rb : rbn;
        const int64_t la1 = !GRP ? g.lda : in1 ? la : lan, lb1 = !GRP ? g.ldb : in1 ? lb : lbn;
        const int64_t la2 = !GRP ? g.lda : in2 ? la : lan, lb2 = !GRP ? g.ldb : in2 ? lb : lbn;
        const int t1 = in1 ? t + 1 : 0, t2 = in2 ? t + 2 : t + 2 - nku;
        const int fst = FIRST ? ep_ops : 0;
        // P0 (A0,B0): DMA B1(t+1); retire B1(t)
        RD_A(ax, buf, 0);
        RD_B(b0, buf, 0);
        if (h1) {
          issue(a1, b1r, t1, buf ^ 1, 3, la1, lb1);
          WAITF();
        } else {
          WAITV(0);
        }
        COMPUTE(0, 0, ax, b0);
        // P1 (A0,B1): DMA A1(t+1); retire A1(t)
        RD_B(b1, buf, 1);
        if (h1) {
          issue(a1, b1r, t1, buf ^ 1, 2, la1, lb1);
          WAITF();
        } else {
          WAITV(0);
        }
        COMPUTE(0, 1, ax, b1);
        // P2 (A1,B1): DMA A0(t+2) into the half read at P0
        RD_A(ay, buf, 1);
        if (h2) issue(a2, b2r, t2, buf, 0, la2, lb2);
        COMPUTE(1, 1, ay, b1);
        // P3 (A1,B0): DMA B0(t+2); retire A0(t+1), B0(t+1)
        if (h2) {
          issue(a2, b2r, t2, buf, 1, la2, lb2);
          WAITF();
        } else {
          WAITV(0);
        }
        COMPUTE(1, 0, ay, b0);
        buf ^= 1;
      };
      if constexpr (F8) {
        // K-steps [0, t8) of this unit are bf16, [t8, nku) e4m3 (wave-uniform)
        const int t8 = max(0, min(nku, g.k8 - ks0 - (int)(kb / BK)));
        if (t8 > 0) kstep(std::true_type{}, std::false_type{}, std::false_type{}, 0);
        else kstep(std::true_type{}, std::false_type{}, std::true_type{}, 0);
        int t = 1;
        for (; t < t8 && t + 2 < nku; ++t) kstep(std::false_type{}, std::true_type{}, std::false_type{}, t);
        for (; t < t8; ++t) kstep(std::false_type{}, std::false_type{}, std::false_type{}, t);
        for (; t + 2 < nku; ++t) kstep(std::false_type{}, std::true_type{}, std::true_type{}, t);
        for (; t < nku; ++t) kstep(std::false_type{}, std::false_type{}, std::true_type{}, t);
      } else {
        kstep(std::true_type{}, std::false_type{}, std::false_type{}, 0);
        int t = 1;
        for (; t + 2 < nku; ++t) kstep(std::false_type{}, std::true_type{}, std::false_type{}, t);
        for (; t < nku; ++t) kstep(std::false_type{}, std::false_type{}, std::false_type{}, t);
      }
#undef COMPUTE
#undef WAITF
#undef WAITV
#undef MMA4
#undef MMA4F8

    stamp(1);
    if constexpr (GRP) {
      // raw fp32 partial of slab zs into problem pc's slab area (row pitch N; rows >= M and
      // columns >= N dropped by the range check and the out-of-range voffset)
      const int64_t Mp = g.grp[pc].M, Np = g.grp[pc].N;
      const __amdgpu_buffer_rsrc_t rw =
          make_rsrc((char*)g.grp[pc].C + ((int64_t)zs * Mp * Np + m0 * Np + n0) * 4, clamp_bytes(((Mp - m0) * Np - n0) * 4));
      const uint32_t wbase = (uint32_t)(((wm * 128 + lr) * Np + wn * 64 + lc4) * 4);
      const int rs16 = (int)(16 * Np * 4);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const uint32_t vo = n0 + wn * 64 + ni * 16 + lc4 < Np ? wbase : 0x80000000u;
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
          asm volatile(VMEM_SGPR_GUARD "buffer_store_dwordx4 %0, %1, %2, %3 offen offset:%4\n\ts_nop 1"
                       :: "v"(acc[mi][ni]), "v"(vo), "s"(rw), "s"(mi * rs16), "i"(ni * 64) : "memory");
      }
    } else
    if ((EPI != EPI_PARTIAL || g.kz <= 1) && tile >= g.t_full) {
      // K-range of a tail tile: raw fp32 partial into its [256][256] slab
      const __amdgpu_buffer_rsrc_t rw = make_rsrc(g.tail_ws + (int64_t)(tile - g.t_full) * BM * BN, BM * BN * 4);
      const uint32_t wbase = (uint32_t)(((wm * 128 + lr) * BN + wn * 64 + lc4) * 4);
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          asm volatile(VMEM_SGPR_GUARD "buffer_store_dwordx4 %0, %1, %2, %3 offen offset:%4\n\ts_nop 1"
                       :: "v"(acc[mi][ni]), "v"(wbase), "s"(rw), "s"(mi * 16 * BN * 4), "i"(ni * 64) : "memory");
    } else
    // ---- epilogue straight from registers: acc[mi][ni] = C^T tile; lane owns row
    // m0 + wm*128 + mi*16 + lr, columns n0 + wn*64 + ni*16 + lc4 .. +3.
    // Stores are inline-asm buffer stores: hipcc would otherwise put `s_waitcnt vmcnt(0)`
    // before every store (it cannot prove C does not alias the in-flight DMA sources),
    // serialising the epilogue.  C never aliases A/B here (host contract).  The range
    // check drops rows >= M; the row offset is a scalar per mi, the column an immediate.
    {
      constexpr int CES = sizeof(TC) == 2 && EPI != EPI_PARTIAL && EB != VITMI_EPI_ACCUM &&
                                  EB != VITMI_EPI_RESIDUAL ? 2 : 4;
      int64_t zoff = 0;
      if constexpr (EPI == EPI_PARTIAL) zoff = (int64_t)(blockIdx.z + zs) * g.split_stride;
      char* cbase = (char*)g.C + (zoff + m0 * g.ldc + n0) * CES;
      const __amdgpu_buffer_rsrc_t rc = make_rsrc(cbase, clamp_bytes(((g.M - m0) * g.ldc - n0) * CES));
      // EPI_GELU_X3: the second hi copy at column N + c, lo at 2N + c
      [[maybe_unused]] __amdgpu_buffer_rsrc_t rc2 = rc, rc3 = rc;
      if constexpr (EPI == EPI_GELU_X3) {
        rc2 = make_rsrc(cbase + g.N * 2, clamp_bytes(((g.M - m0) * g.ldc - n0 - g.N) * 2));
        rc3 = make_rsrc(cbase + g.N * 4, clamp_bytes(((g.M - m0) * g.ldc - n0 - 2 * g.N) * 2));
      }
      // EPI_GELU_F8: the e4m3 part from byte 2N of the 4N-byte row, 64-column blocks [hi8 | lo8]
      // (common.h f8_off): a wave's 64 columns are one block, 128 B per row at 2 n0 + 128 wn --
      // the same byte offsets as its bf16 hi, so `flush` writes it unchanged from its own base
      if constexpr (EPI == EPI_GELU_F8)
        rc2 = make_rsrc((char*)g.C + m0 * g.ldc * 2 + 2 * g.N + n0 * 2,
                        clamp_bytes((g.M - m0) * g.ldc * 2 - 2 * g.N - n0 * 2));
      const int rstride = (int)(16 * g.ldc * CES);     // bytes between mi row groups
      const uint32_t vbase = (uint32_t)(((int64_t)(wm * 128 + lr) * g.ldc + wn * 64 + lc4) * CES);
      // Branch-free ragged N (straight-line epilogue code schedules far better): lanes past
      // N load from a clamped column and store to a voffset beyond the buffer range, so the
      // store is dropped (N % 8 == 0 is a gemm256 precondition).
      bool cok[4];
      uint32_t vb[4];
      int64_t colc[4];
      f32x4 bv[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int64_t col = n0 + wn * 64 + ni * 16 + lc4;
        cok[ni] = col < g.N;
        colc[ni] = cok[ni] ? col : g.N - 4;
        vb[ni] = cok[ni] ? vbase : 0x80000000u;
        bv[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (HAS_BIAS)
          bv[ni] = *(const f32x4*)(smem + 2 * STAGE + tpar * 1024 + (wn * 64 + ni * 16 + lc4) * 4);
      }
      [[maybe_unused]] __amdgpu_buffer_rsrc_t ru = rc;
      [[maybe_unused]] f32x4 csum[4] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f},
                                        f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
      if constexpr (EB == VITMI_EPI_BIAS_GELU)
        ru = g.aux_tiled ? make_rsrc((char*)g.aux + ((m0 >> 8) * g.tiles_n + (n0 >> 8)) * 131072, 131072u)
                         : make_rsrc((char*)g.aux + (m0 * g.ldaux + n0) * 2, clamp_bytes(((g.M - m0) * g.ldaux - n0) * 2));
      // bf16 outputs leave through the wave's LDS image of one 16-row group: each lane holds 4
      // columns of ONE row per fragment (16 rows x 32 B per store instruction: every store would
      // touch 16 lines with a quarter of each), so a row group is written to LDS and read back as
      // row-major 16-B chunks: 2 stores of 8 rows x 128 B, whole lines (epilogue 8.8k -> ~3k
      // cycles per tile measured with s_memtime stamps on the fc1 shape)
      [[maybe_unused]] char* scr = smem + 2 * STAGE + 2048 + wave * EPI_SCR;
      [[maybe_unused]] const int rr = lane >> 3, cc = lane & 7;
      [[maybe_unused]] const bool ccok = n0 + wn * 64 + cc * 8 < g.N;
      auto lds_put = [&](int ni, bf16x4 o) { *(bf16x4*)(scr + lr * EPI_PITCH + (ni * 16 + lc4) * 2) = o; };
      // Lanes exchange data through the image: a compiler barrier between one lane's LDS write
      // and another lane's read of it (no store-to-load forwarding or reordering across it; the
      // LDS executes one wave's accesses in order)
      auto lane_xchg = [] { asm volatile("" ::: "memory"); };
      // the image of row group mi -> rows m0 + wm*128 + 16 mi + (0..15) of the buffer `r` (bf16, ld)
      auto flush = [&](__amdgpu_buffer_rsrc_t r, int64_t ld, int mi, bool aux = false) {
        lane_xchg();
        bf16x8 d[2];
        uint32_t vo[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          d[j] = *(const bf16x8*)(scr + (8 * j + rr) * EPI_PITCH + cc * 16);
          vo[j] = ccok ? (uint32_t)(((int64_t)(wm * 128 + 8 * j + rr) * ld + wn * 64 + cc * 8) * 2) : 0x80000000u;
        }
        if (aux) {
          asm volatile(VMEM_SGPR_GUARD
                       "buffer_store_dwordx4 %0, %2, %4, %5 offen" VITMI_ST_AUX "\n\t"
                       "buffer_store_dwordx4 %1, %3, %4, %5 offen" VITMI_ST_AUX "\n\ts_nop 1"
                       :: "v"(__builtin_bit_cast(u32x4, d[0])), "v"(__builtin_bit_cast(u32x4, d[1])), "v"(vo[0]),
                          "v"(vo[1]), "s"(r), "s"((int)(mi * 16 * ld * 2))
                       : "memory");
        } else {
          asm volatile(VMEM_SGPR_GUARD
                       "buffer_store_dwordx4 %0, %2, %4, %5 offen" VITMI_ST_C16 "\n\t"
                       "buffer_store_dwordx4 %1, %3, %4, %5 offen" VITMI_ST_C16 "\n\ts_nop 1"
                       :: "v"(__builtin_bit_cast(u32x4, d[0])), "v"(__builtin_bit_cast(u32x4, d[1])), "v"(vo[0]),
                          "v"(vo[1]), "s"(r), "s"((int)(mi * 16 * ld * 2))
                       : "memory");
        }
        lane_xchg();   // and the next writes of the image stay after these reads
      };
      [[maybe_unused]] bf16x4 lo3[4];   // EPI_GELU_X3: lo = bf16(a - hi) of the row group's fragments
      [[maybe_unused]] uint32_t f8h[4], f8l[4];   // EPI_GELU_F8: hi8, lo8 (4 e4m3 each) of the fragments
      // one output fragment (row group mi, column group ni); `ld` = the epilogue's loaded operand.
      // Returns the fragment of the second output (gelu') for BIAS_GELU.
      auto emit = [&](int mi, int ni, f32x4 ldv, bf16x4 ldb) -> bf16x4 {
        [[maybe_unused]] bf16x4 u{};   // (gelu' of the GELU epilogues; unused otherwise)
        f32x4 v = acc[mi][ni] + bv[ni];
        const int soff = mi * rstride;
        [[maybe_unused]] f32x4 df;   // dropout factors of the 4 columns
        if constexpr (DROP) {
          const uint32_t rk = drop_row_key(g.drop_seed, g.drop_site, (uint32_t)(m0 + wm * 128 + mi * 16 + lr));
#pragma unroll
          for (int e = 0; e < 4; ++e)
            df[e] = drop_hash(rk, (uint32_t)(colc[ni] + e)) >= g.drop_thresh ? g.drop_scale : 0.f;
        }
        if constexpr (EPI == EPI_RESIDUAL_DROP) v = v * df + ldv;
        if constexpr (EPI == VITMI_EPI_RESIDUAL || EPI == VITMI_EPI_ACCUM) v += ldv;
        if constexpr (EB == VITMI_EPI_BIAS_GELU) {
          f32x4 a4, g4;                        // gelu(u), gelu'(u) (kept for DGELU)
          gelu4(v, a4, g4);
          v = a4;
          if constexpr (DROP) {                // dropped: a = gelu(u) m/(1-p), aux = gelu'(u) m/(1-p)
            v *= df;
            g4 *= df;
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) u[e] = (bf16)g4[e];
        } else if constexpr (EPI == VITMI_EPI_DGELU) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] *= (float)ldb[e];   // aux = gelu'(u) from the forward
          csum[ni] += v;                                       // rows >= M hold 0 (zero A rows)
        }
        if constexpr (CES == 4) {
          if constexpr (EPI == EPI_PARTIAL) {
            asm volatile(VMEM_SGPR_GUARD "buffer_store_dwordx4 %0, %1, %2, %3 offen offset:%4" VITMI_ST_PART "\n\ts_nop 1"
                         :: "v"(v), "v"(vb[ni]), "s"(rc), "s"(soff), "i"(ni * 64) : "memory");
          } else
            asm volatile(VMEM_SGPR_GUARD "buffer_store_dwordx4 %0, %1, %2, %3 offen offset:%4" VITMI_ST_C32 "\n\ts_nop 1"
                         :: "v"(v), "v"(vb[ni]), "s"(rc), "s"(soff), "i"(ni * 64) : "memory");
        } else {
          bf16x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = (bf16)v[e];
          lds_put(ni, o);
          if constexpr (EPI == EPI_GELU_X3) {
#pragma unroll
            for (int e = 0; e < 4; ++e) lo3[ni][e] = (bf16)(v[e] - (float)o[e]);
          }
          if constexpr (EPI == EPI_GELU_F8) {
            bf16x4 h_;
            split_f8(v, h_, f8h[ni], f8l[ni]);
          }
        }
        return u;
      };
      // all four column groups of row group mi: C (and gelu') through the LDS image
      auto emit_row = [&](int mi, const f32x4 (&ldv)[4], const bf16x4 (&ldb)[4]) {
        [[maybe_unused]] bf16x4 us[4];
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) us[ni] = emit(mi, ni, ldv[ni], ldb[ni]);
        if constexpr (CES == 2) {
          flush(rc, g.ldc, mi);
          if constexpr (EPI == EPI_GELU_X3) {   // the same image again at +N, then lo at +2N
            flush(rc2, g.ldc, mi);
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) lds_put(ni, lo3[ni]);
            flush(rc3, g.ldc, mi);
          }
          if constexpr (EPI == EPI_GELU_F8) {   // the [hi8 | lo8] block image, 128 B per row
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) {
              *(uint32_t*)(scr + lr * EPI_PITCH + ni * 16 + lc4) = f8h[ni];
              *(uint32_t*)(scr + lr * EPI_PITCH + 64 + ni * 16 + lc4) = f8l[ni];
            }
            flush(rc2, g.ldc, mi);
          }
          if constexpr (EB == VITMI_EPI_BIAS_GELU) {
            if (g.aux_tiled) {   // straight from the registers: 2 KiB-wide stores (aux_at)
              const u32x4 w0 = __builtin_bit_cast(u32x4, bf16x8{us[0][0], us[0][1], us[0][2], us[0][3],
                                                                us[1][0], us[1][1], us[1][2], us[1][3]});
              const u32x4 w1 = __builtin_bit_cast(u32x4, bf16x8{us[2][0], us[2][1], us[2][2], us[2][3],
                                                                us[3][0], us[3][1], us[3][2], us[3][3]});
              asm volatile(VMEM_SGPR_GUARD
                           "buffer_store_dwordx4 %0, %2, %3, %4 offen" VITMI_ST_AUX "\n\t"
                           "buffer_store_dwordx4 %1, %2, %3, %4 offen offset:1024" VITMI_ST_AUX "\n\ts_nop 1"
                           :: "v"(w0), "v"(w1), "v"((uint32_t)(wave * 16384 + lane * 16)), "s"(ru), "s"(mi * 2048)
                           : "memory");
            } else {
#pragma unroll
              for (int ni = 0; ni < 4; ++ni) lds_put(ni, us[ni]);
              flush(ru, g.ldaux, mi, true);
            }
          }
        }
      };
      if constexpr (EB == VITMI_EPI_RESIDUAL || EPI == VITMI_EPI_ACCUM || EPI == VITMI_EPI_DGELU) {
        // epilogues that load: RB row groups at a time (all 4 column groups each; 64 VGPRs of
        // loaded operand per wait -- the fragment registers are free here), stored row by row
        // like the store-only epilogues below
        constexpr int RB = EPI == VITMI_EPI_DGELU ? VITMI_EPI_RB_BF16 : VITMI_EPI_RB_F32;
        if constexpr (EPI == VITMI_EPI_DGELU) {
          // gelu'(u) arrives as whole 128-B lines too: each lane loads 16 B of one row (8 rows x
          // 128 B per instruction; a C^T-layout load would take 16 rows x 32 B), the wave writes
          // the 16-row group to its LDS image and reads it back in the accumulator's layout.
          // All 16 loads of the tile are issued first (64 VGPRs), the range check zero-fills
          // rows >= M.
          const __amdgpu_buffer_rsrc_t rx =
              make_rsrc((const char*)g.aux + (m0 * g.ldaux + n0) * 2, clamp_bytes(((g.M - m0) * g.ldaux - n0) * 2));
          u32x4 al[8][2];
          const f32x4 z4[4] = {};
          if (g.aux_tiled) {
            // tile-native gelu' (aux_at): the lane's own 16 B of each row group, no exchange.
            // Rows >= M of a tile may hold anything (the forward may have run the 128x128
            // kernel, which writes valid elements only): they are zeroed, so the fused column
            // sums see 0 * 0 there
            const __amdgpu_buffer_rsrc_t rxt =
                make_rsrc((const char*)g.aux + ((m0 >> 8) * g.tiles_n + (n0 >> 8)) * 131072, 131072u);
#pragma unroll
            for (int mi = 0; mi < 8; ++mi)
#pragma unroll
              for (int j = 0; j < 2; ++j)
                al[mi][j] = __builtin_amdgcn_raw_buffer_load_b128(rxt, (uint32_t)(wave * 16384 + lane * 16),
                                                                  mi * 2048 + j * 1024, 0);
#pragma unroll
            for (int mi = 0; mi < 8; ++mi) {
              const bool rok = m0 + wm * 128 + mi * 16 + lr < g.M;
              bf16x4 lb[4];
#pragma unroll
              for (int ni = 0; ni < 4; ++ni) {
                const bf16x8 w = __builtin_bit_cast(bf16x8, rok ? al[mi][ni >> 1] : u32x4{0u, 0u, 0u, 0u});
                const int o = (ni & 1) * 4;
                lb[ni] = bf16x4{w[o], w[o + 1], w[o + 2], w[o + 3]};
              }
              emit_row(mi, z4, lb);
            }
          } else {
#pragma unroll
            for (int mi = 0; mi < 8; ++mi)
#pragma unroll
              for (int j = 0; j < 2; ++j) {
                const uint32_t vo = ccok ? (uint32_t)(((int64_t)(wm * 128 + 8 * j + rr) * g.ldaux + wn * 64 + cc * 8) * 2)
                                         : 0x80000000u;
                al[mi][j] = __builtin_amdgcn_raw_buffer_load_b128(rx, vo, (int)(mi * 16 * g.ldaux * 2), 0);
              }
#pragma unroll
            for (int mi = 0; mi < 8; ++mi) {
#pragma unroll
              for (int j = 0; j < 2; ++j) *(u32x4*)(scr + (8 * j + rr) * EPI_PITCH + cc * 16) = al[mi][j];
              lane_xchg();
              bf16x4 lb[4];
#pragma unroll
              for (int ni = 0; ni < 4; ++ni) lb[ni] = *(const bf16x4*)(scr + lr * EPI_PITCH + (ni * 16 + lc4) * 2);
              lane_xchg();   // (the image is rewritten by emit_row after every lane's read)
              emit_row(mi, z4, lb);
            }
          }
        } else if constexpr (EB == VITMI_EPI_RESIDUAL) {
          // fp32 residual in, fp32 out, both as whole lines through the LDS image, half a row
          // group's columns (16 rows x 32 fp32 = one 128-B line per row) at a time: lane (rr8, c8)
          // moves 16 B of row 8j + rr8, then EVERY lane updates its two accumulator fragments of
          // that column half in place (a row-half split left half the lanes idle in each pass),
          // and the lines go back out.  Pitch 36 dwords: the 16 rows of a fragment access fall on
          // distinct bank quads.  RB row groups of loads in flight (64 VGPRs).
          constexpr int P32 = 144;   // 16 rows x 128 B at a 144-B pitch = the 2304-B image
          const int rr8 = lane >> 3, c8 = lane & 7;
          const __amdgpu_buffer_rsrc_t rres =
              make_rsrc((const char*)(g.residual + m0 * g.ldr + n0), clamp_bytes(((g.M - m0) * g.ldr - n0) * 4));
          auto vo32 = [&](int pp, int j, int64_t ld) -> uint32_t {
            const int col = wn * 64 + pp * 32 + c8 * 4;
            return n0 + col < g.N ? (uint32_t)(((int64_t)(wm * 128 + 8 * j + rr8) * ld + col) * 4) : 0x80000000u;
          };
#pragma unroll
          for (int mp = 0; mp < 8 / RB; ++mp) {
            u32x4 rl[RB][2][2];
#pragma unroll
            for (int h = 0; h < RB; ++h)
#pragma unroll
              for (int pp = 0; pp < 2; ++pp)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                  rl[h][pp][j] = __builtin_amdgcn_raw_buffer_load_b128(rres, vo32(pp, j, g.ldr),
                                                                       (int)((RB * mp + h) * 16 * g.ldr * 4), 0);
#pragma unroll
            for (int h = 0; h < RB; ++h) {
              const int mi = RB * mp + h;
#pragma unroll
              for (int pp = 0; pp < 2; ++pp) {
#pragma unroll
                for (int j = 0; j < 2; ++j) *(u32x4*)(scr + (8 * j + rr8) * P32 + c8 * 16) = rl[h][pp][j];
                lane_xchg();
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                  const int ni = 2 * pp + q;
                  f32x4* pr = (f32x4*)(scr + lr * P32 + (q * 16 + lc4) * 4);
                  f32x4 v = acc[mi][ni] + bv[ni];
                  if constexpr (DROP) {
                    const uint32_t rk = drop_row_key(g.drop_seed, g.drop_site, (uint32_t)(m0 + wm * 128 + mi * 16 + lr));
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                      v[e] *= drop_hash(rk, (uint32_t)(colc[ni] + e)) >= g.drop_thresh ? g.drop_scale : 0.f;
                  }
                  *pr = v + *pr;
                }
                lane_xchg();
                u32x4 d[2];
#pragma unroll
                for (int j = 0; j < 2; ++j) d[j] = *(const u32x4*)(scr + (8 * j + rr8) * P32 + c8 * 16);
                lane_xchg();   // every lane's read before the next pass rewrites the image
#pragma unroll
                for (int j = 0; j < 2; ++j)
                  asm volatile(VMEM_SGPR_GUARD "buffer_store_dwordx4 %0, %1, %2, %3 offen" VITMI_ST_C32 "\n\ts_nop 1"
                               :: "v"(d[j]), "v"(vo32(pp, j, g.ldc)), "s"(rc), "s"((int)(mi * 16 * g.ldc * 4))
                               : "memory");
              }
            }
          }
        } else
#pragma unroll
        for (int mp = 0; mp < 8 / RB; ++mp) {
          f32x4 ld4[RB][4];
          bf16x4 ldu[RB][4];
#pragma unroll
          for (int h = 0; h < RB; ++h) {
            const int64_t row = min(m0 + wm * 128 + (RB * mp + h) * 16 + lr, g.M - 1);
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) {
              if constexpr (EB == VITMI_EPI_RESIDUAL) ld4[h][ni] = *(const f32x4*)(g.residual + row * g.ldr + colc[ni]);
              if constexpr (EPI == VITMI_EPI_ACCUM) ld4[h][ni] = *(const f32x4*)((const float*)g.C + row * g.ldc + colc[ni]);
            }
          }
#pragma unroll
          for (int h = 0; h < RB; ++h) emit_row(RB * mp + h, ld4[h], ldu[h]);
        }
        if constexpr (EPI == VITMI_EPI_DGELU) {
          if (g.colsum) {
            // sum the wave's 128 rows: 8 row groups in registers (above), then the 16 lanes
            // of a column group (lane & 15 = row, one DPP row): four row_shr adds leave the sum
            // in lane 15 of the row (no LDS round trips, unlike ds_bpermute shuffles); lanes
            // 15/31/47/63 store 4 columns per ni
            auto row_shr_add = [](float x, auto n) {
              constexpr int N = decltype(n)::value;
              const int y = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x110 | N, 0xf, 0xf, true);
              return x + __builtin_bit_cast(float, y);   // lanes < N of the row add 0 (bound_ctrl)
            };
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                float x = csum[ni][e];
                x = row_shr_add(x, std::integral_constant<int, 1>{});
                x = row_shr_add(x, std::integral_constant<int, 2>{});
                x = row_shr_add(x, std::integral_constant<int, 4>{});
                x = row_shr_add(x, std::integral_constant<int, 8>{});
                csum[ni][e] = x;
              }
            const int64_t prow = (m0 / BM) * 2 + wm;
            const __amdgpu_buffer_rsrc_t rs = make_rsrc(g.colsum + prow * g.N + n0, clamp_bytes((g.N - n0) * 4));
            const uint32_t cb = lr == 15 ? (uint32_t)((wn * 64 + lc4) * 4) : 0x80000000u;
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
              asm volatile(VMEM_SGPR_GUARD "buffer_store_dwordx4 %0, %1, %2, 0 offen offset:%3\n\ts_nop 1"
                           :: "v"(csum[ni]), "v"(cok[ni] ? cb : 0x80000000u), "s"(rs), "i"(ni * 64) : "memory");
          }
        }
      } else {
        // store-only epilogues go row by row: the 4 column groups of a row (one 128-B line
        // for bf16) leave back to back, so the L2 sees whole lines
        const f32x4 z4[4] = {};
        const bf16x4 zb[4] = {};
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) emit_row(mi, z4, zb);
      }
    }
    stamp(2);
#ifdef VITMI_GEMM_STAMPS
    ++st_it;
#endif
    tpar ^= 1;
    // the epilogue just issued: 32 stores (store-only, split partials) or 64 ops
    {
      // bf16 outputs: 2 stores per row group (+2 for gelu'); fp32 outputs: 32 direct stores;
      // + 16 aux loads for DGELU, + 32 loads for residual / accumulate.  (DGELU's 4 column-sum
      // stores only make the waits below stricter.)
      constexpr int CES2 = sizeof(TC) == 2 && EPI != EPI_PARTIAL && EB != VITMI_EPI_ACCUM &&
                           EB != VITMI_EPI_RESIDUAL;
      constexpr int EP = CES2 ? (EPI == EPI_GELU_X3 ? 64 : EPI == EPI_GELU_F8 ? 48
                                 : EB == VITMI_EPI_BIAS_GELU || EPI == VITMI_EPI_DGELU ? 32 : 16)
                              : (EB == VITMI_EPI_RESIDUAL || EPI == VITMI_EPI_ACCUM ? 64
                                 : EPI == VITMI_EPI_DGELU ? 48 : 32);
      ep_ops = ((EPI != EPI_PARTIAL || g.kz <= 1) && tile >= g.t_full) ? 32 : EP;
    }
    if (!has_next) break;
    it = itn; tile = next; m0 = m0n; n0 = n0n; ks0 = ks0n; nku = nkn; zs = zsn; ra = ran; rb = rbn;
    if constexpr (GRP) {
      pc = pn;
      la = lan;
      lb = lbn;
    }
  }
  // the leading group owes the staggered group its extra barrier: equal counts per wave
  if (!wm) barrier();
#undef RD_A
#undef RD_B
#undef G256_MMA
}

// split-K reduction: dst[i] += sum_z ws[z][i]
// a + slab 0 + slab 1 + ... (this order) at float4 i: the loads of up to 8 slabs are issued
// together (a runtime loop of load-then-add waited for each one in turn, ~3 TB/s)
__device__ __forceinline__ f32x4 add_slabs(f32x4 a, const float* __restrict__ ws, int64_t stride, int64_t i,
                                           int splits) {
  for (int z0 = 0; z0 < splits; z0 += 8) {
    f32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (z0 + u < splits) v[u] = *(const f32x4*)(ws + (int64_t)(z0 + u) * stride + i);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (z0 + u < splits) a += v[u];
  }
  return a;
}

__global__ void splitk_reduce_kernel(const float* __restrict__ ws, float* __restrict__ dst,
                                     int64_t n, int splits, int64_t stride) {
  int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const int64_t step = (int64_t)gridDim.x * blockDim.x * 4;
  for (; i < n; i += step) {
    if (i + 4 <= n) {
      *(f32x4*)(dst + i) = add_slabs(*(const f32x4*)(dst + i), ws, stride, i, splits);
    } else {
      for (int64_t e = i; e < n; ++e) {
        float s = dst[e];
        for (int z = 0; z < splits; ++z) s += ws[z * stride + e];
        dst[e] = s;
      }
    }
  }
}

// The same for small outputs with many slabs (n / 4 <= SMALL_RED_MAX): 16 waves per block split
// the slabs (wave w sums z = w, w + 16, ...), then the 16 wave sums are added in wave order and
// onto dst.  Fixed order, deterministic; one lane per 4 elements would walk up to 512 slabs alone.
constexpr int64_t SMALL_RED_MAX = 16384;
__global__ __launch_bounds__(1024) void splitk_reduce_small_kernel(const float* __restrict__ ws, float* __restrict__ dst,
                                                                   int64_t n, int splits, int64_t stride) {
  __shared__ f32x4 red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t i = ((int64_t)blockIdx.x * 64 + lane) * 4;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (i + 4 <= n) {
#pragma unroll 8
    for (int z = w; z < splits; z += 16) s += *(const f32x4*)(ws + z * stride + i);
  } else if (i < n) {
    for (int z = w; z < splits; z += 16)
      for (int64_t e = i; e < n; ++e) s[e - i] += ws[z * stride + e];
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && i < n) {
    f32x4 t = red[0][lane];
#pragma unroll
    for (int k = 1; k < 16; ++k) t += red[k][lane];
    if (i + 4 <= n) {
      *(f32x4*)(dst + i) = *(const f32x4*)(dst + i) + t;
    } else {
      for (int64_t e = i; e < n; ++e) dst[e] += t[e - i];
    }
  }
}

// The grouped weight gradients' reduction: segment q (up to GRP_MAX, the problems of one grouped
// launch) adds its `splits` slabs at ws + off[q] (stride n[q]) onto dst[q], over one flat index space
// of float4 groups; per element dst + slab 0 + slab 1 + ... as splitk_reduce_kernel sums.
struct RedSegs {
  const float* ws[GRP_MAX];
  float* dst[GRP_MAX];
  int64_t n[GRP_MAX];
  int64_t g0[GRP_MAX + 1];   // first float4 group of each segment (prefix sums of ceil(n / 4))
  int nseg;
};
__global__ void splitk_reduce_group_kernel(RedSegs rs, int splits) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t gi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; gi < rs.g0[rs.nseg]; gi += step) {
    int q = 0;
#pragma unroll
    for (int j = 1; j < GRP_MAX; ++j)
      if (j < rs.nseg && gi >= rs.g0[j]) q = j;
    const int64_t i = (gi - rs.g0[q]) * 4, n = rs.n[q];
    const float* ws = rs.ws[q];
    float* dst = rs.dst[q];
    if (i + 4 <= n) {
      *(f32x4*)(dst + i) = add_slabs(*(const f32x4*)(dst + i), ws, n, i, splits);
    } else {
      for (int64_t e = i; e < n; ++e) {
        float a = dst[e];
        for (int z = 0; z < splits; ++z) a += ws[z * n + e];
        dst[e] = a;
      }
    }
  }
}

// Finish the tail tiles of a split gemm256 launch: sum the nsplit fp32 partials of each
// element and apply the epilogue (the elementwise epi_store of the 128x128 kernel).
template <typename T, typename TC, int EPI>
__global__ __launch_bounds__(256) void gemm_tail_fixup_kernel(GemmArgs g, int ntail) {
  const int64_t groups = (int64_t)ntail * (256 * 256 / 4);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < groups; i += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(i / (256 * 64));
    const int e = (int)(i % (256 * 64)) * 4;
    const int rl = e >> 8, cl = e & 255;
    const int tile = g.t_full + t;
    int tm, tn;
    tile_rc(g, tile, tm, tn);
    const int64_t row = (int64_t)tm * 256 + rl;
    const int64_t col = (int64_t)tn * 256 + cl;
    if (row >= g.M || col >= g.N) continue;
    const float* pw = g.tail_ws + ((int64_t)t * g.nsplit * 256 + rl) * 256 + cl;   // split z at + z * 65536
    f32x4 a = {0.f, 0.f, 0.f, 0.f};
    if (g.nsplit <= 4) {
      // every split's partial in flight at once (S <= 4 is the tail plan's cap), added in split order
      f32x4 pz[4];
#pragma unroll
      for (int z = 0; z < 4; ++z)
        if (z < g.nsplit) pz[z] = *(const f32x4*)(pw + (int64_t)z * 65536);
#pragma unroll
      for (int z = 0; z < 4; ++z)
        if (z < g.nsplit) a += pz[z];
    } else {
      for (int z = 0; z < g.nsplit; ++z) a += *(const f32x4*)(pw + (int64_t)z * 65536);
    }
    if constexpr ((EPI == VITMI_EPI_STORE || EPI == VITMI_EPI_DGELU) && std::is_same<TC, bf16>::value &&
                  std::is_same<T, bf16>::value) {
      // the store-only and DGELU bf16 outputs leave as 8-B vectors (4 columns; N % 8 == 0 is a
      // gemm256 precondition, and 4 aligned columns are contiguous in the tile-native gelu' too),
      // element for element the arithmetic of epi_store
      f32x4 v = a;
      if constexpr (EPI == VITMI_EPI_STORE) {
        if (g.bias) v += *(const f32x4*)(g.bias + col);
      } else {
        const bf16x4 gp = *(const bf16x4*)((const bf16*)g.aux + aux_at(g, row, col));
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] *= (float)gp[j];
      }
      bf16x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (bf16)v[j];
      *(bf16x4*)((bf16*)g.C + row * g.ldc + col) = o;
      continue;
    }
    if constexpr (EPI == VITMI_EPI_RESIDUAL) {
      // fp32 residual in and out as 16-B vectors ((residual + acc) + bias, as epi_store)
      const f32x4 r = *(const f32x4*)(g.residual + row * g.ldr + col);
      const f32x4 bv = g.bias ? *(const f32x4*)(g.bias + col) : f32x4{0.f, 0.f, 0.f, 0.f};
      *(f32x4*)((float*)g.C + row * g.ldc + col) = (r + a) + bv;
      continue;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (col + j >= g.N) break;
      constexpr int EB = EpiOf<EPI>::base;
      const float bv = (g.bias && (EB == VITMI_EPI_STORE || EB == VITMI_EPI_BIAS_GELU || EB == VITMI_EPI_RESIDUAL))
                           ? g.bias[col + j] : 0.f;
      epi_store<T, TC, EPI>(g, row, col + j, a[j], bv);
    }
  }
}

// Column-sum partial rows (GemmArgs::colsum) of the split tail tiles, which skip the fused
// epilogue: block = (tail tile, 128-row half); thread = 4 columns x one of 4 row groups.
template <typename TC>
__global__ __launch_bounds__(256) void tail_colsum_kernel(GemmArgs g) {
  __shared__ f32x4 red[4][64];
  const int t = blockIdx.x >> 1, half = blockIdx.x & 1;
  int tm, tn;
  tile_rc(g, g.t_full + t, tm, tn);
  const int cg = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int64_t col = (int64_t)tn * 256 + cg * 4;
  const int64_t r0 = (int64_t)tm * 256 + half * 128;
  f32x4 a = {0.f, 0.f, 0.f, 0.f};
  if (col < g.N) {
    for (int i = rg; i < 128; i += 4) {
      const int64_t row = r0 + i;
      if (row >= g.M) break;
      const TC* p = (const TC*)g.C + row * g.ldc + col;
#pragma unroll
      for (int e = 0; e < 4; ++e) a[e] += (float)p[e];
    }
  }
  red[rg][cg] = a;
  __syncthreads();
  if (rg == 0 && col < g.N) {
    const f32x4 sum = red[0][cg] + red[1][cg] + red[2][cg] + red[3][cg];
    *(f32x4*)(g.colsum + ((int64_t)tm * 2 + half) * g.N + col) = sum;
  }
}

// ---------------------------------------------------------------- host launch
// GEMM kernel policy: 0 = auto, 1 = always the 128x128 kernel, 2 = always gemm256 (bf16),
// 3 = gemm256 on an 8-block persistent grid (every block walks many tiles; tests only)
static int g_policy = 0;
static int g_cus = 256;   // compute units of the current device (set on first use)

// CUs the persistent grid leaves free (vitmi_gemm_set_reserved_cus).  Atomic: the DP reducer may
// change it from a thread other than the one launching GEMMs.
static std::atomic<int> g_reserved{0};
#ifdef VITMI_GEMM_STAMPS
static unsigned long long* g_stamps = nullptr;
#endif

static void init_cus() {
  static bool done = false;
  if (done) return;
  int dev = 0;
  hipDeviceProp_t p;
  if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0)
    g_cus = p.multiProcessorCount;
  done = true;
}

static int64_t splits_for(int64_t tiles, int64_t ktiles, int64_t target, int64_t cap = 64) {
  int64_t want = target / tiles;
  const int64_t maxs = ktiles / 4;
  if (want > maxs) want = maxs;
  if (want > cap) want = cap;
  return want < 1 ? 1 : want;
}

// gemm256 for this shape?  `split`: the caller may split K (wgrad), which fills the chip
// with units even when there are few output tiles.
static bool use256(int dtype, int64_t M, int64_t N, int64_t K = 0, bool split = false) {
  if (dtype != VITMI_BF16 || (N % 8) != 0) return false;
  if (g_policy == 1) return false;
  if (g_policy >= 2) return true;
  const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256);
  if (tiles >= 16) return true;
  init_cus();
  return split && tiles * splits_for(tiles, (K + 63) / 64, 256) >= 128;
}

// persistent grid of the gemm256 launch for nwg tiles and `splits` K-slabs
static int grid256(int nwg, int splits) {
  int gx = (g_cus - g_reserved.load(std::memory_order_relaxed)) / splits;
  if (gx < 8 || g_policy == 3) gx = 8;   // policy 3: force many tiles per block (tests)
  return gx > nwg ? nwg : gx;
}

// Tail split: when the last round of a persistent launch would leave more than half of the
// blocks idle (ViT N=768 GEMMs: 591 tiles on 256 CUs), its tiles are split into S K-ranges
// (S <= 4, >= 2 K-steps each) so that round takes ~1/S of the time.
#ifndef VITMI_TAIL_SMAX
#define VITMI_TAIL_SMAX 4
#endif
#ifndef VITMI_TAIL_MINK
#define VITMI_TAIL_MINK 16
#endif
static bool tail_plan(int nwg, int gx, int nk, int& S, int& ks, int& ntail) {
  ntail = nwg % gx;
  if (nwg < gx || ntail == 0 || 2 * ntail > gx || nk < 4) return false;
  S = gx / ntail;
  if (S > VITMI_TAIL_SMAX) S = VITMI_TAIL_SMAX;
  if (S < 2) return false;
  ks = (nk + S - 1) / S;
  if (ks < 2) ks = 2;
  S = (nk + ks - 1) / ks;
  while (S > 1 && nk - (S - 1) * ks < 2) { ++ks; S = (nk + ks - 1) / ks; }
  return S > 1;
}

static size_t tail_ws_bytes(int64_t M, int64_t N, int64_t K) {
  init_cus();
  const int nwg = (int)(((M + 255) / 256) * ((N + 255) / 256));
  int S, ks, ntail;
  if (nwg <= 0 || !tail_plan(nwg, grid256(nwg, 1), (int)((K + 63) / 64), S, ks, ntail)) return 0;
  // (sized for any epilogue; launch_t may still decide not to split, see tail_ok)
  return (size_t)ntail * S * 256 * 256 * sizeof(float);
}

// Algorithmic work of one GEMM launch: 2MNK flops; bytes = A and B once, C written once
// (read too for ACCUM: the += of a weight gradient), plus the epilogue's aux / residual.
// Split-K partial slabs and tail partials are implementation traffic, not counted here.
template <typename T, int EPI, typename TC>
static void gemm_stat(const void* kernel, const GemmArgs& g) {
  constexpr int EB = EpiOf<EPI>::base;
  const double M = (double)g.M, N = (double)g.N, K = (double)g.K, es = sizeof(T);
  double bytes = (M * K + N * K) * es;
  if (EPI == EPI_PARTIAL || EB == VITMI_EPI_ACCUM) bytes += 2.0 * M * N * 4;   // dW += (read + write, fp32)
  else bytes += M * N * sizeof(TC) * (EPI == EPI_GELU_X3 ? 3 : 1);
  if (EB == VITMI_EPI_BIAS_GELU || EB == VITMI_EPI_DGELU) bytes += M * N * es;   // gelu' written / read
  if (EB == VITMI_EPI_RESIDUAL) bytes += M * N * 4;                               // residual read
  VITMI_STAT(kernel, 2.0 * M * N * K, bytes);
}

template <typename T, bool AK, bool BKM, int EPI, typename TC, bool F8 = false>
static int launch_t(GemmArgs g, int splits, bool big, hipStream_t s) {
  if constexpr (sizeof(T) == 2) {
    if (big) {
      g.tiles_n = (int)((g.N + 255) / 256);
      int nwg = (int)((g.M + 255) / 256) * g.tiles_n;
      g.kz = 1;
      g.ntiles = nwg;
      if (splits > 1) {
        // fold the K-slabs into the persistent unit space (see GemmArgs::kz)
        g.kz = splits;
        g.kz_steps = (int)(g.k_per_split / 64);
        g.k_per_split = ((g.K + 63) / 64) * 64;
        nwg *= splits;
        splits = 1;
      }
      const int gx = grid256(nwg, splits);
      int units = nwg, S = 1, ks = 0, ntail = 0;
      g.t_full = nwg;
      g.nsplit = 1;
      g.ksplit = 0;
      // measured: pays off for long reductions (>= 16 K-steps) and for the DGELU epilogue
      // (whose partial units skip its aux loads); a wash or a loss for K = 768 otherwise
      // (EPI_GELU_F8: the fix-up kernel does not write the split-f8 rows, so its tiles stay whole)
      const bool tail_ok = (g.k_per_split / 64 >= VITMI_TAIL_MINK || EPI == VITMI_EPI_DGELU) && EPI != EPI_GELU_F8;
      if (splits == 1 && tail_ok && EPI != EPI_PARTIAL && EPI != VITMI_EPI_ACCUM && g.tail_ws &&
          tail_plan(nwg, gx, (int)(g.k_per_split / 64), S, ks, ntail) &&
          g.tail_ws_bytes >= (size_t)ntail * S * 256 * 256 * sizeof(float)) {
        g.t_full = nwg - ntail;
        g.nsplit = S;
        g.ksplit = ks;
        units = g.t_full + ntail * S;
      }
#ifdef VITMI_GEMM_STAMPS
      g.stamps = g_stamps;
#endif
      hipLaunchKernelGGL((gemm256_kernel<AK, BKM, EPI, TC, F8>), dim3(gx, 1, splits), dim3(512), 0, s, g, units);
      VITMI_LAUNCH_CHECK("gemm256_kernel");
      gemm_stat<T, EPI, TC>((const void*)gemm256_kernel<AK, BKM, EPI, TC, F8>, g);
      if constexpr (EPI != EPI_GELU_F8) if (units != nwg) {
        const int blocks = (ntail * 256 * 64 + 255) / 256;
        hipLaunchKernelGGL((gemm_tail_fixup_kernel<T, TC, EPI>), dim3(blocks), dim3(256), 0, s, g, ntail);
        VITMI_LAUNCH_CHECK("gemm_tail_fixup_kernel");
        // partials read, outputs (+ gelu') written
        VITMI_STAT((gemm_tail_fixup_kernel<T, TC, EPI>), 0, (double)ntail * 65536 * (4.0 * S + 2 * sizeof(TC)));
        if (g.colsum) {   // the split tail tiles' column sums, from their finished output
          hipLaunchKernelGGL((tail_colsum_kernel<TC>), dim3(ntail * 2), dim3(256), 0, s, g);
          VITMI_LAUNCH_CHECK("tail_colsum_kernel");
        }
      }
      return VITMI_OK;
    }
  }
  if constexpr (F8) return fail(VITMI_ERR_UNSUPPORTED, "gemm: VITMI_BF16F8 operands need the 256x256 kernel");
  constexpr int BM = 128, BN = 128, WM = 2, WN = 2;
  g.tiles_n = (int)((g.N + BN - 1) / BN);
  const int tiles_m = (int)((g.M + BM - 1) / BM);
  dim3 grid(tiles_m * g.tiles_n, 1, splits);
  hipLaunchKernelGGL((gemm_kernel<T, AK, BKM, EPI, TC, BM, BN, WM, WN>), grid, dim3(WM * WN * 64), 0, s, g);
  VITMI_LAUNCH_CHECK("gemm_kernel");
  gemm_stat<T, EPI, TC>((const void*)gemm_kernel<T, AK, BKM, EPI, TC, BM, BN, WM, WN>, g);
  return VITMI_OK;
}

template <typename T, int EPI, typename TC>
static int launch_layout(int ak, int bk, GemmArgs g, int splits, bool big, hipStream_t s) {
  if (ak && bk) return launch_t<T, true, true, EPI, TC>(g, splits, big, s);
  if (ak && !bk) return launch_t<T, true, false, EPI, TC>(g, splits, big, s);
  if (!ak && !bk) return launch_t<T, false, false, EPI, TC>(g, splits, big, s);
  // A m-major x B k-major: weight gradients with the input operand stored transposed
  if constexpr (EPI == EPI_PARTIAL || EPI == VITMI_EPI_ACCUM) return launch_t<T, false, true, EPI, TC>(g, splits, big, s);
  return fail(VITMI_ERR_UNSUPPORTED, "gemm: layout A m-major x B k-major not instantiated");
}

template <typename T>
static int dispatch(int ak, int bk, int c_dtype, int epi, GemmArgs g, int splits, bool big, hipStream_t s) {
  const bool cbf = (c_dtype == VITMI_BF16);
  switch (epi) {
    case VITMI_EPI_STORE:
      return cbf ? launch_layout<T, VITMI_EPI_STORE, bf16>(ak, bk, g, splits, big, s)
                 : launch_layout<T, VITMI_EPI_STORE, float>(ak, bk, g, splits, big, s);
    case VITMI_EPI_BIAS_GELU:
      // bf16 operands: the GELU epilogue writes bf16 (activation and gelu'); gemm_impl rejects
      // an fp32 C, so that variant is not instantiated
      if constexpr (std::is_same<T, bf16>::value) return launch_layout<T, VITMI_EPI_BIAS_GELU, bf16>(ak, bk, g, splits, big, s);
      else return cbf ? launch_layout<T, VITMI_EPI_BIAS_GELU, bf16>(ak, bk, g, splits, big, s)
                      : launch_layout<T, VITMI_EPI_BIAS_GELU, float>(ak, bk, g, splits, big, s);
    case VITMI_EPI_RESIDUAL:
      return launch_layout<T, VITMI_EPI_RESIDUAL, float>(ak, bk, g, splits, big, s);
    case VITMI_EPI_DGELU:
      return cbf ? launch_layout<T, VITMI_EPI_DGELU, bf16>(ak, bk, g, splits, big, s)
                 : launch_layout<T, VITMI_EPI_DGELU, float>(ak, bk, g, splits, big, s);
    case VITMI_EPI_ACCUM:
      return launch_layout<T, VITMI_EPI_ACCUM, float>(ak, bk, g, splits, big, s);
    case EPI_PARTIAL:
      return launch_layout<T, EPI_PARTIAL, float>(ak, bk, g, splits, big, s);
    case EPI_GELU_DROP:   // forward linear layers only: x and W both k-major
      if (!(ak && bk)) break;
      if constexpr (std::is_same<T, bf16>::value) return launch_t<T, true, true, EPI_GELU_DROP, bf16>(g, splits, big, s);
      else return cbf ? launch_t<T, true, true, EPI_GELU_DROP, bf16>(g, splits, big, s)
                      : launch_t<T, true, true, EPI_GELU_DROP, float>(g, splits, big, s);
    case EPI_RESIDUAL_DROP:
      if (!(ak && bk)) break;
      return launch_t<T, true, true, EPI_RESIDUAL_DROP, float>(g, splits, big, s);
    case EPI_GELU_X3:   // forward linear layers, bf16 operands and output only (gemm_impl checks)
      if (!(ak && bk)) break;
      if constexpr (std::is_same<T, bf16>::value) return launch_t<T, true, true, EPI_GELU_X3, bf16>(g, splits, big, s);
      break;
  }
  return fail(VITMI_ERR_INVALID, "gemm: unknown epilogue %d", epi);
}

// VITMI_BF16F8 operands (the forward linear layers of the bf16f8 knob): gemm256 only
static int dispatch_f8(int c_dtype, int epi, GemmArgs g, hipStream_t s) {
  switch (epi) {
    case VITMI_EPI_STORE:
      return c_dtype == VITMI_BF16 ? launch_t<bf16, true, true, VITMI_EPI_STORE, bf16, true>(g, 1, true, s)
                                   : launch_t<bf16, true, true, VITMI_EPI_STORE, float, true>(g, 1, true, s);
    case VITMI_EPI_RESIDUAL:
      return launch_t<bf16, true, true, VITMI_EPI_RESIDUAL, float, true>(g, 1, true, s);
    case EPI_GELU_F8:
      return launch_t<bf16, true, true, EPI_GELU_F8, bf16, true>(g, 1, true, s);
  }
  return fail(VITMI_ERR_UNSUPPORTED, "gemm: VITMI_BF16F8 operands take STORE, RESIDUAL or BIAS_GELU|SPLIT_F8 (got %d)", epi);
}

static int bk_of(int dtype) { return dtype == VITMI_BF16 ? 64 : 32; }

// split count for a reduction-heavy GEMM (wgrad): about one full round of blocks
// (1 block/CU for gemm256, ~2 for the 128 kernel), at least 4 k-tiles per split.  `reserved`:
// the CUs left free; the workspace queries size for 0 (the most splits), so a workspace sized
// while CUs were reserved is never short after the reservation ends, or the reverse.
static int choose_splits(int dtype, int64_t M, int64_t N, int64_t K, int reserved) {
  const bool big = use256(dtype, M, N, K, true);
  const int64_t t = big ? 256 : 128;
  const int64_t tiles = ((M + t - 1) / t) * ((N + t - 1) / t);
  const int64_t ktiles = (K + bk_of(dtype) - 1) / bk_of(dtype);
  // about one round of the CUs the persistent grid may use: with reserved CUs (DP overlap) a
  // fixed 256 left a few units for a second full round (fc1 wgrad 262 -> 440 us at 8 reserved)
  init_cus();
  const int avail = g_cus - reserved > 8 ? g_cus - reserved : 8;
  // small outputs (the CvT's 64x64 .. 256x256 weight gradients over 16-262 k tokens) may take up
  // to 512 slabs while all of them stay under 32 MiB: with the usual cap of 64 a one-tile output
  // ran 64 workgroups on 256 CUs
  int64_t cap = 64;
  const int64_t slab = M * N * (int64_t)sizeof(float);
  if (slab > 0 && (32LL << 20) / slab > cap) cap = (32LL << 20) / slab < 512 ? (32LL << 20) / slab : 512;
  return (int)splits_for(tiles, ktiles, big ? avail : 2 * avail, cap);
}

static int gemm_impl(int dtype, int ak, int bk, int64_t M, int64_t N, int64_t K, const void* A,
                     int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int c_dtype,
                     int epi, const float* bias, void* aux, int64_t ldaux, const float* residual,
                     int64_t ldr, void* ws, size_t ws_bytes, hipStream_t s, bool allow_split,
                     const GemmArgs* drop = nullptr, float* colsum = nullptr, bool* colsum_done = nullptr) {
  if (colsum_done) *colsum_done = false;
  const bool aux_tiled = (epi & VITMI_EPI_AUX_TILED) != 0;
  const bool x3 = (epi & VITMI_EPI_SPLIT_X3) != 0;
  const bool sf8 = (epi & VITMI_EPI_SPLIT_F8) != 0;
  epi &= ~(VITMI_EPI_AUX_TILED | VITMI_EPI_SPLIT_X3 | VITMI_EPI_SPLIT_F8);
  // VITMI_BF16F8: rows of 2K bf16 units ([hi | e4m3 parts]); the kernel sees bf16 operands over
  // K' = 2K with the e4m3 K-steps from K/64 on (GemmArgs::k8)
  // VITMI_BF16F8W (the weight-side correction alone): rows of 1.5K bf16 units [hi | one e4m3 byte per
  // k]; K' = 1.5K with the K/128 e4m3 K-steps (128 k each: hi8 of x against lo8 of w) from K/64 on
  const bool f8w = dtype == VITMI_BF16F8W;
  const bool f8 = dtype == VITMI_BF16F8 || f8w;
  int64_t k8 = 0;
  if (f8) {
    VITMI_CHECK_ARG(ak && bk && !allow_split, "gemm: VITMI_BF16F8 operands: forward linear layers (k-major A and B) only");
    VITMI_CHECK_ARG(K % (f8w ? 128 : 64) == 0 && N % 16 == 0, "gemm: VITMI_BF16F8%s needs K %% %d == 0 and N %% 16 == 0",
                    f8w ? "W" : "", f8w ? 128 : 64);
    const int64_t kr = f8w ? K + K / 2 : 2 * K;
    VITMI_CHECK_ARG(lda >= kr && ldb >= kr, "gemm: VITMI_BF16F8 rows are 2K (VITMI_BF16F8W: 1.5K) bf16 units");
    k8 = K / 64;
    K = kr;
    dtype = VITMI_BF16;
  }
  if (sf8) {
    VITMI_CHECK_ARG(f8 && epi == VITMI_EPI_BIAS_GELU && c_dtype == VITMI_BF16,
                    "gemm: SPLIT_F8 needs BIAS_GELU, VITMI_BF16F8 operands and a bf16 output");
    VITMI_CHECK_ARG(ldc >= 2 * N && N % 64 == 0, "gemm: SPLIT_F8 needs N %% 64 == 0 and ldc >= 2N (bf16 units)");
    epi = EPI_GELU_F8;
  }
  if (x3) {
    VITMI_CHECK_ARG(epi == VITMI_EPI_BIAS_GELU && dtype == VITMI_BF16 && c_dtype == VITMI_BF16 && ak && bk,
                    "gemm: SPLIT_X3 needs BIAS_GELU, bf16 operands and output, k-major A and B");
    VITMI_CHECK_ARG(ldc >= 3 * N, "gemm: SPLIT_X3 needs ldc >= 3N");
    epi = EPI_GELU_X3;
  }
  VITMI_CHECK_ARG(dtype == VITMI_BF16 || dtype == VITMI_F32, "gemm: bad dtype %d", dtype);
  VITMI_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "gemm: negative size");
  if (M == 0 || N == 0) return VITMI_OK;
  VITMI_CHECK_ARG(A && B && C, "gemm: null operand");
  const int BK = bk_of(dtype);
  if (ak) VITMI_CHECK_ARG(K % BK == 0, "gemm: k-major A needs K %% %d == 0 (K=%lld)", BK, (long long)K);
  if (bk) VITMI_CHECK_ARG(K % BK == 0, "gemm: k-major B needs K %% %d == 0 (K=%lld)", BK, (long long)K);
  const int es = dtype == VITMI_BF16 ? 2 : 4;
  VITMI_CHECK_ARG((lda * es) % 16 == 0 && (ldb * es) % 16 == 0, "gemm: lda/ldb must be 16-byte multiples");
  VITMI_CHECK_ARG(((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0, "gemm: A/B must be 16-byte aligned");
  VITMI_CHECK_ARG(ak ? lda >= K : lda >= M, "gemm: lda too small");
  VITMI_CHECK_ARG(bk ? ldb >= K : ldb >= N, "gemm: ldb too small");
  VITMI_CHECK_ARG(ldc >= N, "gemm: ldc too small");
  const int eb = epi_base(epi);
  if (eb == VITMI_EPI_BIAS_GELU || eb == VITMI_EPI_DGELU)
    VITMI_CHECK_ARG(aux != nullptr && ldaux >= N, "gemm: epilogue needs aux");
  if (aux_tiled) {
    VITMI_CHECK_ARG(eb == VITMI_EPI_BIAS_GELU || eb == VITMI_EPI_DGELU, "gemm: AUX_TILED needs BIAS_GELU or DGELU");
    VITMI_CHECK_ARG(dtype == VITMI_BF16, "gemm: AUX_TILED needs bf16 operands (a bf16 gelu')");
    VITMI_CHECK_ARG(((uintptr_t)aux % 16) == 0, "gemm: AUX_TILED aux must be 16-byte aligned");
  }
  if (eb == VITMI_EPI_RESIDUAL) VITMI_CHECK_ARG(residual != nullptr && ldr >= N, "gemm: residual missing");
  if (eb == VITMI_EPI_RESIDUAL || eb == VITMI_EPI_ACCUM)
    VITMI_CHECK_ARG(c_dtype == VITMI_F32, "gemm: residual/accum epilogues write fp32");
  if (eb == VITMI_EPI_BIAS_GELU && dtype == VITMI_BF16)
    VITMI_CHECK_ARG(c_dtype == VITMI_BF16, "gemm: the bias+GELU epilogue on bf16 operands writes bf16");
  // 32-bit buffer offsets: one block's panel must stay under 2 GiB
  VITMI_CHECK_ARG((ak ? 128 * lda : K * lda) * es < 0x7fffffffLL, "gemm: A panel exceeds 2 GiB");

  const bool big = f8 || use256(dtype, M, N, K, allow_split && epi == VITMI_EPI_ACCUM);
  if (big) {
    init_cus();
    VITMI_CHECK_ARG(ldc % 8 == 0 && (ldr % 4) == 0 && (ldaux % 8) == 0 && ((uintptr_t)C % 16) == 0,
                    "gemm: 16-byte aligned C/aux/residual rows required");
    VITMI_CHECK_ARG(bias == nullptr || ((uintptr_t)bias % 16) == 0, "gemm: bias must be 16-byte aligned");
    VITMI_CHECK_ARG((ak ? 256 * lda : K * lda) * 2 < 0x7fffffffLL, "gemm: A panel exceeds 2 GiB");
  }
  GemmArgs g{};
  g.A = A; g.B = B; g.C = C; g.M = M; g.N = N; g.K = K;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.bias = bias; g.aux = aux; g.ldaux = ldaux;
  g.residual = residual; g.ldr = ldr;
  g.aux_tiled = aux_tiled;
  g.k8 = (int)k8;
  if (drop) {
    g.drop_seed = drop->drop_seed; g.drop_site = drop->drop_site;
    g.drop_thresh = drop->drop_thresh; g.drop_scale = drop->drop_scale;
  }
  int splits = 1;
  if (allow_split && epi == VITMI_EPI_ACCUM) splits = choose_splits(dtype, M, N, K, g_reserved.load(std::memory_order_relaxed));
  const int64_t ktiles = (K + BK - 1) / BK;
  g.k_per_split = ((ktiles + splits - 1) / splits) * BK;
  if (K == 0) g.k_per_split = BK;
  splits = (int)((K + g.k_per_split - 1) / g.k_per_split);
  if (splits < 1) splits = 1;
  if (splits > 1) {
    const size_t need = (size_t)splits * M * N * sizeof(float);
    if (ws == nullptr || ws_bytes < need) splits = 1, g.k_per_split = ktiles * BK;
  }
  bool big2 = big;
  if (big2) {
    // gemm256 keeps two K-steps in flight: every split must span >= 2 k-tiles
    const int64_t kps = g.k_per_split / BK;
    const int64_t last = ktiles - (int64_t)(splits - 1) * kps;
    if (ktiles < 2 || kps < 2 || last < 2) {
      if (splits > 1 && ktiles >= 4) {
        int64_t k2 = kps + 1;
        while (ktiles - ((ktiles + k2 - 1) / k2 - 1) * k2 < 2) ++k2;
        g.k_per_split = k2 * BK;
        splits = (int)((ktiles + k2 - 1) / k2);
      } else {
        big2 = false;
      }
    }
  }
  const bool big_ok = big2;
  if (splits == 1) {
    g.k_per_split = (K > 0 ? ktiles : 1) * BK;
    g.tail_ws = (float*)ws;   // tail split of the persistent gemm256 launch (if it fits)
    g.tail_ws_bytes = ws ? ws_bytes : 0;
    if (colsum && big_ok && dtype == VITMI_BF16 && epi == VITMI_EPI_DGELU) {
      g.colsum = colsum;      // fused column sums (gemm256 DGELU epilogue only)
      if (colsum_done) *colsum_done = true;
    }
    if (f8) {
      VITMI_CHECK_ARG(big_ok, "gemm: VITMI_BF16F8 needs >= 2 K-steps");
      return dispatch_f8(c_dtype, epi, g, s);
    }
    if (dtype == VITMI_BF16) return dispatch<bf16>(ak, bk, c_dtype, epi, g, 1, big_ok, s);
    return dispatch<float>(ak, bk, c_dtype, epi, g, 1, big_ok, s);
  }
  // split-K: partial slabs then one reduction pass into C (+=)
  GemmArgs gp = g;
  gp.C = ws; gp.ldc = N; gp.split_stride = M * N;
  int rc = dtype == VITMI_BF16 ? dispatch<bf16>(ak, bk, VITMI_F32, EPI_PARTIAL, gp, splits, big_ok, s)
                               : dispatch<float>(ak, bk, VITMI_F32, EPI_PARTIAL, gp, splits, big_ok, s);
  if (rc) return rc;
  VITMI_CHECK_ARG(ldc == N, "gemm: split-K accumulate needs a dense C");
  const int64_t n = M * N;
  if ((n + 3) / 4 <= SMALL_RED_MAX && splits >= 16) {
    hipLaunchKernelGGL(splitk_reduce_small_kernel, dim3((unsigned)(((n + 3) / 4 + 63) / 64)), dim3(1024), 0, s,
                       (const float*)ws, (float*)C, n, splits, M * N);
    VITMI_LAUNCH_CHECK("splitk_reduce_small_kernel");
    VITMI_STAT(splitk_reduce_small_kernel, 0, (double)n * 4 * (splits + 2));
    return VITMI_OK;
  }
  int blocks = (int)((n / 4 + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, s, (const float*)ws,
                     (float*)C, n, splits, M * N);
  VITMI_LAUNCH_CHECK("splitk_reduce_kernel");
  VITMI_STAT(splitk_reduce_kernel, 0, (double)n * 4 * (splits + 2));
  return VITMI_OK;
}

// ---------------------------------------------------------------- grouped weight gradients
// dW_p[N_p, K_p] += dy_p[M, N_p]^T x_p[M, K_p] for p < n in ONE gemm256 launch (the K-slabs of
// every problem folded into one persistent unit space) and one reduction launch.  One launch per
// problem pays its own ramp, its own chip-wide burst of slab stores at the end and its own
// reduction; and a small output (the out-projection's 768 x 768: 9 tiles) is cut into 28 slabs of
// 28 K-steps there, against 7 of 113 here.
struct WgProb {
  const void* dy;
  int64_t lddy;
  const void* x;
  int64_t ldx;
  float* dw;
  int64_t N, K;
};

// slabs per tile of a grouped launch: the smallest number of rounds r of the persistent grid whose
// S = r * avail / tiles units fill >= 95 % of the r rounds (ViT-B: 108 tiles -> S = 7, 756 units
// on 3 x 256 CUs; ViT-L: 192 -> 4, 768); each split keeps >= 8 K-steps
static int group_splits(int64_t tiles, int64_t ktiles, int avail) {
  int best = 1;
  double beff = 0.0;
  for (int r = 1; r <= 4; ++r) {
    int64_t S = (int64_t)r * avail / tiles;
    if (S < 1) S = 1;
    if (S > 1 && ktiles / S < 8) break;
    const double eff = (double)(tiles * S) / ((double)r * avail);
    if (eff >= 0.95) return (int)S;
    if (eff > beff) { beff = eff; best = (int)S; }
  }
  return best;
}

static bool group_ok(int dtype, int n, int64_t M, const WgProb* pr) {
  if (dtype != VITMI_BF16 || n < 2 || n > GRP_MAX || M < 4 * 64 || g_policy == 1) return false;
  for (int q = 0; q < n; ++q) {
    const WgProb& w = pr[q];
    if (w.N <= 0 || w.K <= 0 || (w.K % 8) != 0 || !use256(dtype, w.N, w.K, M, true)) return false;
    if (((uintptr_t)w.dy % 16) || ((uintptr_t)w.x % 16) || ((w.lddy * 2) % 16) || ((w.ldx * 2) % 16)) return false;
    if (w.lddy < w.N || w.ldx < w.K || M * w.lddy * 2 >= 0x7fffffffLL || M * w.ldx * 2 >= 0x7fffffffLL) return false;
  }
  return true;
}

static void group_plan(int n, int64_t M, const WgProb* pr, int64_t& tiles, int& S, size_t& need) {
  init_cus();
  tiles = 0;
  int64_t mn = 0;
  for (int q = 0; q < n; ++q) {
    tiles += ((pr[q].N + 255) / 256) * ((pr[q].K + 255) / 256);
    mn += pr[q].N * pr[q].K;
  }
  S = group_splits(tiles, (M + 63) / 64, g_cus);
  need = (size_t)S * mn * sizeof(float);
}

static size_t wgrad_group_ws(int dtype, int n, int64_t M, const WgProb* pr) {
  size_t need = 0;
  if (group_ok(dtype, n, M, pr)) {
    int64_t tiles;
    int S;
    group_plan(n, M, pr, tiles, S, need);
  }
  for (int q = 0; q < n; ++q) {   // the per-problem path (the fallback) may need more
    const int sp = choose_splits(dtype, pr[q].N, pr[q].K, M, 0);
    const size_t b = sp > 1 ? (size_t)sp * pr[q].N * pr[q].K * sizeof(float) : 0;
    need = b > need ? b : need;
  }
  return need;
}

static int wgrad_group_impl(int dtype, int n, int64_t M, const WgProb* pr, void* ws, size_t ws_bytes, hipStream_t s) {
  VITMI_CHECK_ARG(n >= 0 && n <= GRP_MAX, "linear_wgrad_group: 0..%d problems (got %d)", GRP_MAX, n);
  VITMI_CHECK_ARG(M >= 0, "linear_wgrad_group: negative M");
  for (int q = 0; q < n; ++q)
    VITMI_CHECK_ARG(pr[q].dy && pr[q].x && pr[q].dw && pr[q].N >= 0 && pr[q].K >= 0, "linear_wgrad_group: problem %d: "
                    "null operand or negative size", q);
  if (n == 0 || M == 0) return VITMI_OK;
  int64_t tiles = 0;
  int S = 1;
  size_t need = 0;
  const bool grouped = group_ok(dtype, n, M, pr) && (group_plan(n, M, pr, tiles, S, need), S > 1) && ws &&
                       ws_bytes >= need;
  if (!grouped) {
    for (int q = 0; q < n; ++q) {
      const WgProb& w = pr[q];
      if (int rc = gemm_impl(dtype, 0, 0, w.N, w.K, M, w.dy, w.lddy, w.x, w.ldx, w.dw, w.K, VITMI_F32,
                             VITMI_EPI_ACCUM, nullptr, nullptr, 0, nullptr, 0, ws, ws_bytes, s, true))
        return rc;
    }
    return VITMI_OK;
  }
  GemmArgs g{};
  g.K = M;
  g.lda = pr[0].lddy;   // (unused by the grouped kernel: its operands are the table's)
  g.ldb = pr[0].ldx;
  g.M = pr[0].N;
  g.N = pr[0].K;
  g.A = pr[0].dy;
  g.B = pr[0].x;
  g.ngrp = n;
  const int64_t ktiles = (M + 63) / 64;
  RedSegs rs{};
  rs.nseg = n;
  int64_t off = 0, t0 = 0;
  double flops = 0, bytes = 0;
  for (int q = 0; q < n; ++q) {
    GemmArgs::Prob& P = g.grp[q];
    P.A = pr[q].dy; P.lda = pr[q].lddy;
    P.B = pr[q].x;  P.ldb = pr[q].ldx;
    P.M = pr[q].N;  P.N = pr[q].K;
    P.C = (float*)ws + off;
    P.tiles_n = (int)((P.N + 255) / 256);
    P.tile0 = (int)t0;
    t0 += ((P.M + 255) / 256) * P.tiles_n;
    rs.ws[q] = P.C;
    rs.dst[q] = pr[q].dw;
    rs.n[q] = P.M * P.N;
    rs.g0[q + 1] = rs.g0[q] + (rs.n[q] + 3) / 4;
    off += (int64_t)S * P.M * P.N;
    flops += 2.0 * P.M * P.N * M;
    bytes += (double)M * (P.M + P.N) * 2 + 2.0 * P.M * P.N * 4;
  }
  g.ntiles = (int)tiles;
  g.kz = S;
  g.kz_steps = (int)((ktiles + S - 1) / S);
  g.k_per_split = ktiles * 64;
  g.t_full = (int)(tiles * S);
  g.nsplit = 1;
  g.tiles_n = 1;
  // every split must span >= 2 K-steps (the last one too)
  VITMI_CHECK_ARG(ktiles - (int64_t)(S - 1) * g.kz_steps >= 2, "linear_wgrad_group: split plan %d x %d over %lld "
                  "K-steps", S, g.kz_steps, (long long)ktiles);
  const int nwg = (int)(tiles * S);
  const int gx = grid256(nwg, 1);
  hipLaunchKernelGGL((gemm256_kernel<false, false, EPI_PARTIAL, float, false, true>), dim3(gx), dim3(512), 0, s, g, nwg);
  VITMI_LAUNCH_CHECK("gemm256_kernel (grouped wgrad)");
  VITMI_STAT((gemm256_kernel<false, false, EPI_PARTIAL, float, false, true>), flops, bytes);
  int blocks = (int)((rs.g0[n] + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(splitk_reduce_group_kernel, dim3(blocks), dim3(256), 0, s, rs, S);
  VITMI_LAUNCH_CHECK("splitk_reduce_group_kernel");
  VITMI_STAT(splitk_reduce_group_kernel, 0, (double)rs.g0[n] * 16 * (S + 2));
  return VITMI_OK;
}

}  // namespace vitmi

using namespace vitmi;

#ifdef VITMI_GEMM_STAMPS
extern "C" int vitmi_gemm_set_stamps(void* buf) {
  g_stamps = (unsigned long long*)buf;
  return 0;
}
#endif

extern "C" int vitmi_gemm_set_reserved_cus(int n) {
  init_cus();
  return g_reserved.exchange(n < 0 ? 0 : (n > g_cus - 8 ? g_cus - 8 : n));
}

extern "C" int vitmi_gemm_set_policy(int policy) {
  VITMI_CHECK_ARG(policy >= 0 && policy <= 3, "gemm_set_policy: policy must be 0..3");
  g_policy = policy;
  return VITMI_OK;
}

extern "C" int vitmi_gemm(int dtype, int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
                          const void* A, int64_t lda, const void* B, int64_t ldb, void* C,
                          int64_t ldc, int c_dtype, int epilogue, const float* bias, void* aux,
                          int64_t ldaux, const float* residual, int64_t ldr, void* workspace,
                          size_t ws_bytes, vitmi_stream_t stream) {
  return gemm_impl(dtype, a_kmajor, b_kmajor, M, N, K, A, lda, B, ldb, C, ldc, c_dtype, epilogue,
                   bias, aux, ldaux, residual, ldr, workspace, ws_bytes, (hipStream_t)stream, true);
}

extern "C" size_t vitmi_gemm_workspace_size(int dtype, int a_kmajor, int b_kmajor, int64_t M,
                                            int64_t N, int64_t K, int epilogue) {
  (void)a_kmajor; (void)b_kmajor;
  if (epilogue != VITMI_EPI_ACCUM) return use256(dtype, M, N) ? tail_ws_bytes(M, N, K) : 0;
  const int splits = choose_splits(dtype, M, N, K, 0);
  return splits > 1 ? (size_t)splits * M * N * sizeof(float) : 0;
}

extern "C" size_t vitmi_aux_tiled_bytes(int64_t rows, int64_t cols) {
  if (rows <= 0 || cols <= 0) return 0;
  return (size_t)((rows + 255) / 256) * (size_t)((cols + 255) / 256) * 131072;
}

extern "C" size_t vitmi_linear_fwd_workspace_size(int dtype, int64_t M, int64_t N, int64_t K) {
  if (dtype == VITMI_BF16F8) return tail_ws_bytes(M, N, 2 * K);   // (K' = 2K bf16 units)
  if (dtype == VITMI_BF16F8W) return tail_ws_bytes(M, N, K + K / 2);
  return use256(dtype, M, N) ? tail_ws_bytes(M, N, K) : 0;
}

extern "C" int vitmi_linear_fwd(int dtype, int64_t M, int64_t N, int64_t K, const void* x,
                                const void* w, const float* bias, void* y, int y_dtype,
                                int epilogue, void* aux, const float* residual, void* workspace,
                                size_t ws_bytes, vitmi_stream_t stream) {
  const int eb = epilogue & ~(VITMI_EPI_AUX_TILED | VITMI_EPI_SPLIT_X3 | VITMI_EPI_SPLIT_F8);
  VITMI_CHECK_ARG(eb == VITMI_EPI_STORE || eb == VITMI_EPI_BIAS_GELU || eb == VITMI_EPI_RESIDUAL,
                  "linear_fwd: bad epilogue %d", epilogue);
  const int64_t ldy = (epilogue & VITMI_EPI_SPLIT_X3) ? 3 * N : (epilogue & VITMI_EPI_SPLIT_F8) ? 2 * N : N;
  const int64_t ldk = dtype == VITMI_BF16F8 ? 2 * K : dtype == VITMI_BF16F8W ? K + K / 2 : K;   // (bf16 units)
  return gemm_impl(dtype, 1, 1, M, N, K, x, ldk, w, ldk, y, ldy, y_dtype, epilogue, bias, aux, N,
                   residual, N, workspace, ws_bytes, (hipStream_t)stream, false);
}

extern "C" int vitmi_linear_fwd_dropout(int dtype, int64_t M, int64_t N, int64_t K, const void* x,
                                        const void* w, const float* bias, void* y, int y_dtype,
                                        int epilogue, void* aux, const float* residual,
                                        void* workspace, size_t ws_bytes, uint32_t seed,
                                        uint32_t site, uint32_t thresh, float scale,
                                        vitmi_stream_t stream) {
  const int eb = epilogue & ~VITMI_EPI_AUX_TILED;
  VITMI_CHECK_ARG(eb == VITMI_EPI_BIAS_GELU || eb == VITMI_EPI_RESIDUAL,
                  "linear_fwd_dropout: epilogue must be BIAS_GELU or RESIDUAL (got %d)", epilogue);
  GemmArgs d{};
  d.drop_seed = seed; d.drop_site = site; d.drop_thresh = thresh; d.drop_scale = scale;
  const int epi = (eb == VITMI_EPI_BIAS_GELU ? EPI_GELU_DROP : EPI_RESIDUAL_DROP) | (epilogue & VITMI_EPI_AUX_TILED);
  return gemm_impl(dtype, 1, 1, M, N, K, x, K, w, K, y, N, y_dtype, epi, bias, aux, N, residual, N,
                   workspace, ws_bytes, (hipStream_t)stream, false, &d);
}

extern "C" size_t vitmi_linear_dgrad_workspace_size(int dtype, int64_t M, int64_t N, int64_t K) {
  // GEMM rows M, cols K, reduction N
  return use256(dtype, M, K) ? tail_ws_bytes(M, K, N) : 0;
}

extern "C" int vitmi_linear_dgrad(int dtype, int64_t M, int64_t N, int64_t K, const void* dy,
                                  const void* w, void* dx, int dx_dtype, int epilogue,
                                  const void* aux, void* workspace, size_t ws_bytes,
                                  vitmi_stream_t stream) {
  VITMI_CHECK_ARG((epilogue & ~VITMI_EPI_AUX_TILED) == VITMI_EPI_STORE ||
                      (epilogue & ~VITMI_EPI_AUX_TILED) == VITMI_EPI_DGELU,
                  "linear_dgrad: bad epilogue %d", epilogue);
  // dx[M,K] = dy[M,N] . W[N,K]: reduction over N; A = dy (k-major), B = W as [N][K] (n-major)
  return gemm_impl(dtype, 1, 0, M, K, N, dy, N, w, K, dx, K, dx_dtype, epilogue, nullptr,
                   const_cast<void*>(aux), K, nullptr, 0, workspace, ws_bytes, (hipStream_t)stream, false);
}

// Column-sum partial rows of the fused DGELU epilogue (two per 256-row tile).
static int64_t colsum_rows(int64_t M) { return ((M + 255) / 256) * 2; }

extern "C" size_t vitmi_linear_dgrad_bias_workspace_size(int dtype, int64_t M, int64_t N, int64_t K) {
  const size_t fused = (size_t)colsum_rows(M) * K * sizeof(float);
  const size_t unfused = vitmi_bias_grad_workspace_size(M, K);   // the GEMM runs without a tail split
  return fused > unfused ? fused : unfused;
}

extern "C" int vitmi_linear_dgrad_bias(int dtype, int64_t M, int64_t N, int64_t K, const void* dy,
                                       const void* w, void* dx, int dx_dtype, int epilogue, const void* aux,
                                       float* db, void* workspace, size_t ws_bytes, vitmi_stream_t stream) {
  VITMI_CHECK_ARG((epilogue & ~VITMI_EPI_AUX_TILED) == VITMI_EPI_STORE ||
                      (epilogue & ~VITMI_EPI_AUX_TILED) == VITMI_EPI_DGELU,
                  "linear_dgrad_bias: bad epilogue %d", epilogue);
  VITMI_CHECK_ARG(db != nullptr, "linear_dgrad_bias: db is null");
  VITMI_CHECK_ARG(workspace && ws_bytes >= vitmi_linear_dgrad_bias_workspace_size(dtype, M, N, K),
                  "linear_dgrad_bias: workspace too small");
  if (M == 0 || K == 0) return VITMI_OK;
  hipStream_t s = (hipStream_t)stream;
  bool fused = false;
  // the partial rows live in the workspace; the tail split is off on this path, so the
  // GEMM itself needs no other workspace
  int rc = gemm_impl(dtype, 1, 0, M, K, N, dy, N, w, K, dx, K, dx_dtype, epilogue, nullptr, const_cast<void*>(aux),
                     K, nullptr, 0, nullptr, 0, s, false, nullptr, (float*)workspace, &fused);
  if (rc) return rc;
  if (fused) return launch_colsum_finish(K, (int)colsum_rows(M), (const float*)workspace, db, s);
  // other paths (128x128 kernel, fp32): separate column-sum pass over dx
  return vitmi_bias_grad(dx_dtype, M, K, dx, K, db, workspace, ws_bytes, stream);
}

extern "C" size_t vitmi_linear_wgrad_workspace_size(int dtype, int64_t M, int64_t N, int64_t K) {
  // dW[N,K]: GEMM rows N, cols K, reduction M
  const int splits = choose_splits(dtype, N, K, M, 0);
  return splits > 1 ? (size_t)splits * N * K * sizeof(float) : 0;
}

extern "C" int vitmi_linear_wgrad(int dtype, int64_t M, int64_t N, int64_t K, const void* dy,
                                  const void* x, float* dw, void* workspace, size_t ws_bytes,
                                  vitmi_stream_t stream) {
  // dW[N,K] += sum_m dy[m][n] x[m][k]: A(n,m) = dy (m-major rows of n), B(m,k) = x (k contiguous)
  return gemm_impl(dtype, 0, 0, N, K, M, dy, N, x, K, dw, K, VITMI_F32, VITMI_EPI_ACCUM, nullptr,
                   nullptr, 0, nullptr, 0, workspace, ws_bytes, (hipStream_t)stream, true);
}

static int wg_probs(int n, const int64_t* N, const int64_t* K, const void* const* dy, const int64_t* lddy,
                    const void* const* x, const int64_t* ldx, float* const* dw, WgProb* pr) {
  VITMI_CHECK_ARG(n >= 0 && n <= GRP_MAX, "linear_wgrad_group: 0..%d problems (got %d)", GRP_MAX, n);
  VITMI_CHECK_ARG(n == 0 || (N && K), "linear_wgrad_group: null size arrays");
  for (int q = 0; q < n; ++q) {
    pr[q].N = N[q];
    pr[q].K = K[q];
    pr[q].dy = dy ? dy[q] : nullptr;
    pr[q].x = x ? x[q] : nullptr;
    pr[q].dw = dw ? dw[q] : nullptr;
    pr[q].lddy = lddy && lddy[q] > 0 ? lddy[q] : N[q];
    pr[q].ldx = ldx && ldx[q] > 0 ? ldx[q] : K[q];
  }
  return VITMI_OK;
}

extern "C" size_t vitmi_linear_wgrad_group_workspace_size(int dtype, int n, int64_t M, const int64_t* N,
                                                          const int64_t* K) {
  WgProb pr[GRP_MAX];
  if (n < 0 || n > GRP_MAX || wg_probs(n, N, K, nullptr, nullptr, nullptr, nullptr, nullptr, pr)) return 0;
  return wgrad_group_ws(dtype, n, M, pr);
}

extern "C" int vitmi_linear_wgrad_group(int dtype, int n, int64_t M, const int64_t* N, const int64_t* K,
                                        const void* const* dy, const int64_t* lddy, const void* const* x,
                                        const int64_t* ldx, float* const* dw, void* workspace, size_t ws_bytes,
                                        vitmi_stream_t stream) {
  WgProb pr[GRP_MAX];
  if (int rc = wg_probs(n, N, K, dy, lddy, x, ldx, dw, pr)) return rc;
  VITMI_CHECK_ARG(n == 0 || (dy && x && dw), "linear_wgrad_group: null operand arrays");
  return wgrad_group_impl(dtype, n, M, pr, workspace, ws_bytes, (hipStream_t)stream);
}
