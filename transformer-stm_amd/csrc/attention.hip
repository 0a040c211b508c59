// attention.hip — multi-head scaled-dot-product attention, forward and backward, gfx950.
//
// Replaces layers.MultiHeadAttention (models/CvT(Par).py:137,185) / the
// einsum-softmax-einsum of old_codes/MS_CvT.py:202-207.
//
// Layout: qkv [B*N][3*D] token-major (q | k | v, head h at columns h*64), o [B*N][D],
// lse fp32 [B*H][N].  dh = 64.
//
// bf16 path (v_mfma_f32_32x32x16_bf16), flash-style with the whole softmax in registers:
//   * "swapped" S^T = K Q^T: the query sits on the MFMA lane, so a softmax row is
//     lane-local (16 keys per lane + one xor-32 exchange), no LDS round trip;
//   * the S^T accumulator feeds the P.V product directly as the B operand
//     (O^T = V^T P^T sums over the accumulator's ROW index: no lane movement);
//   * V^T / Q^T / K^T / dO^T operands come from row-major LDS tiles through
//     ds_read_b64_tr_b16 (hardware transpose);
//   * one XOR swizzle serves both the row reads (ds_read_b128) and the transposed
//     reads of every 64x64 bf16 tile: chunk' = chunk ^ (((row>>1)&1)<<2 | ((row>>2)&3)).
//   Tiles are staged by LDS-DMA (buffer_load ... lds) with the range check zero-filling
//   keys/queries >= N.  Backward = delta pre-pass + dK/dV kernel (keys on lanes, query
//   tiles streamed) + dQ kernel (queries on lanes, key tiles streamed); no atomics.
// fp32 path: thread-per-row VALU kernels (exact fp32; the parity configuration).
#include "common.h"
#include <stdlib.h>
#include <type_traits>

namespace vitmi {

static constexpr int DH = 64;
// backward kernels: dP - delta formed by the MFMA chain (accumulator initialised to
// -delta) instead of a subtraction per element (0: the subtraction; A/B builds)
#ifndef VITMI_ATT_DPINIT
#define VITMI_ATT_DPINIT 1
#endif
static constexpr float LOG2E = 1.4426950408889634f;
static constexpr float LN2 = 0.6931471805599453f;

// raw v_exp_f32: exp2f() wraps it in denormal range handling (compare, select, ldexp: 5
// extra VALU per element); softmax arguments are <= 0 and results below 2^-126 are
// negligible next to the row sum, so the flush is harmless.  exp2(-inf) = 0.
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ int att_swz(int row) { return (((row >> 1) & 1) << 2) | ((row >> 2) & 3); }

// byte offset of 16-B chunk `ch` of row `row` in a [64][64] bf16 tile (128-B rows)
__device__ __forceinline__ int toff(int row, int ch) { return row * 128 + ((ch ^ att_swz(row)) << 4); }

// Stage 64 rows x 128 B (64 bf16 of one head) of a token-major matrix into a tile.
// rs is rebased at (batch start, column); row r of the tile = token tok0 + r.
template <int NWAVES>
__device__ __forceinline__ void stage_tile(char* lds, __amdgpu_buffer_rsrc_t rs, int64_t ld_bytes,
                                           int tok0, int wave, int lane) {
#pragma unroll
  for (int p = wave; p < 8; p += NWAVES) {
    const int r = p * 8 + (lane >> 3);
    const int c = (lane & 7) ^ att_swz(r);
    const uint32_t voff = (uint32_t)((int64_t)(tok0 + r) * ld_bytes + c * 16);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(void, lds + p * 1024), 16, voff, 0, 0, 0);
  }
}

// A/B fragment of a 32x32x16 step from a row-major tile: lane row = row0 + (lane&31),
// k = 16*s + 8*(lane>>5) + j   -> one ds_read_b128.
// row0 is a multiple of 16 at every call site, so the swizzle (row bits 1..3) depends on the
// lane only: the address is a wave-uniform base plus a lane-constant offset that the
// compiler hoists out of the loops (no per-read swizzle arithmetic).
__device__ __forceinline__ int frag_row_off(int s, int lane) {
  const int r = lane & 31;
  return r * 128 + (((2 * s + (lane >> 5)) ^ att_swz(r)) << 4);
}
__device__ __forceinline__ bf16x8 frag_row(const char* t, int row0, int s, int lane) {
  return *(const bf16x8*)(t + row0 * 128 + frag_row_off(s, lane));
}

// Transposed fragment: operand X^T[col][k] where the tile holds X[k][col] (rows = k).
// lane (col = c0 + (lane&31), h = lane>>5), element j <-> k-row
//   k0 + 8*(j>>2) + 4*h + (j&3)   (the accumulator-as-operand k order)
// k0 is a multiple of 16 and c0 is 0 or 32 at every call site: base k0*128 + lane constant.
__device__ __forceinline__ int frag_tr_off(int i, int c0, int lane) {
  const int g = lane >> 4, tl = lane & 15, q = tl >> 2, p = tl & 3;
  const int row = 8 * i + 4 * (g >> 1) + q;                 // < 16
  const int ch = (c0 >> 3) + 2 * (g & 1) + (p >> 1);
  return row * 128 + ((ch ^ att_swz(row)) << 4) + ((p & 1) << 3);
}
__device__ __forceinline__ bf16x8 frag_tr(const char* t, int k0, int c0, int lane) {
  bf16x8 f;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, t + k0 * 128 + frag_tr_off(i, c0, lane)));
    bf16x4 b = __builtin_bit_cast(bf16x4, v);
    f[4 * i + 0] = b[0];
    f[4 * i + 1] = b[1];
    f[4 * i + 2] = b[2];
    f[4 * i + 3] = b[3];
  }
  return f;
}

// XCD-aware block order of the streamed kernels (grid (ceil(N/128), B*H)): the hardware deals
// workgroups out round-robin over the 8 XCDs by linear id, which puts the ceil(N/128) blocks of
// one (batch, head) on different XCDs, each streaming the pair's whole K/V (or Q/dO) through its
// own L2.  Returned: the (block-in-pair, pair) this workgroup takes, such that every XCD walks a
// contiguous range of the logical order (x fastest), so a pair's blocks share one L2.
__device__ __forceinline__ void xcd_block(int& bx, int& bh) {
  const int gx = gridDim.x, total = gx * gridDim.y;
  const int i = blockIdx.y * gx + blockIdx.x;
  const int x = i & 7, slot = i >> 3, per = total >> 3, rem = total & 7;
  const int j = (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + slot;
  bh = j / gx;
  bx = j - bh * gx;
}

// key/query index held in accumulator register r of a 32x32 tile for lane-half h
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// accumulator regs 8s..8s+7 -> bf16 operand fragment
__device__ __forceinline__ bf16x8 pack8(const f32x16& x, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)x[8 * s + j];
  return r;
}

// 16 B of a token row from global via the range-checked buffer path (zero past the end)
__device__ __forceinline__ bf16x8 load_row16(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
  u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
  return __builtin_bit_cast(bf16x8, v);
}

// store 4 consecutive d values (fp32) of row `row` as bf16 (8 bytes)
__device__ __forceinline__ void store4(bf16* p, float a, float b, float c, float d) {
  bf16x4 v;
  v[0] = (bf16)a; v[1] = (bf16)b; v[2] = (bf16)c; v[3] = (bf16)d;
  *(bf16x4*)p = v;
}

// A wave's 32-row x 64-column output tile in the 32x32 accumulator layout (lane: row =
// lane & 31; acc[c2][r] = column 32*c2 + acc_row(r, lane >> 5)) leaves as whole 128-B lines:
// written as bf16 into a per-wave [32][144 B] LDS image, read back 16 B per lane and stored as
// 8 rows x 128 B per instruction.  Stored straight from the accumulator, every line would be
// written in eight 16-B pieces by eight instructions (store-issue bound).  Row r goes to byte
// offset (row0 + r) * ld_bytes of rs; rows past rs's range (>= N) are dropped by the buffer
// range check.  The compiler barriers keep the cross-lane exchange ordered (each lane reads
// what other lanes wrote).
static constexpr int ST_PITCH = 144;
static constexpr int ST_BYTES = 32 * ST_PITCH;

// the lane index as an opaque value: the lane-derived addresses of an epilogue are formed where
// it runs, not hoisted above the main loop to stay live across it (the dQ kernel sits at 128
// VGPRs, and the hoisted ones pushed a reload into its loop)
__device__ __forceinline__ int lane_here() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
__device__ __forceinline__ void store_tile32(char* scr, const f32x16 (&acc)[2], float mul,
                                             __amdgpu_buffer_rsrc_t rs, int64_t ld_bytes, int row0, int lane) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int c2 = 0; c2 < 2; ++c2)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      bf16x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (bf16)(acc[c2][4 * g4 + i] * mul);
      *(bf16x4*)(scr + r * ST_PITCH + (32 * c2 + 8 * g4 + 4 * h) * 2) = v;
    }
  asm volatile("" ::: "memory");
  const int rr = lane >> 3, cc = lane & 7;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const u32x4 v = *(const u32x4*)(scr + (8 * j + rr) * ST_PITCH + cc * 16);
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, (uint32_t)((int64_t)(row0 + 8 * j + rr) * ld_bytes + cc * 16), 0, 0);
  }
  asm volatile("" ::: "memory");
}

// The e4m3 block of the same tile (the VITMI_BF16F8 knob, common.h split_f8 / f8_off): the head's
// 64 columns are one 64-k block, [hi8 | lo8] = 128 B per row, hi8 = e4m3(bf16(v)), lo8 =
// e4m3((v - bf16(v)) 2^9) of v = acc * mul; the image goes out as whole lines like store_tile32's
__device__ __forceinline__ void store_tile32_f8(char* scr, const f32x16 (&acc)[2], float mul,
                                                __amdgpu_buffer_rsrc_t rs8, int64_t ld_bytes, int row0, int lane) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int c2 = 0; c2 < 2; ++c2)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      f32x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = acc[c2][4 * g4 + i] * mul;
      bf16x4 hi;
      uint32_t hi8, lo8;
      split_f8(v, hi, hi8, lo8);
      char* p = scr + r * ST_PITCH + 32 * c2 + 8 * g4 + 4 * h;
      *(uint32_t*)p = hi8;
      *(uint32_t*)(p + 64) = lo8;
    }
  asm volatile("" ::: "memory");
  const int rr = lane >> 3, cc = lane & 7;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const u32x4 v = *(const u32x4*)(scr + (8 * j + rr) * ST_PITCH + cc * 16);
    __builtin_amdgcn_raw_buffer_store_b128(v, rs8, (uint32_t)((int64_t)(row0 + 8 * j + rr) * ld_bytes + cc * 16), 0, 0);
  }
  asm volatile("" ::: "memory");
}

// Column sums of the rows < nvalid of the tile store_tile32 just wrote (its LDS image, as the
// stored bf16 values): each lane adds 4 rows x 8 columns, xor-shuffles fold the 8 row groups,
// and the block's waves (all of which must call) fold through red[wave][64] in wave order into
// colpart[0..63] -- a bias-gradient partial without a second pass over the stored matrix, in a
// fixed summation order.
__device__ __forceinline__ void tile32_colsum(const char* scr, int row0, int nvalid, float* colpart,
                                              float (*red)[64], int wave, int nw, int lane) {
  const int rr = lane >> 3, cc = lane & 7;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (row0 + 8 * j + rr < nvalid) {
      const bf16x8 b = *(const bf16x8*)(scr + (8 * j + rr) * ST_PITCH + cc * 16);
#pragma unroll
      for (int e = 0; e < 8; ++e) cs[e] += (float)b[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    cs[e] += __shfl_xor(cs[e], 8, 64);
    cs[e] += __shfl_xor(cs[e], 16, 64);
    cs[e] += __shfl_xor(cs[e], 32, 64);
  }
  __syncthreads();                       // red is free (an earlier call's fold is done)
  if (lane < 8) {
#pragma unroll
    for (int e = 0; e < 8; ++e) red[wave][lane * 8 + e] = cs[e];
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    float t = 0.f;
    for (int w = 0; w < nw; ++w) t += red[w][threadIdx.x];
    colpart[threadIdx.x] = t;
  }
}

// =============================================================== forward (bf16)
// grid (ceil(N/128), B*H), 256 threads: wave w owns queries q0 + 32w .. +31.
__global__ __launch_bounds__(256, 3) void attn_fwd_bf16(const bf16* __restrict__ qkv,
                                                     bf16* __restrict__ o, float* __restrict__ lse,
                                                     int N, int H, float scale) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * 8192];  // [buf][K|V] 8 KiB tiles
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int bx, bh;
  xcd_block(bx, bh);
  const int b = bh / H, hd = bh % H;
  const int D = H * DH;
  const int64_t ld = 3 * (int64_t)D;
  const int64_t ldb = ld * 2;
  const int h = lane >> 5;
  const bf16* base = qkv + (int64_t)b * N * ld;
  const uint32_t bytes = (uint32_t)((int64_t)N * ldb);
  __amdgpu_buffer_rsrc_t rq = make_rsrc(base + hd * DH, bytes - hd * DH * 2);
  __amdgpu_buffer_rsrc_t rk = make_rsrc(base + D + hd * DH, bytes - (D + hd * DH) * 2);
  __amdgpu_buffer_rsrc_t rv = make_rsrc(base + 2 * D + hd * DH, bytes - (2 * D + hd * DH) * 2);

  const int qw = bx * 128 + wave * 32;  // first query of this wave
  const int q = qw + (lane & 31);
  // Q^T operand fragments: lane col q, k = d = 16s + 8h + j
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = load_row16(rq, (uint32_t)((int64_t)q * ldb + (16 * s + 8 * h) * 2));

  const float c2 = scale * LOG2E;
  float m = -INFINITY, l = 0.f;
  f32x16 oacc[2] = {zero16(), zero16()};

  const int nt = (N + 63) / 64;
  stage_tile<4>(smem, rk, ldb, 0, wave, lane);
  stage_tile<4>(smem + 8192, rv, ldb, 0, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int buf = t & 1;
    if (t + 1 < nt) {
      char* nb = smem + (buf ^ 1) * 16384;
      stage_tile<4>(nb, rk, ldb, (t + 1) * 64, wave, lane);
      stage_tile<4>(nb + 8192, rv, ldb, (t + 1) * 64, wave, lane);
    }
    const char* kt = smem + buf * 16384;
    const char* vt = kt + 8192;
    // One key tile: U 32-key sub-tiles (U = 1 when the tile holds <= 32 valid keys: padded keys
    // beyond the last 32-key group are never multiplied), the key mask only in the last tile,
    // scale folded into the exp argument, O rescaled only when a lane's running max moved.
    auto tile = [&](auto uc, auto mc) {
      constexpr int U = decltype(uc)::value;
      constexpr bool MASK = decltype(mc)::value;
      f32x16 st[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        st[u] = zero16();
#pragma unroll
        for (int s = 0; s < 4; ++s) st[u] = mfma32(frag_row(kt, 32 * u, s, lane), qf[s], st[u]);
      }
      if constexpr (MASK) {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (t * 64 + 32 * u + acc_row(r, h) >= N) st[u][r] = -INFINITY;
      }
      float tmax = -INFINITY;
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, st[u][r]);
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float mn = fmaxf(m, tmax * c2);
      const float alpha = fexp2(m - mn);  // m=-inf on the first tile -> 0
      const bool first = m == -INFINITY;
      m = mn;
      float rs = 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fexp2(fmaf(st[u][r], c2, -mn));
          st[u][r] = p;
          rs += p;
        }
      l = fmaf(l, alpha, rs);
      if (!first && __builtin_amdgcn_ballot_w64(alpha != 1.f) != 0) {
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
          for (int r = 0; r < 16; ++r) oacc[dt][r] *= alpha;
      }
      // O^T[d][q] += V^T[d][key] P^T[key][q]
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 pb = pack8(st[u], s);
#pragma unroll
          for (int dt = 0; dt < 2; ++dt)
            oacc[dt] = mfma32(frag_tr(vt, 32 * u + 16 * s, 32 * dt, lane), pb, oacc[dt]);
        }
    };
    if (qw < N) {
      if (t * 64 + 64 <= N) tile(std::integral_constant<int, 2>{}, std::false_type{});
      else if (t * 64 + 32 < N) tile(std::integral_constant<int, 2>{}, std::true_type{});
      else tile(std::integral_constant<int, 1>{}, std::true_type{});
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (qw >= N) return;
  const float lt = l + __shfl_xor(l, 32, 64);
  if (q < N && h == 0) lse[(int64_t)bh * N + q] = (m + log2f(lt)) * LN2;
  // O as whole 128-B lines through a per-wave image in the (free: the loop ended on a barrier)
  // K/V buffers; rows >= N fall outside the descriptor's range
  const int64_t ldo = (int64_t)D * 2;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(o + (int64_t)b * N * D + hd * DH, (uint32_t)((int64_t)N * ldo - hd * DH * 2));
  store_tile32(smem + wave * ST_BYTES, oacc, 1.f / lt, ro, ldo, qw, lane_here());
}

// =============================================================== backward (bf16)
// delta[bh][q] = sum_d dO[q][d] * O[q][d]
template <typename T>
__global__ void attn_bwd_delta(const T* __restrict__ o, const T* __restrict__ dout,
                               float* __restrict__ delta, int BN, int N, int H) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (token, head)
  if (i >= (int64_t)BN * H) return;
  const int64_t tok = i / H;
  const int hd = (int)(i % H);
  const int D = H * DH;
  const T* po = o + tok * D + hd * DH;
  const T* pd = dout + tok * D + hd * DH;
  float s = 0.f;
#pragma unroll 8
  for (int d = 0; d < DH; ++d) s += to_f32(po[d]) * to_f32(pd[d]);
  const int b = (int)(tok / N), q = (int)(tok % N);
  delta[((int64_t)b * H + hd) * N + q] = s;
}

// dK/dV: grid (ceil(N/128), B*H), wave w owns keys k0 = 128*bx + 32w .. +31.
__global__ __launch_bounds__(256, 3) void attn_bwd_dkv_bf16(
    const bf16* __restrict__ qkv, const bf16* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, bf16* __restrict__ dqkv, int N, int H, float scale,
    float* __restrict__ colsum) {
  // [buf][Q tile | dO tile] 2 x 16 KiB, then [buf][lse*log2e | delta] 2 x 512 B (one array: the
  // compiler must see a single LDS object next to the DMA, cdna_hip_programming.md §5 trap (a))
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * 8192 + 2 * 512];
  float* rowst = (float*)(smem + 32768);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int bx, bh;
  xcd_block(bx, bh);
  const int b = bh / H, hd = bh % H;
  const int D = H * DH;
  const int64_t ld = 3 * (int64_t)D, ldb = ld * 2, ldo = (int64_t)D * 2;
  const int h = lane >> 5;
  const bf16* base = qkv + (int64_t)b * N * ld;
  const uint32_t bytes = (uint32_t)((int64_t)N * ldb);
  const uint32_t obytes = (uint32_t)((int64_t)N * ldo);
  __amdgpu_buffer_rsrc_t rq = make_rsrc(base + hd * DH, bytes - hd * DH * 2);
  __amdgpu_buffer_rsrc_t rk = make_rsrc(base + D + hd * DH, bytes - (D + hd * DH) * 2);
  __amdgpu_buffer_rsrc_t rv = make_rsrc(base + 2 * D + hd * DH, bytes - (2 * D + hd * DH) * 2);
  __amdgpu_buffer_rsrc_t rdo = make_rsrc(dout + (int64_t)b * N * D + hd * DH, obytes - hd * DH * 2);
  const float* lse_bh = lse + (int64_t)bh * N;
  const float* del_bh = delta + (int64_t)bh * N;
  // per-query row constants of tile t into rowst[buf]: q >= N get L2 = +inf -> p = 0
  auto stage_rows = [&](int t, int buf) {
    if (wave == 0) {
      const int qi = t * 64 + lane;
      rowst[buf * 128 + lane] = qi < N ? lse_bh[qi] * LOG2E : INFINITY;
      rowst[buf * 128 + 64 + lane] = qi < N ? del_bh[qi] : 0.f;
    }
  };

  const int kw = bx * 128 + wave * 32;
  const int key = kw + (lane & 31);
  // K^T / V^T operand fragments (B operands): lane col = key, k = d = 16s + 8h + j
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = load_row16(rk, (uint32_t)((int64_t)key * ldb + (16 * s + 8 * h) * 2));
    vf[s] = load_row16(rv, (uint32_t)((int64_t)key * ldb + (16 * s + 8 * h) * 2));
  }
  const float c2 = scale * LOG2E;
  f32x16 dvt[2] = {zero16(), zero16()}, dkt[2] = {zero16(), zero16()};

  const int nt = (N + 63) / 64;
  stage_tile<4>(smem, rq, ldb, 0, wave, lane);
  stage_tile<4>(smem + 8192, rdo, ldo, 0, wave, lane);
  stage_rows(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int buf = t & 1;
    if (t + 1 < nt) {
      char* nb = smem + (buf ^ 1) * 16384;
      stage_tile<4>(nb, rq, ldb, (t + 1) * 64, wave, lane);
      stage_tile<4>(nb + 8192, rdo, ldo, (t + 1) * 64, wave, lane);
    }
    const char* qt = smem + buf * 16384;
    const char* dt_ = qt + 8192;
    const float* rl = rowst + buf * 128;
    if (kw < N) {
#pragma unroll 1
      for (int u = 0; u < 2; ++u) {  // 32-query sub-tile
        if (t * 64 + 32 * u >= N) break;   // all 32 queries padding: P = 0, dS = 0 there
        f32x16 sa = zero16(), dp;
        f32x4 L2[4];
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {   // row constants first: dP - delta from the MFMA chain
          const int q4 = 32 * u + 8 * g4 + 4 * h;           // rows acc_row(4*g4 + i, h) = q4 + i
          L2[g4] = *(const f32x4*)(rl + q4);
          const f32x4 dl = *(const f32x4*)(rl + 64 + q4);
#pragma unroll
          for (int i = 0; i < 4; ++i) dp[4 * g4 + i] = VITMI_ATT_DPINIT ? -dl[i] : 0.f;
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          sa = mfma32(frag_row(qt, 32 * u, s, lane), kf[s], sa);   // S[q][key]
          dp = mfma32(frag_row(dt_, 32 * u, s, lane), vf[s], dp);  // dP[q][key] - delta[q]
        }
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          [[maybe_unused]] const f32x4 dl = VITMI_ATT_DPINIT ? f32x4{} : *(const f32x4*)(rl + 64 + 32 * u + 8 * g4 + 4 * h);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float p = fexp2(sa[4 * g4 + i] * c2 - L2[g4][i]);
            sa[4 * g4 + i] = p;
            dp[4 * g4 + i] = VITMI_ATT_DPINIT ? p * dp[4 * g4 + i] : p * (dp[4 * g4 + i] - dl[i]);
          }
        }
        // dV^T[d][key] += dO^T[d][q] P[q][key];  dK^T[d][key] += Q^T[d][q] dS[q][key]
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 pb = pack8(sa, s), sb = pack8(dp, s);
#pragma unroll
          for (int d2 = 0; d2 < 2; ++d2) {
            dvt[d2] = mfma32(frag_tr(dt_, 32 * u + 16 * s, 32 * d2, lane), pb, dvt[d2]);
            dkt[d2] = mfma32(frag_tr(qt, 32 * u + 16 * s, 32 * d2, lane), sb, dkt[d2]);
          }
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (t + 1 < nt) stage_rows(t + 1, buf ^ 1);
    __syncthreads();
  }
  // dK, dV as whole lines through a per-wave image in the (free) Q | dO buffers; rows >= N
  // (whole waves past N hold zeros) fall outside the descriptors.  With colsum, the k- and
  // v-bias gradient partials of this (batch, key block) row come from the same images.
  const bf16* db = dqkv + (int64_t)b * N * ld;
  const __amdgpu_buffer_rsrc_t rdk = make_rsrc(db + D + hd * DH, bytes - (D + hd * DH) * 2);
  const __amdgpu_buffer_rsrc_t rdv = make_rsrc(db + 2 * D + hd * DH, bytes - (2 * D + hd * DH) * 2);
  const int ln = lane_here();
  char* scr = smem + wave * ST_BYTES;
  float* part = colsum + ((int64_t)b * gridDim.x + bx) * 3 * D + hd * DH;
  __shared__ float red[4][64];
  store_tile32(scr, dkt, scale, rdk, ldb, kw, ln);
  if (colsum) tile32_colsum(scr, kw, N, part + D, red, wave, 4, ln);
  store_tile32(scr, dvt, 1.f, rdv, ldb, kw, ln);
  if (colsum) tile32_colsum(scr, kw, N, part + 2 * D, red, wave, 4, ln);
}

// dQ: grid (ceil(N/128), B*H), wave w owns queries q0 = 128*bx + 32w .. +31.
// Also produces delta[bh][q] = sum_d dO[q][d] O[q][d] (consumed here and by the dK/dV
// kernel, which therefore runs after this one).
__global__ __launch_bounds__(256, 4) void attn_bwd_dq_bf16(
    const bf16* __restrict__ qkv, const bf16* __restrict__ o, const bf16* __restrict__ dout,
    const float* __restrict__ lse, float* __restrict__ delta, bf16* __restrict__ dqkv, int N, int H,
    float scale, float* __restrict__ colsum) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * 8192];  // [buf][K|V]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int bx, bh;
  xcd_block(bx, bh);
  const int b = bh / H, hd = bh % H;
  const int D = H * DH;
  const int64_t ld = 3 * (int64_t)D, ldb = ld * 2, ldo = (int64_t)D * 2;
  const int h = lane >> 5;
  const bf16* base = qkv + (int64_t)b * N * ld;
  const uint32_t bytes = (uint32_t)((int64_t)N * ldb);
  const uint32_t obytes = (uint32_t)((int64_t)N * ldo);
  __amdgpu_buffer_rsrc_t rq = make_rsrc(base + hd * DH, bytes - hd * DH * 2);
  __amdgpu_buffer_rsrc_t rk = make_rsrc(base + D + hd * DH, bytes - (D + hd * DH) * 2);
  __amdgpu_buffer_rsrc_t rv = make_rsrc(base + 2 * D + hd * DH, bytes - (2 * D + hd * DH) * 2);
  __amdgpu_buffer_rsrc_t rdo = make_rsrc(dout + (int64_t)b * N * D + hd * DH, obytes - hd * DH * 2);

  const int qw = bx * 128 + wave * 32;
  const int q = qw + (lane & 31);
  bf16x8 qf[4], df[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = load_row16(rq, (uint32_t)((int64_t)q * ldb + (16 * s + 8 * h) * 2));
    df[s] = load_row16(rdo, (uint32_t)((int64_t)q * ldo + (16 * s + 8 * h) * 2));
  }
  const bool qok = q < N;
  const float L2 = qok ? lse[(int64_t)bh * N + q] * LOG2E : INFINITY;
  // delta: this lane holds d = 16s + 8h + j of dO[q]; the xor-32 partner the other half
  float dl;
  {
    __amdgpu_buffer_rsrc_t ro = make_rsrc(o + (int64_t)b * N * D + hd * DH, obytes - hd * DH * 2);
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 ov = load_row16(ro, (uint32_t)((int64_t)q * ldo + (16 * s + 8 * h) * 2));
#pragma unroll
      for (int j = 0; j < 8; ++j) part += (float)ov[j] * (float)df[s][j];
    }
    dl = part + __shfl_xor(part, 32, 64);
    if (qok && h == 0) delta[(int64_t)bh * N + q] = dl;
  }
  const float c2 = scale * LOG2E;
  f32x16 dqt[2] = {zero16(), zero16()};

  const int nt = (N + 63) / 64;
  stage_tile<4>(smem, rk, ldb, 0, wave, lane);
  stage_tile<4>(smem + 8192, rv, ldb, 0, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int buf = t & 1;
    if (t + 1 < nt) {
      char* nb = smem + (buf ^ 1) * 16384;
      stage_tile<4>(nb, rk, ldb, (t + 1) * 64, wave, lane);
      stage_tile<4>(nb + 8192, rv, ldb, (t + 1) * 64, wave, lane);
    }
    const char* kt = smem + buf * 16384;
    const char* vt = kt + 8192;
    if (qw < N) {
      const bool last = t * 64 + 64 > N;   // the only tile with keys >= N
#pragma unroll
      for (int u = 0; u < 2; ++u) {  // 32-key sub-tile
        if (t * 64 + 32 * u >= N) break;   // all 32 keys padding: dS = 0 there
        f32x16 st = zero16(), dp;
        float ndl = VITMI_ATT_DPINIT ? -dl : 0.f;   // dP^T - delta from the MFMA chain
        asm volatile("" : "+v"(ndl));                // (splat formed here, not hoisted)
#pragma unroll
        for (int r = 0; r < 16; ++r) dp[r] = ndl;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          st = mfma32(frag_row(kt, 32 * u, s, lane), qf[s], st);  // S^T[key][q]
          dp = mfma32(frag_row(vt, 32 * u, s, lane), df[s], dp);  // dP^T[key][q] (- delta)
        }
        if (last) {
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (t * 64 + 32 * u + acc_row(r, h) >= N) st[r] = -INFINITY;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fexp2(fmaf(st[r], c2, -L2));   // q >= N: L2 = +inf -> p = 0
          dp[r] = VITMI_ATT_DPINIT ? p * dp[r] : p * (dp[r] - dl);
        }
        // dQ^T[d][q] += K^T[d][key] dS^T[key][q]
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 sb = pack8(dp, s);
#pragma unroll
          for (int d2 = 0; d2 < 2; ++d2)
            dqt[d2] = mfma32(frag_tr(kt, 32 * u + 16 * s, 32 * d2, lane), sb, dqt[d2]);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // dQ as whole lines through a per-wave image in the (free) K | V buffers (rows >= N fall
  // outside the descriptor); with colsum also the q-bias gradient partial of this (batch,
  // query block) row
  const __amdgpu_buffer_rsrc_t rdq = make_rsrc(dqkv + (int64_t)b * N * ld + hd * DH, bytes - hd * DH * 2);
  const int ln = lane_here();
  store_tile32(smem + wave * ST_BYTES, dqt, scale, rdq, ldb, qw, ln);
  if (colsum) {
    __shared__ float red[4][64];
    tile32_colsum(smem + wave * ST_BYTES, qw, N, colsum + ((int64_t)b * gridDim.x + bx) * 3 * D + hd * DH, red, wave, 4,
                  ln);
  }
}

// ====================================================== whole-sequence kernels (bf16)
// For N <= NPMAX = 256 (ViT: N = 197): ONE workgroup per (batch, head) with NW = ceil(N/32) waves
// (wave w owns the 32 rows 32w..32w+31 of the lane-side operand).  The streamed operands of
// the whole sequence are staged into LDS once (one DMA wait, one barrier); afterwards every
// wave runs its loop with no synchronisation, so MFMA, softmax VALU and LDS reads of the
// 2 x 7 co-resident waves interleave freely.  Rows are padded to NP = 32*NW only (the
// streamed kernels above pad to 128 queries x 64 keys: 1.69x the work at N = 197, here 1.29x).

// One 1-KiB LDS-DMA piece (64 lanes x 16 B at lds) in inline asm.  The builtin form makes hipcc
// emit `s_waitcnt vmcnt(0)` before LDS reads it cannot prove disjoint from a pending DMA (here:
// the V reads of this pair against the next pair's pieces), which drains the prefetch every
// pair; hidden from the compiler the pieces are counted by the kernel's own waits only (it has
// no compiler-visible vector loads in its loop).  "s_nop 4": the descriptor may come from a VALU
// write (v_readfirstlane); "s_nop 0": M0 written by SALU before the LDS-DMA reads it.
__device__ __forceinline__ void dma_piece(__amdgpu_buffer_rsrc_t rs, uint32_t voff, char* lds) {
  const uint32_t m0 = (uint32_t)(uintptr_t)LDS_PTR(char, lds);
  asm volatile("s_nop 4\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               :: "v"(voff), "s"(rs), "s"(m0) : "memory");   // (hipcc reserves M0; no compiler code here uses it)
}

// Stage rows [0, NP) (128 B of one head each) of a token-major matrix into an LDS image.
__device__ __forceinline__ void stage_seq(char* lds, __amdgpu_buffer_rsrc_t rs, int64_t ld_bytes, int np,
                                          int nw, int wave, int lane) {
  for (int p = wave; p < np / 8; p += nw) {
    const int r = p * 8 + (lane >> 3);
    const int c = (lane & 7) ^ att_swz(r);
    const uint32_t voff = (uint32_t)((int64_t)r * ld_bytes + c * 16);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(void, lds + p * 1024), 16, voff, 0, 0, 0);
  }
}

// Vector loads the compiler does not count (their destinations must not be read before the
// caller's own s_waitcnt and a "+v" statement on them; cdna_hip_programming.md §5.7 item 1 form
// (ii)).  The range check returns 0 past the descriptor's size.
__device__ __forceinline__ u32x4 asm_load16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, int imm) {
  u32x4 v;
  if (imm == 0) asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, 0 offen" : "=&v"(v) : "v"(voff), "s"(rs) : "memory");
  else if (imm == 32) asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, 0 offen offset:32" : "=&v"(v) : "v"(voff), "s"(rs) : "memory");
  else if (imm == 64) asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, 0 offen offset:64" : "=&v"(v) : "v"(voff), "s"(rs) : "memory");
  else asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, 0 offen offset:96" : "=&v"(v) : "v"(voff), "s"(rs) : "memory");
  return v;
}
__device__ __forceinline__ float asm_load4(__amdgpu_buffer_rsrc_t rs, uint32_t voff) {
  float v;
  asm volatile("s_nop 4\n\tbuffer_load_dword %0, %1, %2, 0 offen" : "=&v"(v) : "v"(voff), "s"(rs) : "memory");
  return v;
}

#ifdef VITMI_ATTN_STAMPS
// DIAGNOSTIC build only: [kernel 0 fwd / 1 dQ][pair][8] = s_memrealtime at start, operands
// landed, loop done, end; then HW_ID and XCC_ID (tools/attn_stamps.py)
__device__ unsigned long long* d_attn_stamps;
#define ATTN_STAMP(kern, k)                                                                          \
  do {                                                                                               \
    if (d_attn_stamps && threadIdx.x == 0) {                                                         \
      unsigned long long* p_ = d_attn_stamps + ((int64_t)(kern) * 65536 + blockIdx.x) * 8;           \
      p_[k] = __builtin_amdgcn_s_memrealtime();                                                      \
      if ((k) == 0) {                                                                                \
        p_[4] = __builtin_amdgcn_s_getreg(4 | (31 << 11));                                           \
        p_[5] = __builtin_amdgcn_s_getreg(20 | (15 << 11));                                          \
      }                                                                                              \
    }                                                                                                \
  } while (0)
// the single-pass backward: [2][pair][8] = pair start (its loads landed), phase 1 start, phase 1
// done, phase 2 done, epilogue done; HW_ID, XCC_ID in [6], [7]
#define FUSED_STAMP(pair, k)                                                                         \
  do {                                                                                               \
    if (d_attn_stamps && threadIdx.x == 0) {                                                         \
      unsigned long long* p_ = d_attn_stamps + ((int64_t)2 * 65536 + (pair)) * 8;                     \
      p_[k] = __builtin_amdgcn_s_memrealtime();                                                      \
      if ((k) == 0) {                                                                                \
        p_[6] = __builtin_amdgcn_s_getreg(4 | (31 << 11));                                           \
        p_[7] = __builtin_amdgcn_s_getreg(20 | (15 << 11));                                          \
      }                                                                                              \
    }                                                                                                \
  } while (0)
#else
#define ATTN_STAMP(kern, k) do {} while (0)
#define FUSED_STAMP(pair, k) do {} while (0)
#endif

// stage_seq with the pieces issued by dma_piece (no compiler-visible LDS-DMA; see there)
__device__ __forceinline__ void stage_seq_dma(char* lds, __amdgpu_buffer_rsrc_t rs, int64_t ld_bytes, int np,
                                              int nw, int wave, int lane) {
  for (int p = wave; p < np / 8; p += nw) {
    const int r = p * 8 + (lane >> 3);
    const int c = (lane & 7) ^ att_swz(r);
    dma_piece(rs, (uint32_t)((int64_t)r * ld_bytes + c * 16), lds + p * 1024);
  }
}

// grid B*H, block 64*NW.  Online softmax over key tiles of 64 (a final tile of 32 when NP is
// an odd multiple of 32); keys >= N exist only in the last tile and are masked there.
// XM (the precision knob): 1 (vitmi_attention_fwd_x3) also o3 = [hi | hi | lo] rows of the fp32 O;
// 2 (vitmi_attention_fwd_f8) o3 = the VITMI_BF16F8 A-operand rows [hi | hi8 | lo8] of it.
template <int NPMAX, int XM = 0>
__global__ __launch_bounds__(NPMAX * 2, 4) void attn_fwd_seq_bf16(const bf16* __restrict__ qkv,
                                                               bf16* __restrict__ o, float* __restrict__ lse,
                                                               int N, int H, float scale,
                                                               bf16* __restrict__ o3 = nullptr) {
  __shared__ __attribute__((aligned(16))) char smem[2 * NPMAX * 128];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = blockDim.x >> 6, NP = nw * 32;
  // pairs in DESCENDING order: the producer of this kernel's operand (the qkv GEMM for the
  // forward, the out-proj dgrad writing dO for dQ) finished with the last rows, which are the
  // ones still in the MALL; the dK/dV kernel after dQ then walks ascending (dQ ended at pair 0)
  const int bh = gridDim.x - 1 - blockIdx.x, b = bh / H, hd = bh % H;
  const int D = H * DH;
  const int64_t ld = 3 * (int64_t)D, ldb = ld * 2;
  const int h = lane >> 5;
  const bf16* base = qkv + (int64_t)b * N * ld;
  const uint32_t bytes = (uint32_t)((int64_t)N * ldb);
  __amdgpu_buffer_rsrc_t rq = make_rsrc(base + hd * DH, bytes - hd * DH * 2);
  __amdgpu_buffer_rsrc_t rk = make_rsrc(base + D + hd * DH, bytes - (D + hd * DH) * 2);
  __amdgpu_buffer_rsrc_t rv = make_rsrc(base + 2 * D + hd * DH, bytes - (2 * D + hd * DH) * 2);
  ATTN_STAMP(0, 0);
  char* kt = smem;
  char* vt = smem + NP * 128;
  stage_seq(kt, rk, ldb, NP, nw, wave, lane);
  stage_seq(vt, rv, ldb, NP, nw, wave, lane);
  const int q = wave * 32 + (lane & 31);
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = load_row16(rq, (uint32_t)((int64_t)q * ldb + (16 * s + 8 * h) * 2));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  ATTN_STAMP(0, 1);

  const float c2 = scale * LOG2E;
  float m = -INFINITY, l = 0.f;
  f32x16 oacc[2] = {zero16(), zero16()};
  auto tile = [&](auto uc, auto mc, int k0) {
    constexpr int U = decltype(uc)::value;
    constexpr bool MASK = decltype(mc)::value;
    f32x16 st[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      st[u] = zero16();
#pragma unroll
      for (int s = 0; s < 4; ++s) st[u] = mfma32(frag_row(kt, k0 + 32 * u, s, lane), qf[s], st[u]);
    }
    if constexpr (MASK) {   // last tile: keys >= N out of the softmax
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (k0 + 32 * u + acc_row(r, h) >= N) st[u][r] = -INFINITY;
    }
    float tmax = -INFINITY;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, st[u][r]);
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mn = fmaxf(m, tmax * c2);
    const float alpha = fexp2(m - mn);   // 0 on the first tile (m = -inf)
    const bool first = m == -INFINITY;
    m = mn;
    float rs = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = fexp2(fmaf(st[u][r], c2, -mn));
        st[u][r] = p;
        rs += p;
      }
    l = fmaf(l, alpha, rs);
    // rescale O only when some lane's running max moved (rare after the first tiles)
    if (!first && __builtin_amdgcn_ballot_w64(alpha != 1.f) != 0) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[dt][r] *= alpha;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pb = pack8(st[u], s);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
          oacc[dt] = mfma32(frag_tr(vt, k0 + 32 * u + 16 * s, 32 * dt, lane), pb, oacc[dt]);
      }
  };
  int k0 = 0;
  // full tiles of valid keys without the mask; padding keys (< 32 of them) sit in the last tile
  for (; k0 + 64 <= N; k0 += 64) tile(std::integral_constant<int, 2>{}, std::false_type{}, k0);
  if (k0 + 64 <= NP) {
    tile(std::integral_constant<int, 2>{}, std::true_type{}, k0);
    k0 += 64;
  }
  if (k0 < NP) tile(std::integral_constant<int, 1>{}, std::true_type{}, k0);

  const float lt = l + __shfl_xor(l, 32, 64);
  if (q < N && h == 0) lse[(int64_t)bh * N + q] = (m + log2f(lt)) * LN2;
  // O through the (now free) K/V image: every wave must be done reading it
  __syncthreads();
  ATTN_STAMP(0, 2);
  const int64_t ldo = (int64_t)D * 2;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(o + (int64_t)b * N * D + hd * DH, (uint32_t)((int64_t)N * ldo - hd * DH * 2));
  const float inv = 1.f / lt;
  store_tile32(smem + wave * ST_BYTES, oacc, inv, ro, ldo, wave * 32, lane_here());
  ATTN_STAMP(0, 3);
  if constexpr (XM == 2) {
    // hi (bf16) at columns [0, D) of the 2D-wide row, the head's e4m3 block [hi8 | lo8] at byte
    // 2D + 128 hd
    const int64_t ld8 = 2 * ldo;
    const uint32_t by8 = (uint32_t)((int64_t)N * ld8);
    char* base8 = (char*)(o3 + (int64_t)b * N * 2 * D);
    store_tile32(smem + wave * ST_BYTES, oacc, inv, make_rsrc(base8 + hd * DH * 2, by8 - hd * DH * 2), ld8, wave * 32,
                 lane_here());
    store_tile32_f8(smem + wave * ST_BYTES, oacc, inv, make_rsrc(base8 + 2 * D + hd * 128, by8 - (2 * D + hd * 128)),
                    ld8, wave * 32, lane_here());
  }
  if constexpr (XM == 1) {
    // hi = bf16(O) twice, then lo = bf16(O - hi), O = oacc * inv exactly as store_tile32 forms it
    const int64_t ld3 = 3 * ldo;
    const uint32_t by3 = (uint32_t)((int64_t)N * ld3);
    bf16* base3 = o3 + (int64_t)b * N * 3 * D + hd * DH;
    store_tile32(smem + wave * ST_BYTES, oacc, inv, make_rsrc(base3 + D, by3 - (D + hd * DH) * 2), ld3, wave * 32,
                 lane_here());
    store_tile32(smem + wave * ST_BYTES, oacc, inv, make_rsrc(base3, by3 - hd * DH * 2), ld3, wave * 32, lane_here());
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = oacc[dt][r] * inv;
        oacc[dt][r] = v - (float)(bf16)v;
      }
    store_tile32(smem + wave * ST_BYTES, oacc, 1.f, make_rsrc(base3 + 2 * D, by3 - (2 * D + hd * DH) * 2), ld3,
                 wave * 32, lane_here());
  }
}

#ifndef VITMI_ATTN_Q64
#define VITMI_ATTN_Q64 1
#endif
// The bf16 forward (vitmi_attention_fwd, N <= 256) with 4 waves of 64 queries (two 32-query
// blocks per wave): every K and V fragment read from LDS feeds both blocks' MFMAs, and each wave
// carries two independent softmax chains.  Per query block the arithmetic is attn_fwd_seq_bf16's,
// in the same order (bitwise equal outputs); 213 VGPRs, two workgroups per CU.  C3: 79.4-80.6 µs
// against 82.7-83.6 for the 7 x 32-query form (profiles/r05_q64/).  grid B*H, block 256.
// XM (the precision knobs, as attn_fwd_seq_bf16's): 1 also writes o3 = [hi | hi | lo] rows of the
// fp32 O, 2 the VITMI_BF16F8 rows [hi | hi8 | lo8]; o and lse are the XM = 0 kernel's bit for bit.
template <int NPMAX, int XM = 0>
__global__ __launch_bounds__(256, 2) void attn_fwd_seq64_bf16(const bf16* __restrict__ qkv, bf16* __restrict__ o,
                                                          float* __restrict__ lse, int N, int H, float scale,
                                                          bf16* __restrict__ o3 = nullptr) {
  __shared__ __attribute__((aligned(16))) char smem[2 * NPMAX * 128];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int NP = (N + 31) & ~31;
  const int bh = gridDim.x - 1 - blockIdx.x, b = bh / H, hd = bh % H;
  const int D = H * DH;
  const int64_t ld = 3 * (int64_t)D, ldb = ld * 2;
  const int h = lane >> 5;
  const bf16* base = qkv + (int64_t)b * N * ld;
  const uint32_t bytes = (uint32_t)((int64_t)N * ldb);
  __amdgpu_buffer_rsrc_t rq = make_rsrc(base + hd * DH, bytes - hd * DH * 2);
  __amdgpu_buffer_rsrc_t rk = make_rsrc(base + D + hd * DH, bytes - (D + hd * DH) * 2);
  __amdgpu_buffer_rsrc_t rv = make_rsrc(base + 2 * D + hd * DH, bytes - (2 * D + hd * DH) * 2);
  char* kt = smem;
  char* vt = smem + NP * 128;
  stage_seq(kt, rk, ldb, NP, 4, wave, lane);
  stage_seq(vt, rv, ldb, NP, 4, wave, lane);
  const int q0 = wave * 64;
  bf16x8 qf[2][4];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int s = 0; s < 4; ++s)
      qf[qb][s] = load_row16(rq, (uint32_t)((int64_t)(q0 + 32 * qb + (lane & 31)) * ldb + (16 * s + 8 * h) * 2));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const float c2 = scale * LOG2E;
  const int64_t ldo = (int64_t)D * 2;
  auto body = [&](auto qbc) {
    constexpr int QB = decltype(qbc)::value;
    float m[QB], l[QB];
    f32x16 oacc[QB][2];
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
      m[qb] = -INFINITY;
      l[qb] = 0.f;
      oacc[qb][0] = zero16();
      oacc[qb][1] = zero16();
    }
    auto tile = [&](auto uc, auto mc, int k0) {
      constexpr int U = decltype(uc)::value;
      constexpr bool MASK = decltype(mc)::value;
      f32x16 st[QB][U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) st[qb][u] = zero16();
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const bf16x8 kf = frag_row(kt, k0 + 32 * u, s, lane);
#pragma unroll
          for (int qb = 0; qb < QB; ++qb) st[qb][u] = mfma32(kf, qf[qb][s], st[qb][u]);
        }
      }
#pragma unroll
      for (int qb = 0; qb < QB; ++qb) {
        if constexpr (MASK) {
#pragma unroll
          for (int u = 0; u < U; ++u)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              if (k0 + 32 * u + acc_row(r, h) >= N) st[qb][u][r] = -INFINITY;
        }
        float tmax = -INFINITY;
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, st[qb][u][r]);
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
        const float mn = fmaxf(m[qb], tmax * c2);
        const float alpha = fexp2(m[qb] - mn);
        const bool first = m[qb] == -INFINITY;
        m[qb] = mn;
        float rs = 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float p = fexp2(fmaf(st[qb][u][r], c2, -mn));
            st[qb][u][r] = p;
            rs += p;
          }
        l[qb] = fmaf(l[qb], alpha, rs);
        if (!first && __builtin_amdgcn_ballot_w64(alpha != 1.f) != 0) {
#pragma unroll
          for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int r = 0; r < 16; ++r) oacc[qb][dt][r] *= alpha;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 pb[QB];
#pragma unroll
          for (int qb = 0; qb < QB; ++qb) pb[qb] = pack8(st[qb][u], s);
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            const bf16x8 vf = frag_tr(vt, k0 + 32 * u + 16 * s, 32 * dt, lane);
#pragma unroll
            for (int qb = 0; qb < QB; ++qb) oacc[qb][dt] = mfma32(vf, pb[qb], oacc[qb][dt]);
          }
        }
    };
    int k0 = 0;
    for (; k0 + 64 <= N; k0 += 64) tile(std::integral_constant<int, 2>{}, std::false_type{}, k0);
    if (k0 + 64 <= NP) {
      tile(std::integral_constant<int, 2>{}, std::true_type{}, k0);
      k0 += 64;
    }
    if (k0 < NP) tile(std::integral_constant<int, 1>{}, std::true_type{}, k0);
    float inv[QB];
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
      const float lt = l[qb] + __shfl_xor(l[qb], 32, 64);
      const int q = q0 + 32 * qb + (lane & 31);
      if (q < N && h == 0) lse[(int64_t)bh * N + q] = (m[qb] + log2f(lt)) * LN2;
      inv[qb] = 1.f / lt;
    }
    __syncthreads();   // O through the (now free) K/V image
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(o + (int64_t)b * N * D + hd * DH, (uint32_t)((int64_t)N * ldo - hd * DH * 2));
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
      char* scr = smem + wave * ST_BYTES;
      const int row0 = q0 + 32 * qb;
      store_tile32(scr, oacc[qb], inv[qb], ro, ldo, row0, lane_here());
      if constexpr (XM == 2) {
        // hi (bf16) at columns [0, D) of the 2D-wide row, the head's e4m3 block [hi8 | lo8] at byte
        // 2D + 128 hd (attn_fwd_seq_bf16<.., 2>'s layout)
        const int64_t ld8 = 2 * ldo;
        const uint32_t by8 = (uint32_t)((int64_t)N * ld8);
        char* base8 = (char*)(o3 + (int64_t)b * N * 2 * D);
        store_tile32(scr, oacc[qb], inv[qb], make_rsrc(base8 + hd * DH * 2, by8 - hd * DH * 2), ld8, row0, lane_here());
        store_tile32_f8(scr, oacc[qb], inv[qb], make_rsrc(base8 + 2 * D + hd * 128, by8 - (2 * D + hd * 128)), ld8,
                        row0, lane_here());
      }
      if constexpr (XM == 1) {
        // hi = bf16(O) twice, then lo = bf16(O - hi), O = oacc * inv as store_tile32 forms it
        const int64_t ld3 = 3 * ldo;
        const uint32_t by3 = (uint32_t)((int64_t)N * ld3);
        bf16* base3 = o3 + (int64_t)b * N * 3 * D + hd * DH;
        store_tile32(scr, oacc[qb], inv[qb], make_rsrc(base3 + D, by3 - (D + hd * DH) * 2), ld3, row0, lane_here());
        store_tile32(scr, oacc[qb], inv[qb], make_rsrc(base3, by3 - hd * DH * 2), ld3, row0, lane_here());
        f32x16 lo[2];
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float v = oacc[qb][dt][r] * inv[qb];
            lo[dt][r] = v - (float)(bf16)v;
          }
        store_tile32(scr, lo, 1.f, make_rsrc(base3 + 2 * D, by3 - (2 * D + hd * DH) * 2), ld3, row0, lane_here());
      }
    }
  };
  if (q0 + 32 < N) body(std::integral_constant<int, 2>{});
  else if (q0 < N) body(std::integral_constant<int, 1>{});
  else __syncthreads();
}

// dQ (+ delta = rowsum(dO * O)): grid B*H, block 64*NW, wave w owns queries 32w..+31, K and V
// of the whole sequence in LDS.  Keys >= N need no mask: their K rows are zero in LDS, so
// their dS (whatever it is) meets a zero row of K in dQ = dS K.
// NWC > 0: the wave count (ceil(N / 32)) as a compile-time constant (the ViT shapes, N = 197:
// 7), so the loop over the 32-row blocks unrolls and every LDS fragment address is a lane base
// plus an immediate offset (the runtime loop spent 12 (dQ) / 25 (dK/dV) v_add per block on them)
template <int NPMAX, int NWC = 0>
__global__ __launch_bounds__(NPMAX * 2, 4) void attn_bwd_dq_seq_bf16(
    const bf16* __restrict__ qkv, const bf16* __restrict__ o, const bf16* __restrict__ dout,
    const float* __restrict__ lse, float* __restrict__ delta, bf16* __restrict__ dqkv, int N, int H,
    float scale, float* __restrict__ colsum) {
  // K | V images; after the loop also the [NP][65] fp32 image of the fused bias column sums
  constexpr int SMEM = 2 * NPMAX * 128 > NPMAX * 65 * 4 ? 2 * NPMAX * 128 : NPMAX * 65 * 4;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = NWC > 0 ? NWC : blockDim.x >> 6, NP = nw * 32;
  // pairs in DESCENDING order: the producer of this kernel's operand (the qkv GEMM for the
  // forward, the out-proj dgrad writing dO for dQ) finished with the last rows, which are the
  // ones still in the MALL; the dK/dV kernel after dQ then walks ascending (dQ ended at pair 0)
  const int bh = gridDim.x - 1 - blockIdx.x, b = bh / H, hd = bh % H;
  const int D = H * DH;
  const int64_t ld = 3 * (int64_t)D, ldb = ld * 2, ldo = (int64_t)D * 2;
  const int h = lane >> 5;
  const bf16* base = qkv + (int64_t)b * N * ld;
  const uint32_t bytes = (uint32_t)((int64_t)N * ldb);
  const uint32_t obytes = (uint32_t)((int64_t)N * ldo);
  __amdgpu_buffer_rsrc_t rq = make_rsrc(base + hd * DH, bytes - hd * DH * 2);
  __amdgpu_buffer_rsrc_t rk = make_rsrc(base + D + hd * DH, bytes - (D + hd * DH) * 2);
  __amdgpu_buffer_rsrc_t rv = make_rsrc(base + 2 * D + hd * DH, bytes - (2 * D + hd * DH) * 2);
  __amdgpu_buffer_rsrc_t rdo = make_rsrc(dout + (int64_t)b * N * D + hd * DH, obytes - hd * DH * 2);
  __amdgpu_buffer_rsrc_t ro = make_rsrc(o + (int64_t)b * N * D + hd * DH, obytes - hd * DH * 2);
  ATTN_STAMP(1, 0);
  char* kt = smem;
  char* vt = smem + NP * 128;
  stage_seq(kt, rk, ldb, NP, nw, wave, lane);
  stage_seq(vt, rv, ldb, NP, nw, wave, lane);

  const int q = wave * 32 + (lane & 31);
  const bool qok = q < N;
  bf16x8 qf[4], df[4];
  float dl;
  {
    bf16x8 of[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const uint32_t off = (uint32_t)((int64_t)q * ldo + (16 * s + 8 * h) * 2);
      df[s] = load_row16(rdo, off);
      of[s] = load_row16(ro, off);
    }
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) part += (float)of[s][j] * (float)df[s][j];
    dl = part + __shfl_xor(part, 32, 64);
  }
  if (qok && h == 0) delta[(int64_t)bh * N + q] = dl;
  asm volatile("" ::: "memory");   // keep the Q loads after the delta reduction (registers)
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = load_row16(rq, (uint32_t)((int64_t)q * ldb + (16 * s + 8 * h) * 2));
  const float L2 = qok ? lse[(int64_t)bh * N + q] * LOG2E : INFINITY;   // q >= N -> p = 0
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  ATTN_STAMP(1, 1);

  const float c2 = scale * LOG2E;
  f32x16 dqt[2] = {zero16(), zero16()};
  auto kblock = [&](const int k0) {
    f32x16 st = zero16(), dp;
    // dP^T - delta straight from the MFMA chain: the accumulator starts at -delta (one row
    // constant per lane), so dS = P (dP - delta) is one multiply per element
    // (the opaque copy keeps the 16-register splat inside the block: hoisted out of the
    // unrolled key loop it stays live across it and pushes the kernel past 128 VGPRs)
    float ndl = VITMI_ATT_DPINIT ? -dl : 0.f;
    asm volatile("" : "+v"(ndl));
#pragma unroll
    for (int r = 0; r < 16; ++r) dp[r] = ndl;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      st = mfma32(frag_row(kt, k0, s, lane), qf[s], st);   // S^T[key][q]
      dp = mfma32(frag_row(vt, k0, s, lane), df[s], dp);   // dP^T[key][q] (- delta)
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = fexp2(fmaf(st[r], c2, -L2));
      dp[r] = VITMI_ATT_DPINIT ? p * dp[r] : p * (dp[r] - dl);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 sb = pack8(dp, s);
#pragma unroll
      for (int d2 = 0; d2 < 2; ++d2) dqt[d2] = mfma32(frag_tr(kt, k0 + 16 * s, 32 * d2, lane), sb, dqt[d2]);
    }
  };
  if constexpr (NWC > 0) {
#pragma unroll
    for (int k0 = 0; k0 < NWC * 32; k0 += 32) kblock(k0);
  } else {
#pragma unroll 1
    for (int k0 = 0; k0 < NP; k0 += 32) kblock(k0);
  }
  // dQ through the (now free) K/V image: every wave must be done reading it.  With colsum,
  // also this head's q-bias gradient partial colsum[b][hd*64 ..] (column sums of the stored dQ)
  __syncthreads();
  ATTN_STAMP(1, 2);
  const __amdgpu_buffer_rsrc_t rdq = make_rsrc(dqkv + (int64_t)b * N * ld + hd * DH, bytes - hd * DH * 2);
  const int ln = lane_here();
  store_tile32(smem + wave * ST_BYTES, dqt, scale, rdq, ldb, wave * 32, ln);
  ATTN_STAMP(1, 3);
  if (colsum) {
    __shared__ float red[NPMAX / 32][64];
    tile32_colsum(smem + wave * ST_BYTES, wave * 32, N, colsum + (int64_t)b * 3 * D + hd * DH, red, wave, nw, ln);
  }
}

// dQ (+ delta) with 4 waves of 64 queries (two 32-query blocks per wave, as attn_fwd_seq64_bf16):
// each K / V fragment read feeds both blocks.  NKB = ceil(N / 32) key blocks (compile time).  Per
// query block the arithmetic is attn_bwd_dq_seq_bf16's in the same order, and the q-bias column sums
// fold the 32-row blocks in block order as its tile32_colsum does (bitwise equal outputs).
template <int NPMAX, int NKB>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_seq64_bf16(
    const bf16* __restrict__ qkv, const bf16* __restrict__ o, const bf16* __restrict__ dout,
    const float* __restrict__ lse, float* __restrict__ delta, bf16* __restrict__ dqkv, int N, int H,
    float scale, float* __restrict__ colsum) {
  constexpr int SMEM = 2 * NPMAX * 128;
  constexpr int NP = NKB * 32;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  __shared__ float red[NPMAX / 32][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int bh = gridDim.x - 1 - blockIdx.x, b = bh / H, hd = bh % H;
  const int D = H * DH;
  const int64_t ld = 3 * (int64_t)D, ldb = ld * 2, ldo = (int64_t)D * 2;
  const int h = lane >> 5;
  const bf16* base = qkv + (int64_t)b * N * ld;
  const uint32_t bytes = (uint32_t)((int64_t)N * ldb);
  const uint32_t obytes = (uint32_t)((int64_t)N * ldo);
  __amdgpu_buffer_rsrc_t rq = make_rsrc(base + hd * DH, bytes - hd * DH * 2);
  __amdgpu_buffer_rsrc_t rk = make_rsrc(base + D + hd * DH, bytes - (D + hd * DH) * 2);
  __amdgpu_buffer_rsrc_t rv = make_rsrc(base + 2 * D + hd * DH, bytes - (2 * D + hd * DH) * 2);
  __amdgpu_buffer_rsrc_t rdo = make_rsrc(dout + (int64_t)b * N * D + hd * DH, obytes - hd * DH * 2);
  __amdgpu_buffer_rsrc_t ro = make_rsrc(o + (int64_t)b * N * D + hd * DH, obytes - hd * DH * 2);
  char* kt = smem;
  char* vt = smem + NP * 128;
  stage_seq(kt, rk, ldb, NP, 4, wave, lane);
  stage_seq(vt, rv, ldb, NP, 4, wave, lane);
  const int q0 = wave * 64;
  bf16x8 qf[2][4], df[2][4];
  float dl[2], L2[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int q = q0 + 32 * qb + (lane & 31);
    bf16x8 of[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const uint32_t off = (uint32_t)((int64_t)q * ldo + (16 * s + 8 * h) * 2);
      df[qb][s] = load_row16(rdo, off);
      of[s] = load_row16(ro, off);
    }
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) part += (float)of[s][j] * (float)df[qb][s][j];
    dl[qb] = part + __shfl_xor(part, 32, 64);
    if (q < N && h == 0) delta[(int64_t)bh * N + q] = dl[qb];
  }
  asm volatile("" ::: "memory");   // keep the Q loads after the delta reductions (registers)
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int q = q0 + 32 * qb + (lane & 31);
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[qb][s] = load_row16(rq, (uint32_t)((int64_t)q * ldb + (16 * s + 8 * h) * 2));
    L2[qb] = q < N ? lse[(int64_t)bh * N + q] * LOG2E : INFINITY;   // q >= N -> p = 0
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const float c2 = scale * LOG2E;
  const __amdgpu_buffer_rsrc_t rdq = make_rsrc(dqkv + (int64_t)b * N * ld + hd * DH, bytes - hd * DH * 2);
  auto body = [&](auto qbc) {
    constexpr int QB = decltype(qbc)::value;
    f32x16 dqt[QB][2];
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) dqt[qb][0] = dqt[qb][1] = zero16();
    auto kblock = [&](const int k0) {
      f32x16 st[QB], dp[QB];
#pragma unroll
      for (int qb = 0; qb < QB; ++qb) {
        st[qb] = zero16();
        float ndl = VITMI_ATT_DPINIT ? -dl[qb] : 0.f;
        asm volatile("" : "+v"(ndl));
#pragma unroll
        for (int r = 0; r < 16; ++r) dp[qb][r] = ndl;
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 kf = frag_row(kt, k0, s, lane), vf = frag_row(vt, k0, s, lane);
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) {
          st[qb] = mfma32(kf, qf[qb][s], st[qb]);
          dp[qb] = mfma32(vf, df[qb][s], dp[qb]);
        }
      }
#pragma unroll
      for (int qb = 0; qb < QB; ++qb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fexp2(fmaf(st[qb][r], c2, -L2[qb]));
          dp[qb][r] = VITMI_ATT_DPINIT ? p * dp[qb][r] : p * (dp[qb][r] - dl[qb]);
        }
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int d2 = 0; d2 < 2; ++d2) {
          const bf16x8 kr = frag_tr(kt, k0 + 16 * s, 32 * d2, lane);
#pragma unroll
          for (int qb = 0; qb < QB; ++qb) dqt[qb][d2] = mfma32(kr, pack8(dp[qb], s), dqt[qb][d2]);
        }
    };
#pragma unroll
    for (int k0 = 0; k0 < NP; k0 += 32) kblock(k0);
    __syncthreads();   // dQ through the (now free) K/V image
    const int ln = lane_here();
    const int rr = ln >> 3, cc = ln & 7;
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
      const int row0 = q0 + 32 * qb;
      store_tile32(smem + wave * ST_BYTES, dqt[qb], scale, rdq, ldb, row0, ln);
      if (colsum) {   // this block's column sums (tile32_colsum's first half), folded below
        float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        const char* scr = smem + wave * ST_BYTES;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (row0 + 8 * j + rr < N) {
            const bf16x8 v = *(const bf16x8*)(scr + (8 * j + rr) * ST_PITCH + cc * 16);
#pragma unroll
            for (int e = 0; e < 8; ++e) cs[e] += (float)v[e];
          }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          cs[e] += __shfl_xor(cs[e], 8, 64);
          cs[e] += __shfl_xor(cs[e], 16, 64);
          cs[e] += __shfl_xor(cs[e], 32, 64);
        }
        if (ln < 8) {
#pragma unroll
          for (int e = 0; e < 8; ++e) red[2 * wave + qb][ln * 8 + e] = cs[e];
        }
        asm volatile("" ::: "memory");   // the next store_tile32 rewrites the image these reads used
      }
    }
  };
  if (q0 + 32 < N) body(std::integral_constant<int, 2>{});
  else if (q0 < N) body(std::integral_constant<int, 1>{});
  else __syncthreads();
  if (colsum) {
    __syncthreads();
    if (threadIdx.x < 64) {
      float t = 0.f;
      for (int blk = 0; blk < NKB; ++blk) t += red[blk][threadIdx.x];
      colsum[(int64_t)b * 3 * D + hd * DH + threadIdx.x] = t;
    }
  }
}

// dK/dV, persistent: grid = min(B*H, CUs) workgroups of 64*NW threads, each walking the (batch,
// head) pairs bh = blockIdx.x, + gridDim.x, ...; wave w owns keys 32w..+31 and holds their K and
// V rows in registers, the pair's Q and dO images sit in LDS.  At 165 VGPRs a CU holds one such
// workgroup anyway, so a second LDS buffer costs no occupancy: the next pair's Q | dO DMA is
// issued right after the pair-start barrier and lands under this pair's loop, and its K/V rows
// and lse/delta are loaded into registers as soon as the loop is done, under the dK/dV stores
// (one workgroup per pair left each CU idle during every prologue load).  Queries >= N get
// L2 = +inf -> P = 0, dS = 0.
template <int NPMAX, int NWC = 0>   // NWC: see attn_bwd_dq_seq_bf16
__global__ __launch_bounds__(NPMAX * 2) void attn_bwd_dkv_seq_bf16(
    const bf16* __restrict__ qkv, const bf16* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, bf16* __restrict__ dqkv, int N, int H, float scale,
    float* __restrict__ colsum, int npairs) {
  __shared__ __attribute__((aligned(16))) char smem[2][2 * NPMAX * 128];   // [buffer][Q | dO]
  __shared__ __attribute__((aligned(16))) float l2s[NPMAX];
  __shared__ __attribute__((aligned(16))) float dls[NPMAX];
  __shared__ float red[NPMAX / 32][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = NWC > 0 ? NWC : blockDim.x >> 6, NP = nw * 32;
  const int D = H * DH;
  const int64_t ld = 3 * (int64_t)D, ldb = ld * 2, ldo = (int64_t)D * 2;
  const int h = lane >> 5;
  const uint32_t bytes = (uint32_t)((int64_t)N * ldb);
  const uint32_t obytes = (uint32_t)((int64_t)N * ldo);
  const int key = wave * 32 + (lane & 31);
  const float c2 = scale * LOG2E;
  auto stage_pair = [&](int bh, int buf) {
    const int b = bh / H, hd = bh - b * H;
    const bf16* base = qkv + (int64_t)b * N * ld;
    stage_seq_dma(smem[buf], make_rsrc(base + hd * DH, bytes - hd * DH * 2), ldb, NP, nw, wave, lane);
    stage_seq_dma(smem[buf] + NP * 128, make_rsrc(dout + (int64_t)b * N * D + hd * DH, obytes - hd * DH * 2), ldo, NP,
              nw, wave, lane);
  };
  auto load_regs = [&](int bh, bf16x8 (&kf)[4], bf16x8 (&vf)[4], float& ls, float& dv) {
    const int b = bh / H, hd = bh - b * H;
    const bf16* base = qkv + (int64_t)b * N * ld;
    const __amdgpu_buffer_rsrc_t rk = make_rsrc(base + D + hd * DH, bytes - (D + hd * DH) * 2);
    const __amdgpu_buffer_rsrc_t rv = make_rsrc(base + 2 * D + hd * DH, bytes - (2 * D + hd * DH) * 2);
    // inline-asm loads (see the loop head): the range check returns 0 past N
    const uint32_t kvoff = (uint32_t)((int64_t)key * ldb + 16 * h);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kf[s] = __builtin_bit_cast(bf16x8, asm_load16(rk, kvoff, 32 * s));
      vf[s] = __builtin_bit_cast(bf16x8, asm_load16(rv, kvoff, 32 * s));
    }
    const uint32_t ioff = (uint32_t)threadIdx.x * 4;
    ls = asm_load4(make_rsrc(lse + (int64_t)bh * N, (uint32_t)N * 4), ioff);
    dv = asm_load4(make_rsrc(delta + (int64_t)bh * N, (uint32_t)N * 4), ioff);
  };

  int bh = blockIdx.x;
  if (bh >= npairs) return;
  bf16x8 kf[4], vf[4];
  float ls, dv;
  stage_pair(bh, 0);
  load_regs(bh, kf, vf, ls, dv);
  int buf = 0;
  bool first = true;
  for (;;) {
    // this pair's Q | dO pieces and register loads: everything but the previous pair's dK/dV
    // stores (8 per wave, + 2 column-sum stores on wave 0), which are younger
    if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (colsum && wave == 0) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    first = false;
    // The K/V rows, lse and delta arrive by inline-asm loads and the next pair's Q | dO by
    // inline-asm LDS-DMA (dma_piece): with compiler-visible loads hipcc waited vmcnt(0) here
    // (the merge of the prologue and loop-carried states), draining the prefetch every pair.
    // The wait above retired them; this statement is their definition point for the compiler.
    asm volatile("" : "+v"(kf[0]), "+v"(kf[1]), "+v"(kf[2]), "+v"(kf[3]), "+v"(vf[0]), "+v"(vf[1]), "+v"(vf[2]),
                 "+v"(vf[3]), "+v"(ls), "+v"(dv));
    if (threadIdx.x < NP) {
      const int i = threadIdx.x;
      l2s[i] = i < N ? ls * LOG2E : INFINITY;
      dls[i] = i < N ? dv : 0.f;
    }
    __syncthreads();   // Q | dO and l2s / dls visible; every wave is done with the other buffer
    const int nbh = bh + gridDim.x;
    const bool more = nbh < npairs;
    if (more) stage_pair(nbh, buf ^ 1);
    const char* qt = smem[buf];
    const char* dt_ = qt + NP * 128;
    f32x16 dvt[2] = {zero16(), zero16()}, dkt[2] = {zero16(), zero16()};
    auto qblock = [&](const int q0) {
      f32x16 sa = zero16(), dp;
      // the row constants first: dP - delta straight from the MFMA chain (accumulator started
      // at -delta of each query row), so dS = P (dP - delta) is one multiply per element
      f32x4 L2[4];
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int q4 = q0 + 8 * g4 + 4 * h;   // rows acc_row(4*g4 + i, h) = q4 + i
        L2[g4] = *(const f32x4*)(l2s + q4);
        const f32x4 dl = *(const f32x4*)(dls + q4);
#pragma unroll
        for (int i = 0; i < 4; ++i) dp[4 * g4 + i] = VITMI_ATT_DPINIT ? -dl[i] : 0.f;
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sa = mfma32(frag_row(qt, q0, s, lane), kf[s], sa);    // S[q][key]
        dp = mfma32(frag_row(dt_, q0, s, lane), vf[s], dp);   // dP[q][key] - delta[q]
      }
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        [[maybe_unused]] const f32x4 dl = VITMI_ATT_DPINIT ? f32x4{} : *(const f32x4*)(dls + q0 + 8 * g4 + 4 * h);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = fexp2(fmaf(sa[4 * g4 + i], c2, -L2[g4][i]));
          sa[4 * g4 + i] = p;
          dp[4 * g4 + i] = VITMI_ATT_DPINIT ? p * dp[4 * g4 + i] : p * (dp[4 * g4 + i] - dl[i]);
        }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pb = pack8(sa, s), sb = pack8(dp, s);
#pragma unroll
        for (int d2 = 0; d2 < 2; ++d2) {
          dvt[d2] = mfma32(frag_tr(dt_, q0 + 16 * s, 32 * d2, lane), pb, dvt[d2]);
          dkt[d2] = mfma32(frag_tr(qt, q0 + 16 * s, 32 * d2, lane), sb, dkt[d2]);
        }
      }
    };
    if constexpr (NWC > 0) {
#pragma unroll
      for (int q0 = 0; q0 < NWC * 32; q0 += 32) qblock(q0);
    } else {
#pragma unroll 1
      for (int q0 = 0; q0 < NP; q0 += 32) qblock(q0);
    }
    if (more) load_regs(nbh, kf, vf, ls, dv);   // (kf / vf are dead until the next pair)
    // dK, dV through this pair's (now free) Q | dO image: every wave must be done reading it
    __syncthreads();
    {
      const int b = bh / H, hd = bh - b * H;
      const bf16* db = dqkv + (int64_t)b * N * ld;
      const __amdgpu_buffer_rsrc_t rdk = make_rsrc(db + D + hd * DH, bytes - (D + hd * DH) * 2);
      const __amdgpu_buffer_rsrc_t rdv = make_rsrc(db + 2 * D + hd * DH, bytes - (2 * D + hd * DH) * 2);
      char* scr = smem[buf] + wave * ST_BYTES;
      float* part = colsum + (int64_t)b * 3 * D + hd * DH;   // the k- and v-bias gradient partials
      const int ln = lane_here();
      store_tile32(scr, dkt, scale, rdk, ldb, wave * 32, ln);
      if (colsum) tile32_colsum(scr, wave * 32, N, part + D, red, wave, nw, ln);
      store_tile32(scr, dvt, 1.f, rdv, ldb, wave * 32, ln);
      if (colsum) tile32_colsum(scr, wave * 32, N, part + 2 * D, red, wave, nw, ln);
    }
    if (!more) break;
    bh = nbh;
    buf ^= 1;
  }
}

// ============================================== single-pass backward (bf16, N <= 32 * 7 = 224)
// dQ, dK and dV of one (batch, head) in ONE workgroup that loads Q, K, V, dO and O once (the
// two-kernel path above loads them twice: the dQ kernel's K / V and Q / dO loads were half of its
// time).  NKB = ceil(N / 32) waves; wave w owns key block w.
//   prologue  Q and dO images into LDS (LDS-DMA), the wave's K / V rows into registers, delta =
//             rowsum(dO * O) of the wave's 32 query rows (as the dQ kernel forms it) and lse into
//             LDS row tables.
//   phase 1   per query block: S, P, dP - delta and dS = P (dP - delta) with the keys on the lanes
//             (the dK/dV kernel's arithmetic, in the same order: dK and dV are bitwise its), dV +=
//             dO^T P and dK += Q^T dS in registers, and dS^T (bf16, the value dK takes) into an LDS
//             tile [key block][query block] of [32 keys][32 queries].
//   phase 2   the K rows go from registers into the (now free) Q image; wave w takes query block w:
//             dQ = dS K over all key blocks from the dS^T tiles (transposed reads) and the K image.
//   epilogue  dQ, dK, dV leave through per-wave LDS images as whole lines (store_tile32), with the
//             q/k/v bias-gradient column sums as the two-kernel path forms them.
// LDS: Q + dO images 2 x 28 KiB, dS^T tiles NKB^2 x 2 KiB (98 KiB at NKB = 7), row tables: one
// workgroup per CU, as the persistent dK/dV kernel.  No atomics; fixed summation orders.
// dS^T tile: 64-B rows (32 queries), 16-B chunk c of row r at c ^ ((r >> 2) & 3): the phase-2
// ds_read_b64_tr_b16 reads are conflict free, the phase-1 8-B writes 2-way.
__device__ __forceinline__ int ds_off(int row, int ch) { return row * 64 + ((ch ^ ((row >> 2) & 3)) << 4); }
// frag_tr over a [32][32] tile of 64-B rows: operand X^T[col][k] of the tile X[k][col], element j
// <-> k-row k0 + 8(j>>2) + 4h + (j&3), col = lane & 31 (frag_tr's k order, c0 = 0)
__device__ __forceinline__ bf16x8 frag_tr32(const char* t, int k0, int lane) {
  const int g = lane >> 4, tl = lane & 15, q = tl >> 2, p = tl & 3;
  bf16x8 f;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = k0 + 8 * i + 4 * (g >> 1) + q;
    s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        LDS_PTR(s16x4, t + ds_off(row, 2 * (g & 1) + (p >> 1)) + ((p & 1) << 3)));
    bf16x4 b = __builtin_bit_cast(bf16x4, v);
    f[4 * i + 0] = b[0];
    f[4 * i + 1] = b[1];
    f[4 * i + 2] = b[2];
    f[4 * i + 3] = b[3];
  }
  return f;
}

template <int NKB>
__global__ __launch_bounds__(NKB * 64) void attn_bwd_fused_seq_bf16(
    const bf16* __restrict__ qkv, const bf16* __restrict__ o, const bf16* __restrict__ dout,
    const float* __restrict__ lse, float* __restrict__ delta, bf16* __restrict__ dqkv, int N, int H,
    float scale, float* __restrict__ colsum, int npairs) {
  constexpr int NP = NKB * 32;
  constexpr int IMG = NP * 128;     // one [NP][64] bf16 image
  constexpr int DT = 32 * 64;       // one dS^T tile [32 keys][32 queries] bf16
  // the dS^T tiles, and in the epilogue the waves' three output images
  constexpr int AREA = NKB * NKB * DT > 3 * NKB * ST_BYTES ? NKB * NKB * DT : 3 * NKB * ST_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[2 * IMG + AREA];
  // phase 1: the lse / delta row tables; epilogue: the column-sum partials [3][NKB][64]
  __shared__ __attribute__((aligned(16))) float tab[3 * NKB * 64];
  float* l2s = tab;
  float* dls = tab + NP;
  float (*red)[NKB][64] = reinterpret_cast<float (*)[NKB][64]>(tab);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int D = H * DH;
  const int64_t ld = 3 * (int64_t)D, ldb = ld * 2, ldo = (int64_t)D * 2;
  const int h = lane >> 5;
  const uint32_t bytes = (uint32_t)((int64_t)N * ldb);
  const uint32_t obytes = (uint32_t)((int64_t)N * ldo);
  char* qt = smem;                 // Q image; phase 2: the K image
  char* dt_ = smem + IMG;          // dO image
  char* dst = smem + 2 * IMG;      // dS^T tiles [key block][query block]; epilogue: output images
  const int r32 = wave * 32 + (lane & 31);   // this lane's key (phase 1) and query (delta, phase 2)
  const int kl = lane & 31;
  const float c2 = scale * LOG2E;
  // (batch, head) pairs in DESCENDING order (the out-proj dgrad writing dO finished with the last
  // rows); pair i of this workgroup's walk is blockIdx.x + i * gridDim.x
  auto pair_of = [&](int i) { return npairs - 1 - i; };
  // Loads of a pair.  Q and dO images by inline-asm LDS-DMA (dma_piece) and the K / V / O rows and
  // lse into registers by inline-asm loads: with compiler-visible loads hipcc drains the prefetch
  // with vmcnt(0) at the first LDS access it cannot prove disjoint (attn_bwd_dkv_seq_bf16's note);
  // the kernel's own counted waits retire them.  Rows past N come back zero (range check).
  auto stage_q = [&](int bh) {
    const int b = bh / H, hd = bh - b * H;
    stage_seq_dma(qt, make_rsrc(qkv + (int64_t)b * N * ld + hd * DH, bytes - hd * DH * 2), ldb, NP, NKB, wave, lane);
  };
  auto stage_do = [&](int bh) {
    const int b = bh / H, hd = bh - b * H;
    stage_seq_dma(dt_, make_rsrc(dout + (int64_t)b * N * D + hd * DH, obytes - hd * DH * 2), ldo, NP, NKB, wave, lane);
  };
// Where the next pair's loads go (round 6, profiles/r06_pf5/): 5 = the O rows right after delta (their
// last use), the dO image DMA and the K / V rows + lse after phase 1.  Each lane's 16-B row pieces
// touch 32 lines per instruction, and the cost of those loads (~1.5 us per 4 instructions per wave)
// lands in whichever phase follows their issue; the O rows hide behind the delta barrier and phase 1
// (per layer 212-219 vs 234-243 us).  1 = all of them after phase 1, 0 = after phase 2, 2 / 3 = the
// DMA / the register rows after phase 2, 6 / 7 = K / V spread over phase 2 (and O over phase 1):
// measured, not better than 5.
#ifndef VITMI_FUSED_PF
#define VITMI_FUSED_PF 5
#endif
  // the O rows alone (VITMI_FUSED_PF 5 issues them right after delta, their last use)
  auto load_o = [&](int bh, bf16x8 (&of)[4], int s0 = 0, int s1 = 4) {
    const int b = bh / H, hd = bh - b * H;
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(o + (int64_t)b * N * D + hd * DH, obytes - hd * DH * 2);
    const uint32_t ooff = (uint32_t)((int64_t)r32 * ldo + 16 * h);
#pragma unroll
    for (int s = s0; s < s1; ++s) of[s] = __builtin_bit_cast(bf16x8, asm_load16(ro, ooff, 32 * s));
  };
  // one 16-B piece of the lane's K and V rows (VITMI_FUSED_PF 6 spreads them over phase 2)
  auto load_kv1 = [&](int bh, bf16x8 (&kf)[4], bf16x8 (&vf)[4], int s) {
    const int b = bh / H, hd = bh - b * H;
    const bf16* base = qkv + (int64_t)b * N * ld;
    const __amdgpu_buffer_rsrc_t rk = make_rsrc(base + D + hd * DH, bytes - (D + hd * DH) * 2);
    const __amdgpu_buffer_rsrc_t rv = make_rsrc(base + 2 * D + hd * DH, bytes - (2 * D + hd * DH) * 2);
    const uint32_t kvoff = (uint32_t)((int64_t)r32 * ldb + 16 * h);
    kf[s] = __builtin_bit_cast(bf16x8, asm_load16(rk, kvoff, 32 * s));
    vf[s] = __builtin_bit_cast(bf16x8, asm_load16(rv, kvoff, 32 * s));
  };
  auto load_regs = [&](int bh, bf16x8 (&kf)[4], bf16x8 (&vf)[4], bf16x8 (&of)[4], float& ls, bool with_o = true) {
    const int b = bh / H, hd = bh - b * H;
    const bf16* base = qkv + (int64_t)b * N * ld;
    const __amdgpu_buffer_rsrc_t rk = make_rsrc(base + D + hd * DH, bytes - (D + hd * DH) * 2);
    const __amdgpu_buffer_rsrc_t rv = make_rsrc(base + 2 * D + hd * DH, bytes - (2 * D + hd * DH) * 2);
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(o + (int64_t)b * N * D + hd * DH, obytes - hd * DH * 2);
    const uint32_t kvoff = (uint32_t)((int64_t)r32 * ldb + 16 * h), ooff = (uint32_t)((int64_t)r32 * ldo + 16 * h);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kf[s] = __builtin_bit_cast(bf16x8, asm_load16(rk, kvoff, 32 * s));
      vf[s] = __builtin_bit_cast(bf16x8, asm_load16(rv, kvoff, 32 * s));
      if (with_o) of[s] = __builtin_bit_cast(bf16x8, asm_load16(ro, ooff, 32 * s));
    }
    ls = asm_load4(make_rsrc(lse + (int64_t)bh * N, (uint32_t)N * 4), (uint32_t)r32 * 4);
  };

  int i = blockIdx.x;
  if (i >= npairs) return;
  int bh = pair_of(i);
  bf16x8 kf[4], vf[4], of[4];
  float ls;
  stage_q(bh);
  stage_do(bh);
  load_regs(bh, kf, vf, of, ls);
  bool first = true;
  for (;;) {
    // everything this pair needs has landed: all but the youngest 12 vector-memory ops, which are
    // the previous pair's output stores (12 per wave; the column-sum stores after them, 0..3 per
    // wave, only make this wait stricter)
    if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    first = false;
    asm volatile("" : "+v"(kf[0]), "+v"(kf[1]), "+v"(kf[2]), "+v"(kf[3]), "+v"(vf[0]), "+v"(vf[1]), "+v"(vf[2]),
                 "+v"(vf[3]), "+v"(of[0]), "+v"(of[1]), "+v"(of[2]), "+v"(of[3]), "+v"(ls));
    __syncthreads();   // every wave's Q | dO pieces landed; the previous epilogue is done with tab
    FUSED_STAMP(bh, 0);
    const int b = bh / H, hd = bh - b * H;
    {
      // delta of query row r32 from the dO image and the O row, summed as attn_bwd_dq_seq_bf16
      // does (bitwise the same value)
      float part = 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 df = *(const bf16x8*)(dt_ + toff(r32, 2 * s + h));
#pragma unroll
        for (int j = 0; j < 8; ++j) part += (float)of[s][j] * (float)df[j];
      }
      const float dl = part + __shfl_xor(part, 32, 64);
      const bool ok = r32 < N;
      if (h == 0) {
        l2s[r32] = ok ? ls * LOG2E : INFINITY;   // queries >= N: P = 0
        dls[r32] = ok ? dl : 0.f;
        if (ok) delta[(int64_t)bh * N + r32] = dl;
      }
    }
    const bool more1 = i + (int)gridDim.x < npairs;
    const int nbh1 = more1 ? pair_of(i + gridDim.x) : 0;
    if ((VITMI_FUSED_PF == 5 || VITMI_FUSED_PF == 6) && more1) load_o(pair_of(i + gridDim.x), of);   // (of is dead)
    __syncthreads();
    FUSED_STAMP(bh, 1);

    // ---- phase 1: keys on the lanes (the dK/dV kernel's qblock, plus the dS^T tile)
    f32x16 dvt[2] = {zero16(), zero16()}, dkt[2] = {zero16(), zero16()};
#pragma unroll
    for (int qb = 0; qb < NKB; ++qb) {
      const int q0 = 32 * qb;
      f32x16 sa = zero16(), dp;
      f32x4 L2[4];
      if (VITMI_FUSED_PF == 7 && more1 && qb < 4) load_o(nbh1, of, qb, qb + 1);   // (of is dead after delta)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int q4 = q0 + 8 * g4 + 4 * h;
        L2[g4] = *(const f32x4*)(l2s + q4);
        const f32x4 dl = *(const f32x4*)(dls + q4);
#pragma unroll
        for (int e = 0; e < 4; ++e) dp[4 * g4 + e] = -dl[e];
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sa = mfma32(frag_row(qt, q0, s, lane), kf[s], sa);    // S[q][key]
        dp = mfma32(frag_row(dt_, q0, s, lane), vf[s], dp);   // dP[q][key] - delta[q]
      }
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float p = fexp2(fmaf(sa[4 * g4 + e], c2, -L2[g4][e]));
          sa[4 * g4 + e] = p;
          dp[4 * g4 + e] = p * dp[4 * g4 + e];
        }
      char* tile = dst + (wave * NKB + qb) * DT;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pb = pack8(sa, s), sb = pack8(dp, s);
#pragma unroll
        for (int d2 = 0; d2 < 2; ++d2) {
          dvt[d2] = mfma32(frag_tr(dt_, q0 + 16 * s, 32 * d2, lane), pb, dvt[d2]);
          dkt[d2] = mfma32(frag_tr(qt, q0 + 16 * s, 32 * d2, lane), sb, dkt[d2]);
        }
        // dS^T[key][q]: elements 0..3 are queries 16s + 4h + 0..3 (chunk 2s), 4..7 are 16s + 8 +
        // 4h + 0..3 (chunk 2s + 1), half h of each chunk
        bf16x4 lo4, hi4;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          lo4[j] = sb[j];
          hi4[j] = sb[4 + j];
        }
        *(bf16x4*)(tile + ds_off(kl, 2 * s) + 8 * h) = lo4;
        *(bf16x4*)(tile + ds_off(kl, 2 * s + 1) + 8 * h) = hi4;
      }
    }
    __syncthreads();   // every wave is done with the Q and dO images and wrote its dS^T tiles
    FUSED_STAMP(bh, 2);
    // the K image where Q was: row r32 = this lane's key, chunk 2s + h holds d = 16s + 8h .. +7
#pragma unroll
    for (int s = 0; s < 4; ++s) *(bf16x8*)(qt + toff(r32, 2 * s + h)) = kf[s];
    const int inext = i + gridDim.x;
    const bool more = inext < npairs;
    const int nbh = more ? pair_of(inext) : 0;
    // the next pair's dO image (the dO image is free) and register rows (kf / vf / of are dead)
    // land under phase 2 and the epilogue
    if (more && VITMI_FUSED_PF == 1) {
      stage_do(nbh);
      load_regs(nbh, kf, vf, of, ls);
    }
    if (more && VITMI_FUSED_PF == 2) load_regs(nbh, kf, vf, of, ls);
    if (more && VITMI_FUSED_PF == 3) stage_do(nbh);
    if (more && VITMI_FUSED_PF == 5) {
      stage_do(nbh);
      load_regs(nbh, kf, vf, of, ls, false);
    }
    if (more && (VITMI_FUSED_PF == 6 || VITMI_FUSED_PF == 7)) {
      stage_do(nbh);
      ls = asm_load4(make_rsrc(lse + (int64_t)nbh * N, (uint32_t)N * 4), (uint32_t)r32 * 4);
    }
    __syncthreads();

    // ---- phase 2: wave w takes query block w: dQ^T[d][q] = sum_key K^T[d][key] dS^T[key][q]
    f32x16 dqt[2] = {zero16(), zero16()};
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
      const char* tile = dst + (kb * NKB + wave) * DT;
      if ((VITMI_FUSED_PF == 6 || VITMI_FUSED_PF == 7) && more && kb < 4) load_kv1(nbh, kf, vf, kb);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 sf = frag_tr32(tile, 16 * s, lane);
#pragma unroll
        for (int d2 = 0; d2 < 2; ++d2) dqt[d2] = mfma32(frag_tr(qt, 32 * kb + 16 * s, 32 * d2, lane), sf, dqt[d2]);
      }
    }
    __syncthreads();   // the K image is free (the next Q lands there); dS^T area -> output images
    FUSED_STAMP(bh, 3);
    if (more) stage_q(nbh);
    if (more && VITMI_FUSED_PF == 0) {
      stage_do(nbh);
      load_regs(nbh, kf, vf, of, ls);
    }
    if (more && VITMI_FUSED_PF == 2) stage_do(nbh);
    if (more && VITMI_FUSED_PF == 3) load_regs(nbh, kf, vf, of, ls);

    // ---- epilogue: dQ, dK, dV through three images per wave, then their column sums (the q/k/v
    // bias-gradient partials of this batch row) in one pass, folded in wave order
    {
      const bf16* dbase = dqkv + (int64_t)b * N * ld;
      const __amdgpu_buffer_rsrc_t rdq = make_rsrc(dbase + hd * DH, bytes - hd * DH * 2);
      const __amdgpu_buffer_rsrc_t rdk = make_rsrc(dbase + D + hd * DH, bytes - (D + hd * DH) * 2);
      const __amdgpu_buffer_rsrc_t rdv = make_rsrc(dbase + 2 * D + hd * DH, bytes - (2 * D + hd * DH) * 2);
      char* scr = dst + 3 * wave * ST_BYTES;
      const int ln = lane_here();
      store_tile32(scr, dqt, scale, rdq, ldb, wave * 32, ln);
      store_tile32(scr + ST_BYTES, dkt, scale, rdk, ldb, wave * 32, ln);
      store_tile32(scr + 2 * ST_BYTES, dvt, 1.f, rdv, ldb, wave * 32, ln);
      if (colsum) {
        // tile32_colsum's sums per image (rows < N, 4 rows x 8 columns per lane, xor folds)
        const int rr = ln >> 3, cc = ln & 7, row0 = wave * 32;
#pragma unroll
        for (int im = 0; im < 3; ++im) {
          float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (row0 + 8 * j + rr < N) {
              const bf16x8 v = *(const bf16x8*)(scr + im * ST_BYTES + (8 * j + rr) * ST_PITCH + cc * 16);
#pragma unroll
              for (int e = 0; e < 8; ++e) cs[e] += (float)v[e];
            }
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            cs[e] += __shfl_xor(cs[e], 8, 64);
            cs[e] += __shfl_xor(cs[e], 16, 64);
            cs[e] += __shfl_xor(cs[e], 32, 64);
          }
          if (ln < 8) {
#pragma unroll
            for (int e = 0; e < 8; ++e) red[im][wave][ln * 8 + e] = cs[e];
          }
        }
        __syncthreads();
        for (int x = threadIdx.x; x < 192; x += NKB * 64) {   // (fewer than 3 waves: several each)
          const int im = x >> 6, c = x & 63;
          float t = 0.f;
          for (int w = 0; w < NKB; ++w) t += red[im][w][c];
          colsum[(int64_t)b * 3 * D + im * D + hd * DH + c] = t;
        }
      }
    }
    FUSED_STAMP(bh, 4);
    if (!more) break;
    i = inext;
    bh = nbh;
  }
}

// =============================================================== fp32 path (MFMA, N <= NPMAX)
// The fp32 parity configuration on the fp32 matrix cores (v_mfma_f32_32x32x2_f32: full fp32
// products and sums, no reduced-precision operand), with the whole-sequence structure of the
// bf16 kernels: wave w owns 32 rows (queries, or keys in dK/dV), the other operand's sequence
// sits in LDS as fp32 [NP][FP] images.  A 32x32x2 step consumes d = 32h + t on lane half h
// (any pairing of d with steps is a valid reduction order as long as both operands use it), so
// a lane's register row is 32 contiguous floats and the LDS operand is one ds_read_b128 per four
// steps.  The P.V-type products take P (or dS) straight from the accumulator registers: step r
// pairs the two rows acc_row(r, 0/1) the lane halves hold, and reads the matching LDS rows as
// the A operand (ds_read_b32, 32 consecutive floats per half).  exp is expf (natural) as in the
// VALU kernels; lse is natural-log.
static constexpr int FP = 68;   // image pitch in floats: 16 rows of a b128 read land 16 B apart mod 256 B

__device__ __forceinline__ f32x16 mfma_f32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// rows [0, NP) of one head's 64 columns (rows >= N zero) -> LDS image [NP][FP]; the block has
// 64 * NP / 32 = 2 NP threads, so each moves 8 of the NP * 16 float4 pieces
__device__ __forceinline__ void stage_seq_f32(float* img, const float* __restrict__ src, int64_t ld, int N) {
  const int nt = blockDim.x;
  f32x4 v[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int i = threadIdx.x + t * nt, r = i >> 4, c = (i & 15) * 4;
    v[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (r < N) v[t] = *(const f32x4*)(src + (int64_t)r * ld + c);
  }
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int i = threadIdx.x + t * nt, r = i >> 4, c = (i & 15) * 4;
    *(f32x4*)(img + r * FP + c) = v[t];
  }
}

// the lane's half-row of a head: x[32h + t], t < 32 (zero when the row is >= N), times mul
__device__ __forceinline__ void load_half_row(float (&x)[32], const float* __restrict__ row, bool ok, int h,
                                              float mul) {
#pragma unroll
  for (int t = 0; t < 32; t += 4) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (ok) v = *(const f32x4*)(row + 32 * h + t);
#pragma unroll
    for (int e = 0; e < 4; ++e) x[t + e] = v[e] * mul;
  }
}

// acc[i][j] += sum_d img[rb + i][d] * x_j[d], with lane j's register half-row x (d = 32h + t)
__device__ __forceinline__ f32x16 sblock_f32(const float* img, int rb, const float (&x)[32], int lane, f32x16 acc) {
  const float* row = img + (rb + (lane & 31)) * FP + 32 * (lane >> 5);
#pragma unroll
  for (int t = 0; t < 32; t += 4) {
    const f32x4 a = *(const f32x4*)(row + t);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = mfma_f32(a[e], x[t + e], acc);
  }
  return acc;
}

// acc[dt][d][j] += sum_i img[rb + i][32 dt + d] * w[i][j], w = a 32x32 accumulator (row i = acc_row)
__device__ __forceinline__ void pvblock_f32(const float* img, int rb, const f32x16& w, int lane, f32x16 (&acc)[2]) {
  const float* base = img + rb * FP + (lane & 31);
  const int h = lane >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float* row = base + acc_row(r, h) * FP;
    acc[0] = mfma_f32(row[0], w[r], acc[0]);
    acc[1] = mfma_f32(row[32], w[r], acc[1]);
  }
}

// a wave's transposed 32 x 64 result (acc[dt]: lane j holds column j's d = 32 dt + acc_row(r, h))
// times mul -> rows row0 + j of dst (ld floats, rows >= N skipped), through the wave's LDS
// scratch [32][FP] so each row leaves as one 256-B line
__device__ __forceinline__ void store_tile32_f32(float* scr, const f32x16 (&acc)[2], float mul, float* dst, int64_t ld,
                                                 int row0, int N, int lane) {
  const int j = lane & 31, h = lane >> 5;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *(f32x4*)(scr + j * FP + 32 * dt + 8 * g + 4 * h) =
          f32x4{acc[dt][4 * g] * mul, acc[dt][4 * g + 1] * mul, acc[dt][4 * g + 2] * mul, acc[dt][4 * g + 3] * mul};
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const int c = (lane & 15) * 4;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int r = 4 * it + (lane >> 4);
    const f32x4 v = *(const f32x4*)(scr + r * FP + c);
    if (row0 + r < N) *(f32x4*)(dst + (int64_t)(row0 + r) * ld + c) = v;
  }
}

// grid B*H, block 64*NW (NW = ceil(N/32)); online softmax over key blocks of 32, keys >= N
// (only in the last block) masked
template <int NPMAX>
__global__ __launch_bounds__(NPMAX * 2) void attn_fwd_seq_f32(const float* __restrict__ qkv, float* __restrict__ o,
                                                              float* __restrict__ lse, int N, int H, float scale) {
  __shared__ __attribute__((aligned(16))) float smem[2 * NPMAX * FP];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int NP = (blockDim.x >> 6) * 32;
  const int bh = blockIdx.x, b = bh / H, hd = bh % H;
  const int D = H * DH;
  const int64_t ld = 3 * (int64_t)D;
  const float* base = qkv + (int64_t)b * N * ld;
  float* kt = smem;
  float* vt = smem + NP * FP;
  const int h = lane >> 5, q = wave * 32 + (lane & 31);
  stage_seq_f32(kt, base + D + hd * DH, ld, N);
  stage_seq_f32(vt, base + 2 * D + hd * DH, ld, N);
  float qr[32];
  load_half_row(qr, base + (int64_t)q * ld + hd * DH, q < N, h, scale);
  __syncthreads();

  float m = -INFINITY, l = 0.f;
  f32x16 oacc[2] = {zero16(), zero16()};
#pragma unroll 1
  for (int kb = 0; kb < NP; kb += 32) {
    f32x16 st = sblock_f32(kt, kb, qr, lane, zero16());   // S^T[key][q]
    if (kb + 32 > N) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (kb + acc_row(r, h) >= N) st[r] = -INFINITY;
    }
    float tmax = st[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) tmax = fmaxf(tmax, st[r]);
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mn = fmaxf(m, tmax);                 // finite: every block holds a key < N
    const float alpha = expf(m - mn);                // 0 on the first block
    m = mn;
    float rs = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = expf(st[r] - mn);
      st[r] = p;
      rs += p;
    }
    l = fmaf(l, alpha, rs);
    if (__builtin_amdgcn_ballot_w64(alpha != 1.f) != 0) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[dt][r] *= alpha;
    }
    pvblock_f32(vt, kb, st, lane, oacc);             // O^T[d][q] += V^T[d][key] P^T[key][q]
  }
  const float lt = l + __shfl_xor(l, 32, 64);
  if (q < N && h == 0) lse[(int64_t)bh * N + q] = m + logf(lt);
  __syncthreads();   // the K/V images are free: per-wave output scratch
  store_tile32_f32(smem + wave * 32 * FP, oacc, 1.f / lt, o + (int64_t)b * N * D + hd * DH, D, wave * 32, N, lane);
}

// dQ (+ delta = rowsum(dO * O)): grid B*H, block 64*NW, K and V images in LDS.  Keys >= N have
// zero K and V rows: their dS meets a zero K row in dQ = dS K.
template <int NPMAX>
__global__ __launch_bounds__(NPMAX * 2) void attn_bwd_dq_seq_f32(const float* __restrict__ qkv,
                                                                 const float* __restrict__ o,
                                                                 const float* __restrict__ dout,
                                                                 const float* __restrict__ lse,
                                                                 float* __restrict__ delta, float* __restrict__ dqkv,
                                                                 int N, int H, float scale) {
  __shared__ __attribute__((aligned(16))) float smem[2 * NPMAX * FP];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int NP = (blockDim.x >> 6) * 32;
  const int bh = blockIdx.x, b = bh / H, hd = bh % H;
  const int D = H * DH;
  const int64_t ld = 3 * (int64_t)D;
  const float* base = qkv + (int64_t)b * N * ld;
  float* kt = smem;
  float* vt = smem + NP * FP;
  const int h = lane >> 5, q = wave * 32 + (lane & 31);
  const bool qok = q < N;
  stage_seq_f32(kt, base + D + hd * DH, ld, N);
  stage_seq_f32(vt, base + 2 * D + hd * DH, ld, N);
  float dr[32], qr[32];
  float dl;
  {
    float orow[32];
    load_half_row(dr, dout + ((int64_t)b * N + q) * D + hd * DH, qok, h, 1.f);
    load_half_row(orow, o + ((int64_t)b * N + q) * D + hd * DH, qok, h, 1.f);
    float c[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 32; ++t) c[t & 3] = fmaf(orow[t], dr[t], c[t & 3]);
    const float part = (c[0] + c[1]) + (c[2] + c[3]);
    dl = part + __shfl_xor(part, 32, 64);
  }
  if (qok && h == 0) delta[(int64_t)bh * N + q] = dl;
  load_half_row(qr, base + (int64_t)q * ld + hd * DH, qok, h, scale);
  const float L = qok ? lse[(int64_t)bh * N + q] : INFINITY;   // q >= N -> P = 0
  __syncthreads();

  f32x16 dqa[2] = {zero16(), zero16()};
#pragma unroll 1
  for (int kb = 0; kb < NP; kb += 32) {
    const f32x16 st = sblock_f32(kt, kb, qr, lane, zero16());   // S^T[key][q]
    f32x16 dp = sblock_f32(vt, kb, dr, lane, zero16());         // dP^T[key][q]
#pragma unroll
    for (int r = 0; r < 16; ++r) dp[r] = expf(st[r] - L) * (dp[r] - dl);
    pvblock_f32(kt, kb, dp, lane, dqa);                         // dQ^T[d][q] += K^T[d][key] dS^T[key][q]
  }
  __syncthreads();
  store_tile32_f32(smem + wave * 32 * FP, dqa, scale, dqkv + (int64_t)b * N * ld + hd * DH, ld, wave * 32, N, lane);
}

// dK / dV: grid B*H, block 64*NW, wave w owns keys 32w..+31 (K scaled and V half-rows in
// registers), Q and dO images in LDS.  Queries >= N get lse = +inf -> P = 0, dS = 0.
template <int NPMAX>
__global__ __launch_bounds__(NPMAX * 2) void attn_bwd_dkv_seq_f32(const float* __restrict__ qkv,
                                                                  const float* __restrict__ dout,
                                                                  const float* __restrict__ lse,
                                                                  const float* __restrict__ delta,
                                                                  float* __restrict__ dqkv, int N, int H,
                                                                  float scale) {
  __shared__ __attribute__((aligned(16))) float smem[2 * NPMAX * FP];
  __shared__ __attribute__((aligned(16))) float ls[NPMAX];
  __shared__ __attribute__((aligned(16))) float dls[NPMAX];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int NP = (blockDim.x >> 6) * 32;
  const int bh = blockIdx.x, b = bh / H, hd = bh % H;
  const int D = H * DH;
  const int64_t ld = 3 * (int64_t)D;
  const float* base = qkv + (int64_t)b * N * ld;
  float* qt = smem;
  float* dt_ = smem + NP * FP;
  const int h = lane >> 5, key = wave * 32 + (lane & 31);
  stage_seq_f32(qt, base + hd * DH, ld, N);
  stage_seq_f32(dt_, dout + (int64_t)b * N * D + hd * DH, D, N);
  float kr[32], vr[32];
  load_half_row(kr, base + (int64_t)key * ld + D + hd * DH, key < N, h, scale);
  load_half_row(vr, base + (int64_t)key * ld + 2 * D + hd * DH, key < N, h, 1.f);
  if (threadIdx.x < NP) {
    const int i = threadIdx.x;
    ls[i] = i < N ? lse[(int64_t)bh * N + i] : INFINITY;
    dls[i] = i < N ? delta[(int64_t)bh * N + i] : 0.f;
  }
  __syncthreads();

  f32x16 dka[2] = {zero16(), zero16()}, dva[2] = {zero16(), zero16()};
#pragma unroll 1
  for (int q0 = 0; q0 < NP; q0 += 32) {
    f32x16 sa = sblock_f32(qt, q0, kr, lane, zero16());    // S[q][key]
    f32x16 dp = sblock_f32(dt_, q0, vr, lane, zero16());   // dP[q][key]
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int q4 = q0 + 8 * g4 + 4 * h;                   // rows acc_row(4*g4 + i, h) = q4 + i
      const f32x4 L = *(const f32x4*)(ls + q4);
      const f32x4 dl = *(const f32x4*)(dls + q4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = expf(sa[4 * g4 + i] - L[i]);
        sa[4 * g4 + i] = p;
        dp[4 * g4 + i] = p * (dp[4 * g4 + i] - dl[i]);
      }
    }
    pvblock_f32(dt_, q0, sa, lane, dva);   // dV^T[d][key] += dO^T[d][q] P[q][key]
    pvblock_f32(qt, q0, dp, lane, dka);    // dK^T[d][key] += Q^T[d][q] dS[q][key]
  }
  __syncthreads();
  float* scr = smem + wave * 32 * FP;
  float* db = dqkv + (int64_t)b * N * ld + hd * DH;
  store_tile32_f32(scr, dka, scale, db + D, ld, wave * 32, N, lane);
  store_tile32_f32(scr, dva, 1.f, db + 2 * D, ld, wave * 32, N, lane);
}

// =============================================================== fp32 path (VALU, N > NPMAX)
// Exact fp32 (expf, fp32 FMA; the parity configuration) for sequences longer than the MFMA
// kernels' LDS images (and policy 1).  Four lanes per row, each holding 16
// of its 64 head dims: a dot product is 16 FMAs in 4 independent chains plus a quad xor-reduce,
// and a row's state (q / dO / K / V and the accumulators) fits in <= 64 registers, so a SIMD
// holds several waves.  (One thread per row with 64-float arrays had 1 wave per SIMD and
// 64-long dependent FMA chains: 2.1 ms per ViT-S dK/dV call.)  K/V (or Q/dO) chunks of 64 rows
// are staged in LDS; a wave's 16 rows read the same LDS row (4 distinct addresses per read).
static constexpr int F32_CH = 64;

__device__ __forceinline__ float quad_sum(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  return v;
}
// sum_d a[d] * b[d] over one lane's 16 dims (4 chains)
__device__ __forceinline__ float dot16(const float (&a)[16], const float* __restrict__ b) {
  float c[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const f32x4 v = *(const f32x4*)(b + 4 * t);
#pragma unroll
    for (int e = 0; e < 4; ++e) c[e] = fmaf(a[4 * t + e], v[e], c[e]);
  }
  return (c[0] + c[1]) + (c[2] + c[3]);
}
// rows [r0, r0 + 64) of a head's 64 columns (rows >= N zero) -> LDS [64][DH], 256 threads
__device__ __forceinline__ void stage_chunk_f32(float (*dst)[DH], const float* __restrict__ src, int64_t ld,
                                                int r0, int N) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int i = threadIdx.x + 256 * t, r = i >> 4, c = (i & 15) * 4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (r0 + r < N) v = *(const f32x4*)(src + (int64_t)(r0 + r) * ld + c);
    *(f32x4*)(&dst[r][c]) = v;
  }
}

// grid (ceil(N/64), B*H), 256 threads: row q = 64 * blockIdx.x + tid / 4, dims 16 * (tid % 4) ..
__global__ __launch_bounds__(256) void attn_fwd_f32(const float* __restrict__ qkv,
                                                    float* __restrict__ o, float* __restrict__ lse,
                                                    int N, int H, float scale) {
  __shared__ __attribute__((aligned(16))) float ks[F32_CH][DH];
  __shared__ __attribute__((aligned(16))) float vs[F32_CH][DH];
  const int bh = blockIdx.y, b = bh / H, hd = bh % H;
  const int D = H * DH;
  const int64_t ld = 3 * (int64_t)D;
  const float* base = qkv + (int64_t)b * N * ld;
  const int q = blockIdx.x * 64 + (threadIdx.x >> 2), d0 = (threadIdx.x & 3) * 16;
  const bool ok = q < N;
  float qr[16], acc[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    qr[d] = ok ? base[(int64_t)q * ld + hd * DH + d0 + d] * scale : 0.f;
    acc[d] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < N; k0 += F32_CH) {
    __syncthreads();
    stage_chunk_f32(ks, base + D + hd * DH, ld, k0, N);
    stage_chunk_f32(vs, base + 2 * D + hd * DH, ld, k0, N);
    __syncthreads();
    const int kn = min(F32_CH, N - k0);
    for (int r = 0; r < kn; ++r) {
      const float s = quad_sum(dot16(qr, &ks[r][d0]));
      const float mn = fmaxf(m, s);
      const float a = expf(m - mn), p = expf(s - mn);
      l = l * a + p;
#pragma unroll
      for (int d = 0; d < 16; ++d) acc[d] = acc[d] * a + p * vs[r][d0 + d];
      m = mn;
    }
  }
  if (!ok) return;
  const float inv = 1.f / l;
  float* orow = o + ((int64_t)b * N + q) * D + hd * DH + d0;
#pragma unroll
  for (int t = 0; t < 4; ++t)
    *(f32x4*)(orow + 4 * t) = f32x4{acc[4 * t] * inv, acc[4 * t + 1] * inv, acc[4 * t + 2] * inv, acc[4 * t + 3] * inv};
  if ((threadIdx.x & 3) == 0) lse[(int64_t)bh * N + q] = m + logf(l);
}

// dQ (row = query) -- dq = scale * sum_k P (dP - delta) K
__global__ __launch_bounds__(256) void attn_bwd_dq_f32(const float* __restrict__ qkv,
                                                       const float* __restrict__ dout,
                                                       const float* __restrict__ lse,
                                                       const float* __restrict__ delta,
                                                       float* __restrict__ dqkv, int N, int H,
                                                       float scale) {
  __shared__ __attribute__((aligned(16))) float ks[F32_CH][DH];
  __shared__ __attribute__((aligned(16))) float vs[F32_CH][DH];
  const int bh = blockIdx.y, b = bh / H, hd = bh % H;
  const int D = H * DH;
  const int64_t ld = 3 * (int64_t)D;
  const float* base = qkv + (int64_t)b * N * ld;
  const int q = blockIdx.x * 64 + (threadIdx.x >> 2), d0 = (threadIdx.x & 3) * 16;
  const bool ok = q < N;
  float qr[16], dor[16], acc[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    qr[d] = ok ? base[(int64_t)q * ld + hd * DH + d0 + d] * scale : 0.f;
    dor[d] = ok ? dout[((int64_t)b * N + q) * D + hd * DH + d0 + d] : 0.f;
    acc[d] = 0.f;
  }
  const float L = ok ? lse[(int64_t)bh * N + q] : 0.f;
  const float dl = ok ? delta[(int64_t)bh * N + q] : 0.f;
  for (int k0 = 0; k0 < N; k0 += F32_CH) {
    __syncthreads();
    stage_chunk_f32(ks, base + D + hd * DH, ld, k0, N);
    stage_chunk_f32(vs, base + 2 * D + hd * DH, ld, k0, N);
    __syncthreads();
    const int kn = min(F32_CH, N - k0);
    for (int r = 0; r < kn; ++r) {
      const float s = quad_sum(dot16(qr, &ks[r][d0]));
      const float dp = quad_sum(dot16(dor, &vs[r][d0]));
      const float ds = expf(s - L) * (dp - dl);
#pragma unroll
      for (int d = 0; d < 16; ++d) acc[d] += ds * ks[r][d0 + d];
    }
  }
  if (!ok) return;
  float* row = dqkv + ((int64_t)b * N + q) * ld + hd * DH + d0;
#pragma unroll
  for (int t = 0; t < 4; ++t)
    *(f32x4*)(row + 4 * t) = f32x4{acc[4 * t] * scale, acc[4 * t + 1] * scale, acc[4 * t + 2] * scale,
                                   acc[4 * t + 3] * scale};
}

// dK, dV (row = key) -- dv = sum_q P dO, dk = scale * sum_q P (dP - delta) Q
__global__ __launch_bounds__(256) void attn_bwd_dkv_f32(const float* __restrict__ qkv,
                                                        const float* __restrict__ dout,
                                                        const float* __restrict__ lse,
                                                        const float* __restrict__ delta,
                                                        float* __restrict__ dqkv, int N, int H,
                                                        float scale) {
  __shared__ __attribute__((aligned(16))) float qs[F32_CH][DH];
  __shared__ __attribute__((aligned(16))) float ds_[F32_CH][DH];
  __shared__ float ls[F32_CH], dls[F32_CH];
  const int bh = blockIdx.y, b = bh / H, hd = bh % H;
  const int D = H * DH;
  const int64_t ld = 3 * (int64_t)D;
  const float* base = qkv + (int64_t)b * N * ld;
  const int key = blockIdx.x * 64 + (threadIdx.x >> 2), d0 = (threadIdx.x & 3) * 16;
  const bool ok = key < N;
  float kr[16], vr[16], dk[16], dv[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    kr[d] = ok ? base[(int64_t)key * ld + D + hd * DH + d0 + d] * scale : 0.f;
    vr[d] = ok ? base[(int64_t)key * ld + 2 * D + hd * DH + d0 + d] : 0.f;
    dk[d] = 0.f;
    dv[d] = 0.f;
  }
  for (int q0 = 0; q0 < N; q0 += F32_CH) {
    __syncthreads();
    stage_chunk_f32(qs, base + hd * DH, ld, q0, N);
    stage_chunk_f32(ds_, dout + (int64_t)b * N * D + hd * DH, D, q0, N);
    if (threadIdx.x < F32_CH) {
      const int q = q0 + threadIdx.x;
      ls[threadIdx.x] = q < N ? lse[(int64_t)bh * N + q] : 0.f;
      dls[threadIdx.x] = q < N ? delta[(int64_t)bh * N + q] : 0.f;
    }
    __syncthreads();
    const int qn = min(F32_CH, N - q0);
    for (int r = 0; r < qn; ++r) {
      float qv[16], dov[16];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const f32x4 a = *(const f32x4*)(&qs[r][d0 + 4 * t]), c = *(const f32x4*)(&ds_[r][d0 + 4 * t]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          qv[4 * t + e] = a[e];
          dov[4 * t + e] = c[e];
        }
      }
      float cs[4] = {0.f, 0.f, 0.f, 0.f}, cp[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int d = 0; d < 16; ++d) {
        cs[d & 3] = fmaf(kr[d], qv[d], cs[d & 3]);
        cp[d & 3] = fmaf(vr[d], dov[d], cp[d & 3]);
      }
      const float s = quad_sum((cs[0] + cs[1]) + (cs[2] + cs[3]));
      const float dp = quad_sum((cp[0] + cp[1]) + (cp[2] + cp[3]));
      const float p = expf(s - ls[r]);
      const float dsv = p * (dp - dls[r]);
#pragma unroll
      for (int d = 0; d < 16; ++d) {
        dv[d] = fmaf(p, dov[d], dv[d]);
        dk[d] = fmaf(dsv, qv[d], dk[d]);
      }
    }
  }
  if (!ok) return;
  float* row = dqkv + ((int64_t)b * N + key) * ld + hd * DH + d0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    *(f32x4*)(row + D + 4 * t) = f32x4{dk[4 * t] * scale, dk[4 * t + 1] * scale, dk[4 * t + 2] * scale,
                                       dk[4 * t + 3] * scale};
    *(f32x4*)(row + 2 * D + 4 * t) = f32x4{dv[4 * t], dv[4 * t + 1], dv[4 * t + 2], dv[4 * t + 3]};
  }
}

}  // namespace vitmi

using namespace vitmi;

// whole-sequence kernels for N <= SEQ_MAX (8 waves, 2 workgroups of <= 64 KiB LDS per CU).
// Kernel policy (vitmi_attention_set_policy; tests): 0 = auto, 1 = always the streamed kernels,
// 2 = the whole-sequence 32-query-per-wave forward / dQ (attn_fwd_seq_bf16 / attn_bwd_dq_seq_bf16)
// where auto takes their 64-query forms (bitwise equal by construction; the tests compare them),
// and the two-kernel backward; 3 = auto's forward with the two-kernel backward (64-query dQ, then
// dK/dV) where auto runs the single-pass attn_bwd_fused_seq_bf16 (N <= 224).
static constexpr int SEQ_MAX = 256;

static int device_cus() {   // compute units of the current device (the persistent dK/dV grid)
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      cus = n;
    else
      cus = 256;
  }
  return cus;
}
static int g_attn_policy = 0;
static bool seq_path(int N) { return N <= SEQ_MAX && g_attn_policy != 1; }
static bool q64() { return VITMI_ATTN_Q64 && g_attn_policy != 2; }
#ifndef VITMI_ATTN_FUSED_BWD
#define VITMI_ATTN_FUSED_BWD 1
#endif
static constexpr int FUSED_NKB = 7;   // the single-pass backward's LDS holds NKB^2 dS^T tiles: N <= 224
static bool fused_bwd(int N) { return VITMI_ATTN_FUSED_BWD && g_attn_policy == 0 && (N + 31) / 32 <= FUSED_NKB; }

template <int NKB>
static void launch_fused(int B, int N, int H, float scale, const void* qkv, const void* o, const void* dout,
                         const float* lse, float* delta, void* dqkv, float* colsum, hipStream_t s) {
  // persistent: one workgroup per CU (its LDS), each walking the (batch, head) pairs
  const int npairs = B * H, cus = device_cus();
  hipLaunchKernelGGL(attn_bwd_fused_seq_bf16<NKB>, dim3(npairs < cus ? npairs : cus), dim3(64 * NKB), 0, s,
                     (const bf16*)qkv, (const bf16*)o, (const bf16*)dout, lse, delta, (bf16*)dqkv, N, H, scale,
                     colsum, npairs);
  // algorithmic backward = dP, dQ, dV, dK: 8 N^2 dh flops per head (recomputing S is not counted);
  // bytes: q/k/v/o/dO read and dq/dk/dv written once, lse read and delta written
  const double bh = (double)B * H, t = bh * N * DH;
  VITMI_STAT(attn_bwd_fused_seq_bf16<NKB>, 8.0 * bh * N * N * DH, t * 8 * 2 + bh * N * 8);
}

extern "C" int vitmi_attention_set_policy(int policy) {
  VITMI_CHECK_ARG(policy >= 0 && policy <= 3, "attention_set_policy: policy must be 0..3");
  const int prev = g_attn_policy;
  g_attn_policy = policy;
  return prev;
}

static int attn_check(int dtype, int B, int N, int H, int dh) {
  VITMI_CHECK_ARG(dtype == VITMI_BF16 || dtype == VITMI_F32, "attention: bad dtype %d", dtype);
  VITMI_CHECK_ARG(dh == DH, "attention: head dim must be 64 (got %d)", dh);
  VITMI_CHECK_ARG(B > 0 && N > 0 && H > 0, "attention: empty problem");
  VITMI_CHECK_ARG((int64_t)N * 3 * H * DH * (dtype == VITMI_BF16 ? 2 : 4) < 0x7fffffffLL,
                  "attention: one batch row block exceeds 2 GiB");
  return VITMI_OK;
}

extern "C" int vitmi_attention_fwd(int dtype, int B, int N, int H, int dh, float scale,
                                   const void* qkv, void* o, float* lse, vitmi_stream_t stream) {
  if (int rc = attn_check(dtype, B, N, H, dh)) return rc;
  VITMI_CHECK_ARG(qkv && o && lse, "attention_fwd: null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == VITMI_BF16 && seq_path(N) && q64()) {
    hipLaunchKernelGGL(attn_fwd_seq64_bf16<SEQ_MAX>, dim3(B * H), dim3(256), 0, s, (const bf16*)qkv, (bf16*)o, lse,
                       N, H, scale);
  } else if (dtype == VITMI_BF16 && seq_path(N)) {
    const dim3 block(64 * ((N + 31) / 32));
    hipLaunchKernelGGL(attn_fwd_seq_bf16<SEQ_MAX>, dim3(B * H), block, 0, s, (const bf16*)qkv, (bf16*)o, lse, N,
                       H, scale);
  } else if (dtype == VITMI_BF16) {
    dim3 grid((N + 127) / 128, B * H);
    hipLaunchKernelGGL(attn_fwd_bf16, grid, dim3(256), 0, s, (const bf16*)qkv, (bf16*)o, lse, N, H, scale);
  } else if (seq_path(N)) {
    hipLaunchKernelGGL(attn_fwd_seq_f32<SEQ_MAX>, dim3(B * H), dim3(64 * ((N + 31) / 32)), 0, s, (const float*)qkv,
                       (float*)o, lse, N, H, scale);
  } else {
    dim3 grid((N + 63) / 64, B * H);
    hipLaunchKernelGGL(attn_fwd_f32, grid, dim3(256), 0, s, (const float*)qkv, (float*)o, lse, N, H, scale);
  }
  VITMI_LAUNCH_CHECK("attention_fwd");
  {
    // QK^T and PV: 4 N^2 dh flops per (batch, head); q/k/v read, o + lse written
    const double es = dtype == VITMI_BF16 ? 2 : 4, bh = (double)B * H;
    const double fl = 4.0 * bh * N * N * DH, by = bh * N * DH * 4 * es + bh * N * 4;
    if (dtype == VITMI_BF16 && seq_path(N) && q64()) VITMI_STAT(attn_fwd_seq64_bf16<SEQ_MAX>, fl, by);
    else if (dtype == VITMI_BF16 && seq_path(N)) VITMI_STAT(attn_fwd_seq_bf16<SEQ_MAX>, fl, by);
    else if (dtype == VITMI_BF16) VITMI_STAT(attn_fwd_bf16, fl, by);
    else if (seq_path(N)) VITMI_STAT(attn_fwd_seq_f32<SEQ_MAX>, fl, by);
    else VITMI_STAT(attn_fwd_f32, fl, by);
  }
  return VITMI_OK;
}

extern "C" int vitmi_attention_fwd_x3(int B, int N, int H, int dh, float scale, const void* qkv, void* o, void* o3,
                                      float* lse, vitmi_stream_t stream) {
  if (int rc = attn_check(VITMI_BF16, B, N, H, dh)) return rc;
  VITMI_CHECK_ARG(N <= SEQ_MAX, "attention_fwd_x3: N must be <= %d (the whole-sequence kernel)", SEQ_MAX);
  VITMI_CHECK_ARG(qkv && o && o3 && lse, "attention_fwd_x3: null pointer");
  VITMI_CHECK_ARG((int64_t)N * 3 * H * DH * 2 < 0x7fffffffLL, "attention_fwd_x3: one batch row block exceeds 2 GiB");
  const double bh = (double)B * H, fl = 4.0 * bh * N * N * DH, by = bh * N * DH * 2 * (3 + 1 + 3) + bh * N * 4;
  if (q64()) {
    hipLaunchKernelGGL((attn_fwd_seq64_bf16<SEQ_MAX, 1>), dim3(B * H), dim3(256), 0, (hipStream_t)stream,
                       (const bf16*)qkv, (bf16*)o, lse, N, H, scale, (bf16*)o3);
    VITMI_STAT((attn_fwd_seq64_bf16<SEQ_MAX, 1>), fl, by);
  } else {
    hipLaunchKernelGGL((attn_fwd_seq_bf16<SEQ_MAX, 1>), dim3(B * H), dim3(64 * ((N + 31) / 32)), 0,
                       (hipStream_t)stream, (const bf16*)qkv, (bf16*)o, lse, N, H, scale, (bf16*)o3);
    VITMI_STAT((attn_fwd_seq_bf16<SEQ_MAX, 1>), fl, by);
  }
  VITMI_LAUNCH_CHECK("attention_fwd_x3");
  return VITMI_OK;
}

extern "C" int vitmi_attention_fwd_f8(int B, int N, int H, int dh, float scale, const void* qkv, void* o, void* o8,
                                      float* lse, vitmi_stream_t stream) {
  if (int rc = attn_check(VITMI_BF16, B, N, H, dh)) return rc;
  VITMI_CHECK_ARG(N <= SEQ_MAX, "attention_fwd_f8: N must be <= %d (the whole-sequence kernel)", SEQ_MAX);
  VITMI_CHECK_ARG(qkv && o && o8 && lse, "attention_fwd_f8: null pointer");
  VITMI_CHECK_ARG((int64_t)N * 3 * H * DH * 2 < 0x7fffffffLL, "attention_fwd_f8: one batch row block exceeds 2 GiB");
  const double bh = (double)B * H, fl = 4.0 * bh * N * N * DH, by = bh * N * DH * 2 * (3 + 1 + 2) + bh * N * 4;
  if (q64()) {
    hipLaunchKernelGGL((attn_fwd_seq64_bf16<SEQ_MAX, 2>), dim3(B * H), dim3(256), 0, (hipStream_t)stream,
                       (const bf16*)qkv, (bf16*)o, lse, N, H, scale, (bf16*)o8);
    VITMI_STAT((attn_fwd_seq64_bf16<SEQ_MAX, 2>), fl, by);
  } else {
    hipLaunchKernelGGL((attn_fwd_seq_bf16<SEQ_MAX, 2>), dim3(B * H), dim3(64 * ((N + 31) / 32)), 0,
                       (hipStream_t)stream, (const bf16*)qkv, (bf16*)o, lse, N, H, scale, (bf16*)o8);
    VITMI_STAT((attn_fwd_seq_bf16<SEQ_MAX, 2>), fl, by);
  }
  VITMI_LAUNCH_CHECK("attention_fwd_f8");
  return VITMI_OK;
}

#ifdef VITMI_ATTN_STAMPS
extern "C" int vitmi_attn_set_stamps(void* buf) {
  VITMI_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(d_attn_stamps), &buf, sizeof(buf)), "attn stamps");
  return 0;
}
#endif

extern "C" size_t vitmi_attention_bwd_workspace_size(int B, int N, int H) {
  return (size_t)B * H * N * sizeof(float);
}

static int attention_bwd_impl(int dtype, int B, int N, int H, int dh, float scale, const void* qkv, const void* o,
                              const void* dout, const float* lse, void* dqkv, void* workspace, size_t ws_bytes,
                              vitmi_stream_t stream, float* colsum, int* colsum_rows) {
  if (colsum_rows) *colsum_rows = 0;
  if (int rc = attn_check(dtype, B, N, H, dh)) return rc;
  VITMI_CHECK_ARG(qkv && o && dout && lse && dqkv, "attention_bwd: null pointer");
  VITMI_CHECK_ARG(workspace && ws_bytes >= vitmi_attention_bwd_workspace_size(B, N, H),
                  "attention_bwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  float* delta = (float*)workspace;
  const int64_t rows = (int64_t)B * N * H;
  const int blocks = (int)((rows + 255) / 256);
  if (dtype == VITMI_BF16 && seq_path(N) && fused_bwd(N)) {
    switch ((N + 31) / 32) {
      case 1: launch_fused<1>(B, N, H, scale, qkv, o, dout, lse, delta, dqkv, colsum, s); break;
      case 2: launch_fused<2>(B, N, H, scale, qkv, o, dout, lse, delta, dqkv, colsum, s); break;
      case 3: launch_fused<3>(B, N, H, scale, qkv, o, dout, lse, delta, dqkv, colsum, s); break;
      case 4: launch_fused<4>(B, N, H, scale, qkv, o, dout, lse, delta, dqkv, colsum, s); break;
      case 5: launch_fused<5>(B, N, H, scale, qkv, o, dout, lse, delta, dqkv, colsum, s); break;
      case 6: launch_fused<6>(B, N, H, scale, qkv, o, dout, lse, delta, dqkv, colsum, s); break;
      default: launch_fused<7>(B, N, H, scale, qkv, o, dout, lse, delta, dqkv, colsum, s); break;
    }
    if (colsum_rows) *colsum_rows = colsum ? B : 0;   // one partial row per batch
  } else if (dtype == VITMI_BF16 && seq_path(N)) {
    // dQ first: it also writes delta, which the dK/dV kernel consumes
    const dim3 block(64 * ((N + 31) / 32));
    {
      const int npairs = B * H, cus = device_cus();
      const dim3 gkv(npairs < cus ? npairs : cus);
      const bool n7 = (N + 31) / 32 == 7;   // N in (192, 224]: the ViT-B/ViT-S shape, N = 197
      if (n7 && q64())
        hipLaunchKernelGGL((attn_bwd_dq_seq64_bf16<SEQ_MAX, 7>), dim3(B * H), dim3(256), 0, s, (const bf16*)qkv,
                           (const bf16*)o, (const bf16*)dout, lse, delta, (bf16*)dqkv, N, H, scale, colsum);
      else if (n7)
        hipLaunchKernelGGL((attn_bwd_dq_seq_bf16<SEQ_MAX, 7>), dim3(B * H), block, 0, s, (const bf16*)qkv,
                           (const bf16*)o, (const bf16*)dout, lse, delta, (bf16*)dqkv, N, H, scale, colsum);
      else
        hipLaunchKernelGGL((attn_bwd_dq_seq_bf16<SEQ_MAX>), dim3(B * H), block, 0, s, (const bf16*)qkv,
                           (const bf16*)o, (const bf16*)dout, lse, delta, (bf16*)dqkv, N, H, scale, colsum);
      if (n7)
        hipLaunchKernelGGL((attn_bwd_dkv_seq_bf16<SEQ_MAX, 7>), gkv, block, 0, s, (const bf16*)qkv, (const bf16*)dout,
                           lse, (const float*)delta, (bf16*)dqkv, N, H, scale, colsum, npairs);
      else
        hipLaunchKernelGGL((attn_bwd_dkv_seq_bf16<SEQ_MAX>), gkv, block, 0, s, (const bf16*)qkv, (const bf16*)dout,
                           lse, (const float*)delta, (bf16*)dqkv, N, H, scale, colsum, npairs);
      if (colsum_rows) *colsum_rows = colsum ? B : 0;   // one partial row per batch
    }
  } else if (dtype == VITMI_BF16) {
    // dQ first: it also writes delta, which the dK/dV kernel consumes
    dim3 grid((N + 127) / 128, B * H);
    hipLaunchKernelGGL(attn_bwd_dq_bf16, grid, dim3(256), 0, s, (const bf16*)qkv, (const bf16*)o,
                       (const bf16*)dout, lse, delta, (bf16*)dqkv, N, H, scale, colsum);
    hipLaunchKernelGGL(attn_bwd_dkv_bf16, grid, dim3(256), 0, s, (const bf16*)qkv, (const bf16*)dout,
                       lse, (const float*)delta, (bf16*)dqkv, N, H, scale, colsum);
    // one bias-gradient partial row per (batch, 128-row block)
    if (colsum_rows) *colsum_rows = colsum ? B * (int)grid.x : 0;
  } else if (seq_path(N)) {
    // dQ first: it also writes delta, which the dK/dV kernel consumes
    const dim3 block(64 * ((N + 31) / 32));
    hipLaunchKernelGGL(attn_bwd_dq_seq_f32<SEQ_MAX>, dim3(B * H), block, 0, s, (const float*)qkv, (const float*)o,
                       (const float*)dout, lse, delta, (float*)dqkv, N, H, scale);
    hipLaunchKernelGGL(attn_bwd_dkv_seq_f32<SEQ_MAX>, dim3(B * H), block, 0, s, (const float*)qkv,
                       (const float*)dout, lse, (const float*)delta, (float*)dqkv, N, H, scale);
  } else {
    hipLaunchKernelGGL(attn_bwd_delta<float>, dim3(blocks), dim3(256), 0, s, (const float*)o,
                       (const float*)dout, delta, B * N, N, H);
    dim3 grid((N + 63) / 64, B * H);
    hipLaunchKernelGGL(attn_bwd_dkv_f32, grid, dim3(256), 0, s, (const float*)qkv, (const float*)dout,
                       lse, (const float*)delta, (float*)dqkv, N, H, scale);
    hipLaunchKernelGGL(attn_bwd_dq_f32, grid, dim3(256), 0, s, (const float*)qkv, (const float*)dout,
                       lse, (const float*)delta, (float*)dqkv, N, H, scale);
  }
  VITMI_LAUNCH_CHECK("attention_bwd");
  {
    // algorithmic backward = dP, dQ (dQ kernel) + dV, dK (dK/dV kernel): 8 N^2 dh flops per head
    // (recomputing S is not counted); bytes: q/k/v/o/dO read, dq/dk/dv written, lse/delta
    const double es = dtype == VITMI_BF16 ? 2 : 4, bh = (double)B * H, t = bh * N * DH;
    const double fl = 4.0 * bh * N * N * DH;
    if (dtype == VITMI_BF16 && seq_path(N) && fused_bwd(N)) {
      // (launch_fused records its own)
    } else if (dtype == VITMI_BF16 && seq_path(N)) {
      if ((N + 31) / 32 == 7) {
        if (q64()) VITMI_STAT((attn_bwd_dq_seq64_bf16<SEQ_MAX, 7>), fl, t * 6 * es + bh * N * 8);
        else VITMI_STAT((attn_bwd_dq_seq_bf16<SEQ_MAX, 7>), fl, t * 6 * es + bh * N * 8);
        VITMI_STAT((attn_bwd_dkv_seq_bf16<SEQ_MAX, 7>), fl, t * 6 * es + bh * N * 8);
      } else {
        VITMI_STAT(attn_bwd_dq_seq_bf16<SEQ_MAX>, fl, t * 6 * es + bh * N * 8);
        VITMI_STAT(attn_bwd_dkv_seq_bf16<SEQ_MAX>, fl, t * 6 * es + bh * N * 8);
      }
    } else if (dtype == VITMI_BF16) {
      VITMI_STAT(attn_bwd_dq_bf16, fl, t * 6 * es + bh * N * 8);
      VITMI_STAT(attn_bwd_dkv_bf16, fl, t * 6 * es + bh * N * 8);
    } else if (seq_path(N)) {
      VITMI_STAT(attn_bwd_dq_seq_f32<SEQ_MAX>, fl, t * 6 * es + bh * N * 8);
      VITMI_STAT(attn_bwd_dkv_seq_f32<SEQ_MAX>, fl, t * 6 * es + bh * N * 8);
    }
  }
  return VITMI_OK;
}

extern "C" int vitmi_attention_bwd(int dtype, int B, int N, int H, int dh, float scale,
                                   const void* qkv, const void* o, const void* dout,
                                   const float* lse, void* dqkv, void* workspace, size_t ws_bytes,
                                   vitmi_stream_t stream) {
  return attention_bwd_impl(dtype, B, N, H, dh, scale, qkv, o, dout, lse, dqkv, workspace, ws_bytes, stream, nullptr,
                            nullptr);
}

extern "C" size_t vitmi_attention_bwd_bias_workspace_size(int B, int N, int H) {
  const size_t delta = ((size_t)B * H * N * sizeof(float) + 255) / 256 * 256;
  // fused partial rows: one per batch (whole-sequence kernels) or per (batch, 128-row block)
  const size_t part = (size_t)B * ((N + 127) / 128) * 3 * H * DH * sizeof(float);
  const size_t fallback = vitmi_bias_grad_workspace_size((int64_t)B * N, 3LL * H * DH);
  return delta + (part > fallback ? part : fallback);
}

extern "C" int vitmi_attention_bwd_bias(int dtype, int B, int N, int H, int dh, float scale, const void* qkv,
                                        const void* o, const void* dout, const float* lse, void* dqkv,
                                        float* dbias, void* workspace, size_t ws_bytes, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(dbias != nullptr, "attention_bwd_bias: dbias is null");
  VITMI_CHECK_ARG(workspace && ws_bytes >= vitmi_attention_bwd_bias_workspace_size(B, N, H),
                  "attention_bwd_bias: workspace too small");
  const size_t delta = ((size_t)B * H * N * sizeof(float) + 255) / 256 * 256;
  float* part = (float*)((char*)workspace + delta);
  int rows = 0;
  if (int rc = attention_bwd_impl(dtype, B, N, H, dh, scale, qkv, o, dout, lse, dqkv, workspace, delta,
                                  stream, part, &rows))
    return rc;
  const int64_t D3 = 3LL * H * DH;
  if (rows) return launch_colsum_finish(D3, rows, part, dbias, (hipStream_t)stream);
  return vitmi_bias_grad(dtype, (int64_t)B * N, D3, dqkv, D3, dbias, part, ws_bytes - delta, stream);
}
