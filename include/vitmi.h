/*
 * vitmi.h — C ABI of libvitmi.so, the MI355X (gfx950 / CDNA4) ViT training path.
 *
 * Drop-in boundary.  The reference's hot path is the forward + autodiff backward
 * of its transformer stage, dispatched by Keras to TensorFlow GPU library ops
 * (SURVEY.md §2 op table).  Each entry point below replaces one such library op
 * at its call site in the reference; the Python layer (vitmi/ops.py, vitmi/modules.py)
 * mirrors the reference's layer API and calls these through ctypes.
 *
 * Conventions
 *   - All pointers are DEVICE pointers owned by the caller (the PyTorch caching
 *     allocator).  No entry point allocates, frees or synchronises the host.
 *   - Every call is stream-ordered on `stream` (a hipStream_t) and re-entrant.
 *   - Matrices are row-major with an explicit leading dimension in ELEMENTS.
 *   - Accumulating outputs (parameter gradients) are fp32 and updated with +=,
 *     the semantics of torch's .grad accumulation.
 *   - Return 0 on success, otherwise a VITMI_ERR_* code; vitmi_last_error()
 *     returns a thread-local message.  Shapes are validated on the host before
 *     any launch; there is no silent fallback path.
 */
#ifndef VITMI_H
#define VITMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* vitmi_stream_t; /* hipStream_t */

enum { VITMI_OK = 0, VITMI_ERR_INVALID = 1, VITMI_ERR_HIP = 2, VITMI_ERR_UNSUPPORTED = 3, VITMI_ERR_COMM = 4 };
enum {
  VITMI_F32 = 0,
  VITMI_BF16 = 1,
  VITMI_F64 = 2,    /* comm only */
  VITMI_BF16X3 = 3, /* vitmi_layernorm_fwd's y only: bf16 rows [hi | hi | lo] of 3D columns, the
                       split-bf16 A operand of the precision knob (vitmi_split_bf16x3) */
  VITMI_BF16F8 = 4, /* the knob's cheaper form (ViTConfig dtype "bf16f8"): a row of K values is 4K
                       bytes (2K bf16 units), [hi = bf16(x) (K bf16) | OCP e4m3 part (2K bytes)],
                       the e4m3 part in 64-k blocks of 128 B, [hi8 | lo8] for an A operand
                       (activations) and [lo8 | hi8] for a weight, hi8 = e4m3(hi), lo8 =
                       e4m3((x - hi) * 2^9) (vitmi_split_bf16f8; K % 64 == 0).
                       vitmi_linear_fwd dtype (x and w both so; K % 64 == 0, N % 16 == 0): the
                       GEMM runs K/64 bf16 K-steps (hi.hi) and K/64 block-scaled fp8 K-steps
                       (hi.lo + lo.hi, v_mfma_scale_f32_16x16x128_f8f6f4): 2K-equivalent MFMA
                       work instead of bf16x3's 3K.  Also vitmi_layernorm_fwd's y dtype. */
  VITMI_BF16F8W = 5 /* the weight-side correction alone (the bf16f8 knob's qkv GEMM): a row of K values
                       is 3K bytes (1.5K bf16 units), [hi = bf16(x) (K bf16) | one OCP e4m3 byte per
                       k (K bytes)], the byte hi8 = e4m3(hi) for an A operand (activations) and lo8 =
                       e4m3((x - hi) * 2^9) for a weight (vitmi_split_bf16f8 patterns 2 / 3; K % 128
                       == 0).  vitmi_linear_fwd dtype (x and w both so): K/64 bf16 K-steps (hi.hi) and
                       K/128 block-scaled fp8 K-steps (hi.lo_w only): 1.5K-equivalent work.  The qkv
                       GEMM's error is its weight rounding's (q and k of every token move together);
                       the activation side's averages out (tools/precision_sides.py).  Also
                       vitmi_layernorm_fwd's y dtype (A-operand rows). */
};

/* GEMM epilogues (all apply `bias` (fp32, may be NULL) first where it applies) */
enum {
  VITMI_EPI_STORE = 0,     /* C = acc + bias                                        */
  VITMI_EPI_BIAS_GELU = 1, /* u = acc + bias: C = gelu(u), aux = gelu'(u) (saved)     */
  VITMI_EPI_RESIDUAL = 2,  /* C(f32) = residual(f32) + acc + bias                    */
  VITMI_EPI_DGELU = 3,     /* C = acc * aux   (aux = gelu'(u) from BIAS_GELU)        */
  VITMI_EPI_ACCUM = 4      /* C(f32) += acc                                          */
};
/* OR'ed into BIAS_GELU / DGELU (bf16 operands only): aux is kept in the library's tile-native
 * layout instead of a row-major [M][N] array -- vitmi_aux_tiled_bytes(M, N) bytes, written by a
 * BIAS_GELU call and read by a DGELU call of the same M x N output, opaque to the caller.  The
 * GEMM epilogues then store and load it straight from the accumulator registers (no LDS
 * transpose): the fc1 forward / fc2 dgrad pair of the ViT MLP (models/CvT(Par).py:253-258). */
#define VITMI_EPI_AUX_TILED 0x100
size_t vitmi_aux_tiled_bytes(int64_t rows, int64_t cols);
/* OR'ed into BIAS_GELU of vitmi_linear_fwd (bf16 operands and output; the precision knob,
 * ViTConfig dtype "bf16x3"): y is bf16 [M][3N], each row [hi | hi | lo] of the fp32 gelu(u)
 * (hi = bf16(a), lo = bf16(a - hi): the split A operand of the next GEMM, vitmi_split_bf16x3
 * pattern 0); aux = gelu'(u) as for BIAS_GELU. */
#define VITMI_EPI_SPLIT_X3 0x200
/* OR'ed into BIAS_GELU of vitmi_linear_fwd with dtype VITMI_BF16F8 (y_dtype VITMI_BF16; N % 64 == 0):
 * y is [M][2N] bf16 units, each row the VITMI_BF16F8 A-operand layout of gelu(u); aux as for BIAS_GELU. */
#define VITMI_EPI_SPLIT_F8 0x400

enum { VITMI_LOSS_CE = 0, VITMI_LOSS_MSE = 1 };

int vitmi_version(void);
/* "<sources>-<flags>": 16 hex digits of the content hash of the sources the library was built
 * from (csrc/ + this header), then 8 of the hash of its compiler command line
 * (vitmi_build_flags); __graft_entry__ compares the first part with the tree it runs in, so a
 * stale .so is caught, and a variant built with other flags or -D switches has another id */
const char* vitmi_build_id(void);
const char* vitmi_build_flags(void);
const char* vitmi_last_error(void);
/* number of hipDevice compute units seen by the library (0 on error) */
int vitmi_device_cus(void);
/* Per-kernel algorithmic work accounting (host side, off by default): while enabled every
 * launch adds its 2 x MAC flops and minimum HBM bytes to its kernel's entry (keyed by the
 * mangled device symbol).  Enabling clears the table.  bench.py joins these with a rocprofv3
 * kernel trace of the same run (per-kernel TFLOP/s, GB/s). */
int vitmi_stats_enable(int on);
int vitmi_stats_count(void);
int vitmi_stats_get(int i, char* name, int name_len, int64_t* calls, double* flops, double* bytes);
/* ROCTx ranges (rocprofv3 --marker-trace): off by default; enabling binds the ROCm marker
 * library at run time (VITMI_ERR_UNSUPPORTED if absent).  vitmi/trace.py wraps the training
 * step's forward / backward / all-reduce / optimizer phases in them. */
int vitmi_trace_enable(int on);
int vitmi_trace_push(const char* name);
int vitmi_trace_pop(void);

/* ---------------------------------------------------------------------------
 * Generic MFMA GEMM:  C[M,N] (op)= sum_k A(m,k) * B(k,n)
 *   a_kmajor=1: A stored [M][lda] (k contiguous);  0: A stored [K][lda] (m contiguous)
 *   b_kmajor=1: B stored [N][ldb] (k contiguous);  0: B stored [K][ldb] (n contiguous)
 *   dtype: operand type (VITMI_BF16 -> v_mfma_f32_16x16x32_bf16, VITMI_F32 -> v_mfma_f32_16x16x4_f32)
 *   c_dtype: output type; aux (the saved GELU derivative gelu'(u)) has the operand dtype.
 *   BIAS_GELU on bf16 operands writes bf16 (c_dtype VITMI_F32 is rejected).
 *   k-major operands need K % 64 == 0 (bf16) / K % 32 == 0 (f32); ragged M/N and a
 *   ragged reduction over m-major operands are zero-filled by the buffer range check.
 * Replaces the reference's Dense/EinsumDense MatMul and their autodiff transposes
 * (models/CvT(Par).py:132-134,137,142,188,254,256).
 */
int vitmi_gemm(int dtype, int a_kmajor, int b_kmajor, int64_t M, int64_t N, int64_t K,
               const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc,
               int c_dtype, int epilogue, const float* bias, void* aux, int64_t ldaux,
               const float* residual, int64_t ldr, void* workspace, size_t ws_bytes,
               vitmi_stream_t stream);
/* Kernel selection (process-wide): 0 = auto (default), 1 = always the 128x128 tile kernel,
 * 2 = always the 256x256 8-wave bf16 kernel where the dtype allows, 3 = as 2 on an 8-block
 * persistent grid (each block walks many tiles).  For tests/diagnostics. */
int vitmi_gemm_set_policy(int policy);
size_t vitmi_gemm_workspace_size(int dtype, int a_kmajor, int b_kmajor, int64_t M, int64_t N,
                                 int64_t K, int epilogue);

/* Linear layer y = x W^T + b  (keras layers.Dense, models/CvT(Par).py:132-134,142,254,256;
 * torch nn.Linear in old_codes/MS_CvT.py:63-65,116-121).  x [M,K], W [N,K] -> y [M,N]. */
/* workspace: optional (NULL/0 allowed).  With vitmi_linear_*_workspace_size() bytes the
 * persistent bf16 GEMM splits the tiles of an under-filled last round over K (fp32 partials
 * in the workspace, finished by a fix-up kernel): same results up to fp32 summation order. */
int vitmi_linear_fwd(int dtype, int64_t M, int64_t N, int64_t K, const void* x, const void* w,
                     const float* bias, void* y, int y_dtype, int epilogue, void* aux,
                     const float* residual, void* workspace, size_t ws_bytes,
                     vitmi_stream_t stream);
size_t vitmi_linear_fwd_workspace_size(int dtype, int64_t M, int64_t N, int64_t K);
/* dx[M,K] = dy[M,N] W[N,K]   (epilogue STORE or DGELU with aux = gelu'(u) [M,K]) */
int vitmi_linear_dgrad(int dtype, int64_t M, int64_t N, int64_t K, const void* dy, const void* w,
                       void* dx, int dx_dtype, int epilogue, const void* aux, void* workspace,
                       size_t ws_bytes, vitmi_stream_t stream);
size_t vitmi_linear_dgrad_workspace_size(int dtype, int64_t M, int64_t N, int64_t K);
/* dW[N,K] (f32) += dy[M,N]^T x[M,K]; uses split-K over M with fp32 partial slabs */
int vitmi_linear_wgrad(int dtype, int64_t M, int64_t N, int64_t K, const void* dy, const void* x,
                       float* dw, void* workspace, size_t ws_bytes, vitmi_stream_t stream);
/* Linear dgrad with the bias gradient of its OUTPUT fused: dx = dy W (optionally * aux, DGELU)
 * and db[k] += sum_m dx[m][k] (fp32).  The bias of the layer whose INPUT gradient dx is: for
 * the MLP, du = (g W2) * gelu'(u) is fc1's output gradient, so db = fc1's bias gradient
 * (models/CvT(Par).py:254; Keras Dense bias).  On the gemm256 DGELU path the column sums come
 * from the epilogue registers (one fp32 partial row per 128 output rows, folded in a fixed
 * order), elsewhere from a second pass over dx.  workspace >= vitmi_linear_dgrad_bias_workspace_size. */
size_t vitmi_linear_dgrad_bias_workspace_size(int dtype, int64_t M, int64_t N, int64_t K);
int vitmi_linear_dgrad_bias(int dtype, int64_t M, int64_t N, int64_t K, const void* dy, const void* w, void* dx,
                            int dx_dtype, int epilogue, const void* aux, float* db, void* workspace, size_t ws_bytes,
                            vitmi_stream_t stream);

size_t vitmi_linear_wgrad_workspace_size(int dtype, int64_t M, int64_t N, int64_t K);
/* Grouped weight gradients over ONE row count M: for p < n (n <= 4), dW_p[N[p], K[p]] (f32) +=
 * dy_p[M, N[p]]^T x_p[M, K[p]], dy_p rows of pitch lddy[p] and x_p of pitch ldx[p] elements (NULL
 * or 0: dense).  The four weight gradients of a transformer block (models/CvT(Par).py:253-258,
 * 132-142: fc2, fc1, out-projection, qkv) in one split-K launch over all their tiles and one
 * reduction launch (bf16; other dtypes and shapes run one vitmi_linear_wgrad-equivalent GEMM per
 * problem).  workspace >= vitmi_linear_wgrad_group_workspace_size(dtype, n, M, N, K). */
int vitmi_linear_wgrad_group(int dtype, int n, int64_t M, const int64_t* N, const int64_t* K,
                             const void* const* dy, const int64_t* lddy, const void* const* x,
                             const int64_t* ldx, float* const* dw, void* workspace, size_t ws_bytes,
                             vitmi_stream_t stream);
size_t vitmi_linear_wgrad_group_workspace_size(int dtype, int n, int64_t M, const int64_t* N,
                                               const int64_t* K);
/* db[N] (f32) += sum_m dy[m, n]  (dy [M][ldy] of `dtype`) */
int vitmi_bias_grad(int dtype, int64_t M, int64_t N, const void* dy, int64_t ldy, float* db,
                    void* workspace, size_t ws_bytes, vitmi_stream_t stream);
size_t vitmi_bias_grad_workspace_size(int64_t M, int64_t N);

/* ---------------------------------------------------------------------------
 * LayerNorm over the last dim D (layers.LayerNormalization, models/CvT(Par).py:248,328;
 * old_codes/MS_CvT.py:39-45).  x is fp32 [M][ldx]; y [M][ldy] of y_dtype; mean/rstd fp32 [M].
 * y_dtype VITMI_BF16X3: y is bf16 [M][ldy >= 3D], each row [hi | hi | lo] of the fp32 result.
 * y_dtype VITMI_BF16F8: y is [M][ldy >= 2D] bf16 units, each row the VITMI_BF16F8 A-operand layout.
 */
int vitmi_layernorm_fwd(int64_t M, int D, const float* x, int64_t ldx, const float* gamma,
                        const float* beta, float eps, void* y, int y_dtype, int64_t ldy,
                        float* mean, float* rstd, vitmi_stream_t stream);
/* dx = dres + LN'(dy); optional low-precision copy dx_lp (bf16); dgamma/dbeta += (fp32);
 * optional dxsum[D] += column sums of dx (the bias gradient of the Dense layer whose output
 * gradient dx is: fused so that gradient is never re-read). NULL pointers skip outputs. */
int vitmi_layernorm_bwd(int64_t M, int D, const void* dy, int dy_dtype, int64_t lddy,
                        const float* x, int64_t ldx, const float* mean, const float* rstd,
                        const float* gamma, const float* dres, int64_t ldres, float* dx,
                        int64_t lddx, void* dx_lp, int64_t lddx_lp, float* dgamma, float* dbeta,
                        float* dxsum, void* workspace, size_t ws_bytes, vitmi_stream_t stream);
size_t vitmi_layernorm_bwd_workspace_size(int64_t M, int D);
/* ---------------------------------------------------------------------------
 * Multi-head scaled-dot-product attention (layers.MultiHeadAttention called (q, v, k),
 * models/CvT(Par).py:137,185; einsum-softmax-einsum old_codes/MS_CvT.py:202-207).
 * qkv: [B*N][3*H*dh] token-major (q | k | v column blocks, head h at h*dh); o: [B*N][H*dh];
 * lse: fp32 [B*H][N] (natural-log softmax normaliser per query, saved for backward).
 * dh must be 64.  dtype selects bf16 MFMA (VITMI_BF16) or fp32 (VITMI_F32) kernels.
 */
int vitmi_attention_fwd(int dtype, int B, int N, int H, int dh, float scale, const void* qkv,
                        void* o, float* lse, vitmi_stream_t stream);
/* The precision knob's attention forward (bf16 q, k, v; ViTConfig dtype "bf16x3"): as
 * vitmi_attention_fwd(VITMI_BF16, ...) -- o (bf16 [B*N][H*dh]) and lse bit for bit -- plus o3,
 * bf16 [B*N][3*H*dh], each row [hi | hi | lo] of the fp32 output (the out-projection GEMM's
 * split A operand, vitmi_split_bf16x3 pattern 0).  N <= 256 (the whole-sequence kernel). */
int vitmi_attention_fwd_x3(int B, int N, int H, int dh, float scale, const void* qkv, void* o, void* o3,
                           float* lse, vitmi_stream_t stream);
/* As vitmi_attention_fwd_x3 for the VITMI_BF16F8 knob: o8 is [B*N][2*H*dh] bf16 units, each row the
 * VITMI_BF16F8 A-operand layout [hi | hi8 | lo8] of the fp32 output. */
int vitmi_attention_fwd_f8(int B, int N, int H, int dh, float scale, const void* qkv, void* o, void* o8,
                           float* lse, vitmi_stream_t stream);
int vitmi_attention_bwd(int dtype, int B, int N, int H, int dh, float scale, const void* qkv,
                        const void* o, const void* dout, const float* lse, void* dqkv,
                        void* workspace, size_t ws_bytes, vitmi_stream_t stream);
size_t vitmi_attention_bwd_workspace_size(int B, int N, int H);
/* Kernel selection (process-wide; tests): 0 = auto (bf16, N <= 224: the single-pass backward, dQ,
 * dK and dV in one persistent kernel), 1 = always the streamed (64-key LDS-tiled) kernels, 2 = the
 * whole-sequence kernels' 32-query-per-wave forward and dQ forms and the two-kernel backward (auto
 * runs their 64-query forms, bitwise equal), 3 = auto's forward with the two-kernel backward
 * (64-query dQ, then dK/dV).  Returns the previous policy. */
int vitmi_attention_set_policy(int policy);
/* vitmi_attention_bwd plus the qkv bias gradient: dbias[3*H*dh] += column sums of dqkv (the
 * q/k/v Dense biases, models/CvT(Par).py:132-134).  On the bf16 paths the sums come from the
 * backward kernels' output images (per (batch, head) block on the whole-sequence path,
 * N <= 256, per (batch, head, 128-row block) on the streamed one, then a fixed-order fold); the
 * fp32 paths take a second pass over dqkv. */
size_t vitmi_attention_bwd_bias_workspace_size(int B, int N, int H);
int vitmi_attention_bwd_bias(int dtype, int B, int N, int H, int dh, float scale, const void* qkv, const void* o,
                             const void* dout, const float* lse, void* dqkv, float* dbias, void* workspace,
                             size_t ws_bytes, vitmi_stream_t stream);

/* ---------------------------------------------------------------------------
 * Patch embedding Conv2D(k=P, s=P) as a GEMM (models/CvT(Par).py:203-212;
 * old_codes/MS_CvT.py:352-361): im2col of the fp32 NCHW images into
 * patches [B*(S/P)^2][C*P*P] of `dtype` (column order c, kh, kw = the conv weight's).
 * Limits: S % P == 0, P % 4 == 0, C*P*P <= 4096 (one thread per 4 columns of a patch row).
 */
int vitmi_patch_im2col(int dtype, int B, int C, int S, int P, const float* img, void* patches,
                       vitmi_stream_t stream);
/* x[b][0] = cls + pos[0];  x[b][1+p] = tok[b*np+p] + pos[1+p]   (cls/pos may be NULL) */
int vitmi_tokens_assemble(int B, int np, int D, const float* tok, const float* cls,
                          const float* pos, float* x, vitmi_stream_t stream);
/* backward of assemble: dtok (f32, and optional bf16 copy) = dx[:,1:];  dpos += sum_b dx,
 * dcls += sum_b dx[:,0]   (NULL pointers skip that output) */
int vitmi_tokens_assemble_bwd(int B, int np, int D, const float* dx, float* dtok, void* dtok_lp,
                              float* dcls, float* dpos, vitmi_stream_t stream);

/* ---------------------------------------------------------------------------
 * Per-op entry points under the names of SURVEY.md §8(b) (csrc/boundary.cpp).  Each composes
 * the kernel-level entry points above on the same stream (bit-identical results) and takes a
 * caller-owned workspace of at least the queried size.
 *
 * vitmi_patch_embed_fwd replaces ConvEmbed.call's Conv2D (models/CvT(Par).py:211-217) plus the
 * block's cls concat (:264-268) and the position embedding:
 *   patches (out, saved for the backward) = im2col(img) [B*np][C*P*P] of dtype, np = (S/P)^2;
 *   x (out, fp32 [B][np+1][D]) = [cls ; patches W^T + bias] + pos   (cls/pos/bias may be NULL);
 *   w: [D][C*P*P] of dtype (the conv weight flattened).
 * vitmi_patch_embed_bwd: dW += ..., dbias += ..., dcls += ..., dpos += ... from dx (NULL skips). */
size_t vitmi_patch_embed_fwd_workspace_size(int dtype, int B, int C, int S, int P, int D);
int vitmi_patch_embed_fwd(int dtype, int B, int C, int S, int P, int D, const float* img, const void* w,
                          const float* bias, const float* cls, const float* pos, void* patches, float* x,
                          void* workspace, size_t ws_bytes, vitmi_stream_t stream);
size_t vitmi_patch_embed_bwd_workspace_size(int dtype, int B, int C, int S, int P, int D);
int vitmi_patch_embed_bwd(int dtype, int B, int C, int S, int P, int D, const float* dx, const void* patches,
                          float* dw, float* dbias, float* dcls, float* dpos, void* workspace, size_t ws_bytes,
                          vitmi_stream_t stream);
/* Autodiff of layers.Dense (models/CvT(Par).py:132-134,142,188,254,256): dx = dy W (dx_dtype,
 * NULL skips), dW += dy^T x, db += column sums of dy (fp32, NULL skips).  dy/x/w of dtype. */
size_t vitmi_linear_bwd_workspace_size(int dtype, int64_t M, int64_t N, int64_t K);
int vitmi_linear_bwd(int dtype, int64_t M, int64_t N, int64_t K, const void* dy, const void* x, const void* w,
                     void* dx, int dx_dtype, float* dw, float* db, void* workspace, size_t ws_bytes,
                     vitmi_stream_t stream);
/* Losses, mean over the batch: softmax cross-entropy (BASELINE configs, target int64 [B]) and
 * Keras 'mean_squared_error' (models/CvT(Par).py:464-466, target fp32 [B][C]).  _fwd writes
 * the scalar loss, _bwd d(loss)/d(logits) [B][C] (upstream gradient 1). */
int vitmi_xent_fwd(int B, int C, const float* logits, const int64_t* target, float* loss, vitmi_stream_t stream);
int vitmi_xent_bwd(int B, int C, const float* logits, const int64_t* target, float* dlogits, vitmi_stream_t stream);
int vitmi_mse_fwd(int B, int C, const float* pred, const float* target, float* loss, vitmi_stream_t stream);
int vitmi_mse_bwd(int B, int C, const float* pred, const float* target, float* dpred, vitmi_stream_t stream);

/* ---------------------------------------------------------------------------
 * Head (layers.Dense(num_classes) on LN(cls), models/CvT(Par).py:326-329,350) and loss
 * (compile(loss='mean_squared_error') :464-466; softmax-CE for >=2 classes).
 * y: fp32 [B][ldy]; W fp32 [C][D].
 */
int vitmi_head_fwd(int B, int D, int C, const float* y, int64_t ldy, const float* w,
                   const float* b, float* logits, vitmi_stream_t stream);
int vitmi_head_bwd(int B, int D, int C, const float* dlogits, const float* y, int64_t ldy,
                   const float* w, float* dy, float* dw, float* db, vitmi_stream_t stream);
/* loss = mean over batch; dlogits = d loss / d logits.  target: int64 [B] (CE) or f32 [B][C] (MSE).
 * Either output may be NULL (not both). */
int vitmi_loss_fwd_bwd(int kind, int B, int C, const float* logits, const void* target,
                       float* loss, float* dlogits, vitmi_stream_t stream);

/* ---------------------------------------------------------------------------
 * Dropout (layers.Dropout, models/CvT(Par).py:189 after the out-projection, :255 after the
 * GELU, :257 after fc2; Keras rate 0.1, active in training only).  Element (row, col) of
 * dropout site `site` is kept iff vitmi_dropout_hash(seed, site, row, col) >= thresh, with
 * thresh = round(p * 2^32), and kept values are scaled by `scale` = 1/(1-p).  The mask is a
 * pure function of its coordinates: it is regenerated in the backward, never stored.
 */
uint32_t vitmi_dropout_hash(uint32_t seed, uint32_t site, uint32_t row, uint32_t col);
/* vitmi_linear_fwd with the dropout fused into the epilogue:
 *   BIAS_GELU: y = gelu(u) * keep * scale, aux = gelu'(u) * keep * scale (so the DGELU
 *              backward of the dropped activation needs no mask);
 *   RESIDUAL:  y = residual + (acc + bias) * keep * scale.   (x, W k-major as in linear_fwd) */
int vitmi_linear_fwd_dropout(int dtype, int64_t M, int64_t N, int64_t K, const void* x,
                             const void* w, const float* bias, void* y, int y_dtype, int epilogue,
                             void* aux, const float* residual, void* workspace, size_t ws_bytes,
                             uint32_t seed, uint32_t site, uint32_t thresh, float scale,
                             vitmi_stream_t stream);
/* y[M][ldy] (f32 or bf16) = x[M][ldx] (f32) * keep * scale   (N % 4 == 0): the masked
 * gradient of a dropped branch in the backward */
int vitmi_dropout_apply(int64_t M, int64_t N, const float* x, int64_t ldx, void* y, int y_dtype,
                        int64_t ldy, uint32_t seed, uint32_t site, uint32_t thresh, float scale,
                        vitmi_stream_t stream);

/* ---------------------------------------------------------------------------
 * CvT stages (the reference's actual SLS model, models/CvT(Par).py:66-72).
 *
 * ConvEmbed = layers.Conv2D(D, kernel=k, strides=s, padding='same') (:203-212) as a GEMM over
 * patches.  TF 'same': Ho = ceil(H/s), pad_total = max((Ho-1)s + k - H, 0), pad_before =
 * pad_total/2 (vitmi_conv_same_geometry).  Input rows are NHWC tokens: image b, pixel (h, w)
 * is row b*img_stride + row_off + h*W + w of x [..][ldx] (fp32).  Patch rows [B*Ho*Wo][Kp]
 * (dtype) in column order (kh, kw, c) -- the Keras kernel [kh][kw][Cin][Cout] flattened --
 * zero-padded to Kp (a multiple of the GEMM's K step).
 */
int vitmi_conv_same_geometry(int H, int W, int kh, int kw, int s, int* Ho, int* Wo, int* pad_top, int* pad_left);
/* explicit geometry (pad_top/pad_left/Ho/Wo): TF 'same' from vitmi_conv_same_geometry, or the
 * symmetric padding of torch Conv2d (old_codes/MS_CvT.py PATCH_PADDING) */
int vitmi_conv_im2col(int dtype, int B, int H, int W, int C, int kh, int kw, int s, int pad_top, int pad_left,
                      int Ho, int Wo, const float* x, int64_t ldx, int64_t img_stride, int64_t row_off,
                      void* patches, int Kp, vitmi_stream_t stream);
/* adjoint of im2col: dx (f32, rows as x) (+)= the sum over every window reading a pixel (C % 4 == 0) */
int vitmi_conv_col2im(int dtype, int B, int H, int W, int C, int kh, int kw, int s, int pad_top, int pad_left,
                      int Ho, int Wo, const void* dpatches, int Kp, float* dx, int64_t ldx, int64_t img_stride,
                      int64_t row_off, int accumulate, vitmi_stream_t stream);
/* Projection(method='dw_bn') (:83-112): z = DepthwiseConv2D(3, 'same', no bias)(x) [3][3][C],
 * y = BatchNormalization: training != 0 -> batch statistics over n = B*H*W (biased variance) and the
 * moving statistics m <- momentum m + (1-momentum) stat (NULL to skip; the moving variance takes
 * the unbiased n/(n-1) estimate, as Keras' fused BN and torch's BatchNorm2d do); training == 0 -> the
 * moving statistics normalise (Keras inference).  x/dx rows as above (cls row skipped via
 * x_off), y rows b*y_img + y_off + hw of y [..][ldy] (y_dtype).  z [B*H*W][C], mean/rstd [C]
 * are saved for the backward.  C % 4 == 0 and 1024 % C == 0. */
size_t vitmi_dwconv_bn_workspace_size(int B, int H, int W, int C);
int vitmi_dwconv_bn_fwd(int B, int H, int W, int C, const float* x, int64_t ldx, int64_t x_img, int64_t x_off,
                        const float* w, const float* gamma, const float* beta, float eps, float momentum,
                        int training, float* run_mean, float* run_var, float* z, float* mean, float* rstd, void* y,
                        int y_dtype,
                        int64_t ldy, int64_t y_img, int64_t y_off, void* workspace, size_t ws_bytes,
                        vitmi_stream_t stream);
/* dx += d/dx, dw/dgamma/dbeta += (f32) from dy (rows as y, dy_dtype) */
int vitmi_dwconv_bn_bwd(int B, int H, int W, int C, const void* dy, int dy_dtype, int64_t lddy, int64_t dy_img,
                        int64_t dy_off, const float* x, int64_t ldx, int64_t x_img, int64_t x_off, const float* w,
                        const float* gamma, const float* z, const float* mean, const float* rstd, float* dx,
                        float* dw, float* dgamma, float* dbeta, void* workspace, size_t ws_bytes,
                        vitmi_stream_t stream);

/* Projection(method='avg') (models/CvT(Par).py:95-96,107-108): AveragePooling2D(pool 3,
 * stride 1, padding 'same') over [B, H, W, C] token rows laid out like vitmi_dwconv_bn_fwd's
 * (image b pixel p at row b*x_img + x_off + p), the mean over the in-bounds taps (TF 'same'
 * pooling excludes the padding from the divisor; count_pad=1: always 9, torch's AvgPool2d as in
 * old_codes/MS_CvT.py:145-153).  y (bf16 | f32) rows likewise.  The
 * backward ACCUMULATES dx += pool^T(dy).  C % 4 == 0, 1024 % C == 0. */
int vitmi_avgpool3_fwd(int B, int H, int W, int C, const float* x, int64_t ldx, int64_t x_img, int64_t x_off,
                       void* y, int y_dtype, int64_t ldy, int64_t y_img, int64_t y_off, int count_pad,
                       vitmi_stream_t stream);
int vitmi_avgpool3_bwd(int B, int H, int W, int C, const void* dy, int dy_dtype, int64_t lddy, int64_t dy_img,
                       int64_t dy_off, float* dx, int64_t ldx, int64_t x_img, int64_t x_off, int count_pad,
                       vitmi_stream_t stream);

/* Small fp32 Dense layers: Proc_Dense_1/2 = layers.Dense(256, activation='relu') on the
 * standardised process parameters (models/CvT(Par).py:343-344).  y = act(x W^T + b),
 * act 0 = linear, 1 = relu; x [M][ldx], W [N][K] fp32, y [M][ldy].  The backward takes the
 * forward's output y (the relu mask), writes dx = (dy * act'(y)) W when dx != NULL and
 * ACCUMULATES dW += (dy * act'(y))^T x, db += column sums (db may be NULL).  Exact fp32 FMA
 * in a fixed order (deterministic). */
int vitmi_dense_f32_fwd(int M, int N, int K, const float* x, int64_t ldx, const float* w, const float* b, float* y,
                        int64_t ldy, int act, vitmi_stream_t stream);
int vitmi_dense_f32_bwd(int M, int N, int K, const float* dy, int64_t lddy, const float* y, int64_t ldy,
                        const float* x, int64_t ldx, const float* w, float* dx, int64_t lddx, float* dw, float* db,
                        int act, vitmi_stream_t stream);

/* Keras Adam step (models/CvT(Par).py:458-460: keras.optimizers.Adam(1e-3); beta_1 0.9,
 * beta_2 0.999, epsilon 1e-7) over n fp32 parameters in place:
 *   g' = g * grad_scale;  m += (g' - m)(1 - b1);  v += (g'^2 - v)(1 - b2);
 *   p -= alpha m / (sqrt(v) + eps),   alpha = lr sqrt(1 - b2^t) / (1 - b1^t) (caller, step t >= 1).
 * p_lp (optional, bf16) receives the updated parameters' operand shadow in the same pass.
 * (1 - beta) is formed in double and rounded once (Keras' Python-float hyper-parameters).
 * Explicitly rounded fp32 ops in this order: bit-identical to a float32 evaluation.  Buffers
 * 16-byte aligned (a ParamArena's flat buffers; one launch for the whole model). */
int vitmi_adam_step(int64_t n, float* p, const float* g, float* m, float* v, void* p_lp, float alpha, double beta_1,
                    double beta_2, float epsilon, float grad_scale, vitmi_stream_t stream);

/* SLS data pipeline (models/CvT(Par).py:414-428).
 * vitmi_sls_resize_table (host): cv2 INTER_LINEAR table of one axis, ssize -> dsize:
 *   ofs[d] first source index, w[2d], w[2d+1] its Q11 weights (OpenCV 8-bit fixed point).
 * vitmi_sls_preprocess: n decoded uint8 frames (interleaved 3 channels, RGB, or BGR if bgr=1;
 *   frame i row y at src + i*img_bytes + y*row_bytes) -> cv2.resize to Wo x Ho ->
 *   BGR2GRAY -> /255.0 -> fp32 out[n][Ho*Wo].  Tables are device copies of the two axis
 *   tables (xofs/xw for W -> Wo, yofs/yw for H -> Ho).
 * vitmi_gather_rows: dst[i] = src[idx[i]] for n rows of row_bytes (batch assembly from the
 *   HBM-resident dataset; idx device int64; an index outside [0, n_src) gives a zero row). */
int vitmi_sls_resize_table(int ssize, int dsize, int* ofs, short* w);
int vitmi_sls_preprocess(int n, int H, int W, const void* src, int64_t img_bytes, int64_t row_bytes, int bgr, int Ho,
                         int Wo, const int* xofs, const short* xw, const int* yofs, const short* yw, float* out,
                         vitmi_stream_t stream);
int vitmi_gather_rows(int64_t n, int64_t row_bytes, const void* src, int64_t n_src, const int64_t* idx, void* dst,
                      vitmi_stream_t stream);

/* Split-bf16 operands of the precision knob (ViTConfig dtype "bf16x3"; csrc/split.hip).  The reference
 * computes in fp32 (models/CvT(Par).py, Keras floatx); an operand carried as x = hi + lo, hi = bf16(x),
 * lo = bf16(x - hi), makes a bf16 MFMA product good to ~2^-16: hi.hi + hi.lo + lo.hi, computed by the
 * GEMMs above unchanged as ONE product over K' = 3K with the A rows laid out [hi | hi | lo] (pattern 0)
 * and the weight rows [hi | lo | hi] (pattern 1).
 *   vitmi_split_bf16x3: src fp32 [rows][ld_src] (K % 4 == 0) -> dst bf16 [rows][ld_dst >= 3K];
 *     hi_copy (optional, bf16 [rows][ld_copy]) receives hi alone (the bf16 operand of the backward).
 * The activation operands come split straight from their producers: vitmi_layernorm_fwd (y dtype
 * VITMI_BF16X3), vitmi_attention_fwd_x3 and the fc1 epilogue (VITMI_EPI_SPLIT_X3). */
int vitmi_split_bf16x3(int64_t rows, int64_t K, const float* src, int64_t ld_src, void* dst, int64_t ld_dst,
                       int pattern, void* hi_copy, int64_t ld_copy, vitmi_stream_t stream);
/* VITMI_BF16F8 rows: src fp32 [rows][ld_src] (K % 64 == 0) -> dst [rows][ld_dst >= 2K bf16 units],
 * pattern 0 the A-operand layout (e4m3 blocks [hi8 | lo8]), pattern 1 the weight layout ([lo8 | hi8]);
 * patterns 2 / 3: the VITMI_BF16F8W rows (ld_dst >= 1.5K bf16 units, K % 128 == 0), [hi | hi8] (A
 * operand) / [hi | lo8] (weight); hi_copy as above. */
int vitmi_split_bf16f8(int64_t rows, int64_t K, const float* src, int64_t ld_src, void* dst, int64_t ld_dst,
                       int pattern, void* hi_copy, int64_t ld_copy, vitmi_stream_t stream);
/* Up to 8 dense weights (srcs[j] fp32 [rows[j]][K[j]]) to pattern-1 VITMI_BF16F8 rows (dsts[j]
 * [rows[j]][2 K[j]] bf16 units) in one launch (the knob's per-forward weight split). */
int vitmi_split_bf16f8_weights(int n, const float* const* srcs, void* const* dsts, const int64_t* rows,
                               const int64_t* K, vitmi_stream_t stream);
/* The same with a layout per weight: patterns[j] 1 (VITMI_BF16F8 rows, [rows][2K]) or 3
 * (VITMI_BF16F8W rows [hi | lo8], [rows][1.5K], K % 128 == 0: the qkv weight of the bf16f8 knob). */
int vitmi_split_bf16f8_weights_mixed(int n, const float* const* srcs, void* const* dsts, const int64_t* rows,
                                     const int64_t* K, const int* patterns, vitmi_stream_t stream);

/* fp32 -> bf16 cast of n elements (weight shadows for the bf16 MFMA path) */
int vitmi_cast_f32_bf16(int64_t n, const float* src, void* dst, vitmi_stream_t stream);
/* bf16 -> fp32 cast of n elements (the bf16 gradient all-reduce writes back into the fp32 arena) */
int vitmi_cast_bf16_f32(int64_t n, const void* src, float* dst, vitmi_stream_t stream);

/* ---------------------------------------------------------------------------
 * Data-parallel gradient exchange over RCCL (xGMI within a node).  Replaces the cross-replica
 * gradient reduction of tf.distribute.MirroredStrategy (old_codes/BayConvT(Par)(Muti).py:16-19,
 * the reference's only parallel construct; TF runs it as an NCCL all-reduce on one host).
 * One process per GPU, one communicator per process (bound to the HIP device current at
 * vitmi_comm_init).  Rank 0 creates the 128-byte id; the caller distributes it (vitmi/dp.py
 * uses torch.distributed's TCPStore).  RCCL is bound at run time (the copy already loaded by
 * the process, else librccl.so); errors return VITMI_ERR_COMM.
 */
#define VITMI_COMM_UID_BYTES 128
enum { VITMI_REDUCE_SUM = 0, VITMI_REDUCE_AVG = 1 };
int vitmi_comm_get_unique_id(char* uid /* [VITMI_COMM_UID_BYTES] */);
int vitmi_comm_init(int rank, int world, const char* uid /* [VITMI_COMM_UID_BYTES] */);
int vitmi_comm_info(int* rank, int* world);
/* file name of the RCCL library the comm leg bound (dladdr of its ncclAllReduce): the copy
 * torch already mapped, so the process holds one RCCL instance */
int vitmi_comm_library(char* path, int len);
/* In-place all-reduce of `count` elements (VITMI_F32 | VITMI_BF16 | VITMI_F64) on the side stream `side`,
 * after `ready_event` (a hipEvent_t recorded on the compute stream, may be NULL).  Returns once
 * enqueued; the caller orders its consumers after `side` (record an event / stream wait). */
int vitmi_comm_allreduce_async(void* ptr, int64_t count, int dtype, int op, vitmi_stream_t side, void* ready_event);
/* in-place broadcast from `root` (parameter replication at start-up) */
int vitmi_comm_broadcast(void* ptr, int64_t count, int dtype, int root, vitmi_stream_t stream);
/* VITMI_ERR_COMM if the communicator reported an asynchronous error */
int vitmi_comm_check(void);
/* abort != 0: ncclCommAbort (tear down after a peer failure without waiting) */
int vitmi_comm_destroy(int abort);

/* Deferred partial-sum folds.  The parameter-gradient outputs of vitmi_layernorm_bwd (dgamma, dbeta,
 * dxsum), of the fused column sums of vitmi_linear_dgrad_bias / vitmi_attention_bwd_bias and of
 * vitmi_bias_grad are formed in two steps: per-block partial rows in the caller's workspace, then a
 * small fold launch (out += the column sums of the partial rows, fixed order).  Between
 * vitmi_fold_begin() and vitmi_fold_end() on one host thread, those folds are queued instead of
 * launched, and vitmi_fold_end launches them together (one launch per 16 folds, on the stream of the
 * calls that queued them) and orders `stream` after every other stream that ran folds since
 * vitmi_fold_begin (an event wait).  The caller keeps the workspaces of the queued calls alive until
 * then; the outputs are final in `stream` order after vitmi_fold_end.  vitmi/modules.py brackets
 * each block's backward with them: one fold launch per block instead of four. */
int vitmi_fold_begin(void);
int vitmi_fold_end(vitmi_stream_t stream);

/* Compute units the persistent GEMM leaves free (default 0): with data-parallel gradient
 * all-reduces in flight, RCCL's kernels need CUs while a one-block-per-CU GEMM would hold all
 * of them for its whole duration.  Returns the previous value. */
int vitmi_gemm_set_reserved_cus(int n);

#ifdef __cplusplus
}
#endif
#endif /* VITMI_H */
