// boundary.cpp — the per-op entry points SURVEY.md §8(b) names for the drop-in boundary
// (vitmi_{patch_embed,linear,xent,mse}_{fwd,bwd} + their workspace queries), composed on the
// host from the kernel-level entry points of the other files.  Each replaces one library op of
// the reference at its call site (include/vitmi.h cites them); the composites launch exactly
// the kernels the Python modules launch one by one, so results are bit-identical to that path.
#include <hip/hip_runtime.h>
#include "common.h"

using namespace vitmi;

namespace {

constexpr size_t kAlign = 256;
size_t align_up(size_t n) { return (n + kAlign - 1) / kAlign * kAlign; }

struct PatchGeom {
  int64_t np, rows, K;
};

int patch_geom(int B, int C, int S, int P, int D, PatchGeom& g) {
  VITMI_CHECK_ARG(B > 0 && C > 0 && D > 0 && P > 0 && S % P == 0, "patch_embed: bad shape");
  VITMI_CHECK_ARG(D % 4 == 0, "patch_embed: D %% 4 != 0");
  g.np = (int64_t)(S / P) * (S / P);
  g.rows = (int64_t)B * g.np;
  g.K = (int64_t)C * P * P;
  return VITMI_OK;
}

int es_of(int dtype) { return dtype == VITMI_BF16 ? 2 : 4; }

}  // namespace

// ---- patch embedding: Conv2D(D, k=P, s=P) + cls + pos (models/CvT(Par).py:203-212,244-245)
extern "C" size_t vitmi_patch_embed_fwd_workspace_size(int dtype, int B, int C, int S, int P, int D) {
  PatchGeom g;
  if (patch_geom(B, C, S, P, D, g)) return 0;
  return align_up((size_t)g.rows * D * sizeof(float)) + vitmi_linear_fwd_workspace_size(dtype, g.rows, D, g.K);
}

extern "C" int vitmi_patch_embed_fwd(int dtype, int B, int C, int S, int P, int D, const float* img, const void* w,
                                     const float* bias, const float* cls, const float* pos, void* patches, float* x,
                                     void* workspace, size_t ws_bytes, vitmi_stream_t stream) {
  PatchGeom g;
  if (int rc = patch_geom(B, C, S, P, D, g)) return rc;
  VITMI_CHECK_ARG(img && w && patches && x, "patch_embed_fwd: null pointer");
  const size_t need = vitmi_patch_embed_fwd_workspace_size(dtype, B, C, S, P, D);
  VITMI_CHECK_ARG(workspace && ws_bytes >= need, "patch_embed_fwd: workspace %zu < %zu bytes", ws_bytes, need);
  float* conv = (float*)workspace;
  char* lin_ws = (char*)workspace + align_up((size_t)g.rows * D * sizeof(float));
  if (int rc = vitmi_patch_im2col(dtype, B, C, S, P, img, patches, stream)) return rc;
  if (int rc = vitmi_linear_fwd(dtype, g.rows, D, g.K, patches, w, bias, conv, VITMI_F32, VITMI_EPI_STORE, nullptr,
                                nullptr, lin_ws, ws_bytes - (lin_ws - (char*)workspace), stream))
    return rc;
  return vitmi_tokens_assemble(B, (int)g.np, D, conv, cls, pos, x, stream);
}

extern "C" size_t vitmi_patch_embed_bwd_workspace_size(int dtype, int B, int C, int S, int P, int D) {
  PatchGeom g;
  if (patch_geom(B, C, S, P, D, g)) return 0;
  const size_t wg = vitmi_linear_wgrad_workspace_size(dtype, g.rows, D, g.K);
  const size_t bg = vitmi_bias_grad_workspace_size(g.rows, D);
  return align_up((size_t)g.rows * D * es_of(dtype)) + (wg > bg ? wg : bg);
}

extern "C" int vitmi_patch_embed_bwd(int dtype, int B, int C, int S, int P, int D, const float* dx,
                                     const void* patches, float* dw, float* dbias, float* dcls, float* dpos,
                                     void* workspace, size_t ws_bytes, vitmi_stream_t stream) {
  PatchGeom g;
  if (int rc = patch_geom(B, C, S, P, D, g)) return rc;
  VITMI_CHECK_ARG(dx && patches, "patch_embed_bwd: null pointer");
  const size_t need = vitmi_patch_embed_bwd_workspace_size(dtype, B, C, S, P, D);
  VITMI_CHECK_ARG(workspace && ws_bytes >= need, "patch_embed_bwd: workspace %zu < %zu bytes", ws_bytes, need);
  void* dtok = workspace;
  char* rest = (char*)workspace + align_up((size_t)g.rows * D * es_of(dtype));
  const size_t rest_bytes = ws_bytes - (rest - (char*)workspace);
  const bool lp = dtype == VITMI_BF16;
  if (int rc = vitmi_tokens_assemble_bwd(B, (int)g.np, D, dx, lp ? nullptr : (float*)dtok, lp ? dtok : nullptr, dcls,
                                         dpos, stream))
    return rc;
  if (dw)
    if (int rc = vitmi_linear_wgrad(dtype, g.rows, D, g.K, dtok, patches, dw, rest, rest_bytes, stream)) return rc;
  if (dbias)
    if (int rc = vitmi_bias_grad(dtype, g.rows, D, dtok, D, dbias, rest, rest_bytes, stream)) return rc;
  return VITMI_OK;
}

// ---- Dense backward: dx = dy W, dW += dy^T x, db += colsum(dy)  (autodiff of layers.Dense)
extern "C" size_t vitmi_linear_bwd_workspace_size(int dtype, int64_t M, int64_t N, int64_t K) {
  size_t a = vitmi_linear_dgrad_workspace_size(dtype, M, N, K);
  const size_t b = vitmi_linear_wgrad_workspace_size(dtype, M, N, K);
  const size_t c = vitmi_bias_grad_workspace_size(M, N);
  if (b > a) a = b;
  return c > a ? c : a;
}

extern "C" int vitmi_linear_bwd(int dtype, int64_t M, int64_t N, int64_t K, const void* dy, const void* x,
                                const void* w, void* dx, int dx_dtype, float* dw, float* db, void* workspace,
                                size_t ws_bytes, vitmi_stream_t stream) {
  VITMI_CHECK_ARG(dy != nullptr, "linear_bwd: null dy");
  const size_t need = vitmi_linear_bwd_workspace_size(dtype, M, N, K);
  VITMI_CHECK_ARG(workspace && ws_bytes >= need, "linear_bwd: workspace %zu < %zu bytes", ws_bytes, need);
  // the three launches share the workspace: they are ordered on one stream
  if (dx) {
    VITMI_CHECK_ARG(w != nullptr, "linear_bwd: dx needs w");
    if (int rc = vitmi_linear_dgrad(dtype, M, N, K, dy, w, dx, dx_dtype, VITMI_EPI_STORE, nullptr, workspace,
                                    ws_bytes, stream))
      return rc;
  }
  if (dw) {
    VITMI_CHECK_ARG(x != nullptr, "linear_bwd: dw needs x");
    if (int rc = vitmi_linear_wgrad(dtype, M, N, K, dy, x, dw, workspace, ws_bytes, stream)) return rc;
  }
  if (db)
    if (int rc = vitmi_bias_grad(dtype, M, N, dy, N, db, workspace, ws_bytes, stream)) return rc;
  return VITMI_OK;
}

// ---- losses: softmax cross-entropy (BASELINE configs) and Keras 'mean_squared_error'
// (models/CvT(Par).py:464-466), mean over the batch.  _bwd writes d(mean loss)/d logits.
extern "C" int vitmi_xent_fwd(int B, int C, const float* logits, const int64_t* target, float* loss,
                              vitmi_stream_t stream) {
  VITMI_CHECK_ARG(loss != nullptr, "xent_fwd: null loss");
  return vitmi_loss_fwd_bwd(VITMI_LOSS_CE, B, C, logits, target, loss, nullptr, stream);
}
extern "C" int vitmi_xent_bwd(int B, int C, const float* logits, const int64_t* target, float* dlogits,
                              vitmi_stream_t stream) {
  VITMI_CHECK_ARG(dlogits != nullptr, "xent_bwd: null dlogits");
  return vitmi_loss_fwd_bwd(VITMI_LOSS_CE, B, C, logits, target, nullptr, dlogits, stream);
}
extern "C" int vitmi_mse_fwd(int B, int C, const float* pred, const float* target, float* loss,
                             vitmi_stream_t stream) {
  VITMI_CHECK_ARG(loss != nullptr, "mse_fwd: null loss");
  return vitmi_loss_fwd_bwd(VITMI_LOSS_MSE, B, C, pred, target, loss, nullptr, stream);
}
extern "C" int vitmi_mse_bwd(int B, int C, const float* pred, const float* target, float* dpred,
                             vitmi_stream_t stream) {
  VITMI_CHECK_ARG(dpred != nullptr, "mse_bwd: null dpred");
  return vitmi_loss_fwd_bwd(VITMI_LOSS_MSE, B, C, pred, target, nullptr, dpred, stream);
}
