/* Host-side AddressSanitizer driver of the C ABI (SURVEY §5 "race detection / sanitizers":
 * an -fsanitize=address host build of the C ABI).  Links the ASan build of libvitmi
 * (make -C transformer-stm_amd asan) and drives every host-only path: argument validation
 * that must reject before any launch, workspace-size queries, TF-'same' conv geometry, the
 * cv2 resize tables, the dropout hash, the comm entry points without a communicator and the
 * work-accounting table.  No GPU: nothing here may launch a kernel.  Exit 0 = all checks
 * passed and ASan saw no memory error (it aborts the process on the first one). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../../include/vitmi.h"

static int fails = 0;
#define EXPECT(c)                                                        \
  do {                                                                   \
    if (!(c)) {                                                          \
      fprintf(stderr, "FAIL %s:%d: %s (%s)\n", __FILE__, __LINE__, #c,   \
              vitmi_last_error());                                       \
      ++fails;                                                           \
    }                                                                    \
  } while (0)

int main(void) {
  EXPECT(vitmi_version() >= 300);
  EXPECT(strlen(vitmi_build_id()) >= 17 && vitmi_build_id()[16] == '-');
  EXPECT(strlen(vitmi_build_flags()) > 0);
  /* SURVEY §8(b) composites: workspace queries, and validation before any launch */
  EXPECT(vitmi_patch_embed_fwd_workspace_size(VITMI_BF16, 256, 3, 224, 16, 768) >= (size_t)256 * 196 * 768 * 4);
  EXPECT(vitmi_patch_embed_bwd_workspace_size(VITMI_BF16, 256, 3, 224, 16, 768) > 0);
  EXPECT(vitmi_patch_embed_fwd_workspace_size(VITMI_BF16, 2, 3, 30, 8, 64) == 0);
  EXPECT(vitmi_patch_embed_fwd(VITMI_BF16, 2, 3, 32, 8, 64, (float*)16, (void*)16, NULL, NULL, NULL, (void*)16,
                               (float*)16, (void*)16, 8, NULL) == VITMI_ERR_INVALID);
  EXPECT(vitmi_patch_embed_bwd(VITMI_BF16, 2, 3, 32, 8, 64, NULL, (void*)16, NULL, NULL, NULL, NULL, (void*)16,
                               1 << 30, NULL) == VITMI_ERR_INVALID);
  EXPECT(vitmi_linear_bwd_workspace_size(VITMI_BF16, 50432, 768, 3072) > 0);
  EXPECT(vitmi_linear_bwd(VITMI_BF16, 64, 64, 64, (void*)16, (void*)16, (void*)16, (void*)16, VITMI_BF16, NULL,
                          NULL, (void*)16, 8, NULL) == VITMI_ERR_INVALID);
  EXPECT(vitmi_xent_fwd(2, 2, (float*)16, (int64_t*)16, NULL, NULL) == VITMI_ERR_INVALID);
  EXPECT(vitmi_xent_bwd(2, 2, (float*)16, (int64_t*)16, NULL, NULL) == VITMI_ERR_INVALID);
  EXPECT(vitmi_mse_fwd(2, 1, (float*)16, (float*)16, NULL, NULL) == VITMI_ERR_INVALID);
  EXPECT(vitmi_mse_bwd(0, 1, (float*)16, (float*)16, (float*)16, NULL) == VITMI_ERR_INVALID);
  EXPECT(vitmi_trace_push("off") == VITMI_OK && vitmi_trace_pop() == VITMI_OK);   /* disabled: no-ops */
  /* GEMM validation: k-major with K % 64 != 0, null operands, bad dtype, tiny lda */
  EXPECT(vitmi_gemm(VITMI_BF16, 1, 1, 128, 128, 100, (void*)16, 128, (void*)16, 128, (void*)16, 128,
                    VITMI_BF16, VITMI_EPI_STORE, NULL, NULL, 0, NULL, 0, NULL, 0, NULL) == VITMI_ERR_INVALID);
  EXPECT(vitmi_gemm(VITMI_BF16, 1, 1, 128, 128, 128, NULL, 128, (void*)16, 128, (void*)16, 128,
                    VITMI_BF16, VITMI_EPI_STORE, NULL, NULL, 0, NULL, 0, NULL, 0, NULL) == VITMI_ERR_INVALID);
  EXPECT(vitmi_gemm(7, 1, 1, 128, 128, 128, (void*)16, 128, (void*)16, 128, (void*)16, 128,
                    VITMI_BF16, VITMI_EPI_STORE, NULL, NULL, 0, NULL, 0, NULL, 0, NULL) == VITMI_ERR_INVALID);
  EXPECT(vitmi_gemm(VITMI_BF16, 1, 1, 128, 128, 128, (void*)16, 64, (void*)16, 128, (void*)16, 128,
                    VITMI_BF16, VITMI_EPI_STORE, NULL, NULL, 0, NULL, 0, NULL, 0, NULL) == VITMI_ERR_INVALID);
  EXPECT(vitmi_linear_fwd(VITMI_BF16, 64, 64, 64, (void*)16, (void*)16, NULL, (void*)16, VITMI_BF16, 9, NULL,
                          NULL, NULL, 0, NULL) == VITMI_ERR_INVALID);
  /* the tile-native gelu' layout is bf16-only */
  EXPECT(vitmi_linear_fwd(VITMI_F32, 64, 64, 64, (void*)16, (void*)16, NULL, (void*)16, VITMI_F32,
                          VITMI_EPI_BIAS_GELU | VITMI_EPI_AUX_TILED, (void*)16, NULL, NULL, 0, NULL) == VITMI_ERR_INVALID);
  EXPECT(vitmi_gemm(VITMI_BF16, 1, 1, 0, 128, 128, NULL, 128, NULL, 128, NULL, 128, VITMI_BF16,
                    VITMI_EPI_STORE, NULL, NULL, 0, NULL, 0, NULL, 0, NULL) == VITMI_OK);   /* empty */
  /* workspace queries at every ViT shape */
  const int64_t Ms[] = {1, 197, 50432, 64 * 577};
  for (int i = 0; i < 4; ++i) {
    (void)vitmi_linear_fwd_workspace_size(VITMI_BF16, Ms[i], 3072, 768);
    EXPECT(vitmi_aux_tiled_bytes(Ms[i], 3072) == (size_t)((Ms[i] + 255) / 256) * 12 * 131072);
    (void)vitmi_linear_dgrad_workspace_size(VITMI_BF16, Ms[i], 3072, 768);
    (void)vitmi_linear_dgrad_bias_workspace_size(VITMI_BF16, Ms[i], 3072, 768);
    EXPECT(vitmi_linear_wgrad_workspace_size(VITMI_BF16, Ms[i], 768, 768) < ((size_t)1 << 34));
    EXPECT(vitmi_bias_grad_workspace_size(Ms[i], 768) > 0);
    (void)vitmi_gemm_workspace_size(VITMI_F32, 0, 0, 768, 768, Ms[i], VITMI_EPI_ACCUM);
  }
  EXPECT(vitmi_attention_bwd_workspace_size(2, 197, 12) == (size_t)2 * 197 * 12 * 4);
  EXPECT(vitmi_attention_bwd_bias_workspace_size(2, 577, 16) > 0);
  EXPECT(vitmi_layernorm_bwd_workspace_size(50432, 768) > 0);
  EXPECT(vitmi_dwconv_bn_workspace_size(128, 32, 32, 64) > 0);
  /* attention / layernorm / loss / cast validation */
  EXPECT(vitmi_attention_fwd(VITMI_BF16, 1, 10, 2, 32, 1.f, (void*)16, (void*)16, (float*)16, NULL) ==
         VITMI_ERR_INVALID);
  EXPECT(vitmi_attention_fwd(VITMI_BF16, 0, 10, 2, 64, 1.f, (void*)16, (void*)16, (float*)16, NULL) ==
         VITMI_ERR_INVALID);
  EXPECT(vitmi_layernorm_fwd(4, 30, (float*)16, 30, (float*)16, (float*)16, 1e-6f, (void*)16, 0, 30, (float*)16,
                             (float*)16, NULL) == VITMI_ERR_INVALID);
  EXPECT(vitmi_cast_f32_bf16(8, (float*)17, (void*)16, NULL) == VITMI_ERR_INVALID);
  EXPECT(vitmi_cast_bf16_f32(8, NULL, (float*)16, NULL) == VITMI_ERR_INVALID);
  /* host tables: TF 'same' conv geometry, cv2 INTER_LINEAR resize tables */
  int ho, wo, pt, pl;
  EXPECT(vitmi_conv_same_geometry(128, 128, 7, 7, 4, &ho, &wo, &pt, &pl) == VITMI_OK && ho == 32 && wo == 32);
  EXPECT(vitmi_conv_same_geometry(32, 32, 3, 3, 2, &ho, &wo, &pt, &pl) == VITMI_OK && ho == 16 && pt == 0);
  const int sizes[][2] = {{345, 128}, {340, 128}, {128, 128}, {64, 224}, {1, 8}};
  for (int i = 0; i < 5; ++i) {
    const int d = sizes[i][1];
    int* ofs = (int*)malloc(sizeof(int) * d);
    short* w = (short*)malloc(sizeof(short) * 2 * d);
    EXPECT(vitmi_sls_resize_table(sizes[i][0], d, ofs, w) == VITMI_OK);
    for (int j = 0; j < d; ++j) EXPECT(ofs[j] >= 0 && ofs[j] < sizes[i][0] && w[2 * j] + w[2 * j + 1] == 2048);
    free(ofs);
    free(w);
  }
  /* dropout hash: a pure function of its coordinates */
  EXPECT(vitmi_dropout_hash(1, 2, 3, 4) == vitmi_dropout_hash(1, 2, 3, 4));
  EXPECT(vitmi_dropout_hash(1, 2, 3, 4) != vitmi_dropout_hash(1, 2, 3, 5));
  /* comm without a communicator */
  EXPECT(vitmi_comm_destroy(0) == VITMI_OK);
  EXPECT(vitmi_comm_check() == VITMI_OK);
  EXPECT(vitmi_comm_allreduce_async((void*)16, 4, VITMI_F32, VITMI_REDUCE_AVG, NULL, NULL) == VITMI_ERR_INVALID);
  EXPECT(vitmi_comm_init(3, 2, "xx") == VITMI_ERR_INVALID);
  EXPECT(vitmi_comm_get_unique_id(NULL) == VITMI_ERR_INVALID);
  int r = -5, w = -5;
  EXPECT(vitmi_comm_info(&r, &w) == VITMI_ERR_INVALID && r == -1 && w == 0);
  /* work-accounting table: enable/clear, out-of-range reads rejected */
  EXPECT(vitmi_stats_enable(1) == VITMI_OK && vitmi_stats_count() == 0);
  char name[8];
  EXPECT(vitmi_stats_get(0, name, (int)sizeof(name), NULL, NULL, NULL) == VITMI_ERR_INVALID);
  EXPECT(vitmi_stats_enable(0) == VITMI_OK);
  /* policy knobs */
  EXPECT(vitmi_gemm_set_policy(9) == VITMI_ERR_INVALID);
  EXPECT(vitmi_attention_set_policy(5) == VITMI_ERR_INVALID);
  EXPECT(vitmi_gemm_set_reserved_cus(1 << 20) == 0 && vitmi_gemm_set_reserved_cus(0) > 0);
  /* the error message buffer survives a very long formatted message */
  char big[4096];
  memset(big, 'a', sizeof(big) - 1);
  big[sizeof(big) - 1] = 0;
  (void)vitmi_last_error();
  if (fails == 0) printf("asan driver: all checks passed\n");
  return fails ? 1 : 0;
}
