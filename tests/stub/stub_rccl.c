/* A stand-in librccl.so for the CPU tests of the comm leg's abort path (tests/test_dp_cpu.py):
 * the NCCL 2.x entry points csrc/comm.cpp binds, with ncclAllReduce / ncclBroadcast blocking
 * the way an enqueue does when a peer is gone, until ncclCommAbort releases them (then they
 * return ncclRemoteError).  A safety limit ends a block after STUB_MAX_BLOCK_S seconds so a
 * broken library cannot hang the test runner.  Loaded through VITMI_RCCL_LIB; test only. */
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct { char internal[128]; } ncclUniqueId;
typedef struct stub_comm { atomic_int aborted; int rank, world; } *ncclComm_t;
typedef int ncclResult_t;
enum { STUB_MAX_BLOCK_S = 20 };

static atomic_int g_calls_in;   /* calls that entered a blocking entry point */

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) { memset(id->internal, 7, 128); return 0; }

ncclResult_t ncclCommInitRank(ncclComm_t* c, int world, ncclUniqueId id, int rank) {
  (void)id;
  *c = (ncclComm_t)calloc(1, sizeof(**c));
  (*c)->rank = rank;
  (*c)->world = world;
  return 0;
}

static ncclResult_t block_until_abort(ncclComm_t c) {
  atomic_fetch_add(&g_calls_in, 1);
  struct timespec t0, t;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (;;) {
    if (atomic_load(&c->aborted)) return 6; /* ncclRemoteError */
    clock_gettime(CLOCK_MONOTONIC, &t);
    if (t.tv_sec - t0.tv_sec > STUB_MAX_BLOCK_S) return 3; /* ncclInternalError */
    struct timespec d = {0, 1000000};
    nanosleep(&d, NULL);
  }
}

ncclResult_t ncclAllReduce(const void* s, void* r, size_t n, int t, int op, ncclComm_t c, void* stream) {
  (void)s; (void)r; (void)n; (void)t; (void)op; (void)stream;
  return block_until_abort(c);
}

ncclResult_t ncclBroadcast(const void* s, void* r, size_t n, int t, int root, ncclComm_t c, void* stream) {
  (void)s; (void)r; (void)n; (void)t; (void)root; (void)stream;
  return block_until_abort(c);
}

/* The comm object is leaked on purpose: a call released by the abort may still read its flag. */
ncclResult_t ncclCommAbort(ncclComm_t c) { atomic_store(&c->aborted, 1); return 0; }
ncclResult_t ncclCommDestroy(ncclComm_t c) { atomic_store(&c->aborted, 1); return 0; }
const char* ncclGetErrorString(ncclResult_t r) { return r == 6 ? "remote error (stub: aborted)" : "stub error"; }
ncclResult_t ncclCommGetAsyncError(ncclComm_t c, ncclResult_t* a) { *a = atomic_load(&c->aborted) ? 6 : 0; return 0; }
int stub_calls_in(void) { return atomic_load(&g_calls_in); }
