/* A stand-in librccl.so for the tests of the library's RCCL leg (csrc/comm.cpp), loaded through
 * VITMI_RCCL_LIB; test only.  It exports the NCCL 2.x entry points comm.cpp binds and runs in one of
 * two modes (environment STUB_RCCL_MODE):
 *
 *   block (default)  the abort path (tests/test_dp_cpu.py): an all-reduce / broadcast never
 *                    completes, as when a peer is gone, until ncclCommAbort.  A blocking
 *                    communicator (ncclCommInitRank, or the config refused: STUB_RCCL_NO_CONFIG=1)
 *                    blocks inside the call; a non-blocking one (ncclCommInitRankConfig with
 *                    blocking = 0) returns ncclInProgress and ncclCommGetAsyncError reports
 *                    ncclInProgress until the abort.  ncclCommAbort frees (and poisons) a
 *                    non-blocking communicator, so a call that touched it after the abort would
 *                    read freed memory; a blocking one is leaked, since its blocked call still
 *                    reads the abort flag.
 *   shm              a FUNCTIONAL all-reduce / broadcast between the processes of one host
 *                    (tests/test_gpu_dp.py: two ranks on the one GPU of the test box, where real
 *                    RCCL refuses two ranks per device).  Stream-ordered by synchronising the
 *                    passed HIP stream, then each rank copies its buffer device -> a POSIX shared
 *                    memory slot, all ranks meet at a barrier, each sums the slots in rank order
 *                    (so every rank gets the same bits), scales for ncclAvg, and copies the result
 *                    back host -> device.  HIP is taken from the process (dlsym), not linked.
 *                    With STUB_RCCL_HOST=1 the buffers are host memory (no HIP at all): the CPU
 *                    tests run the library's world-2 path across two processes that way.
 *
 * A safety limit ends any wait after STUB_MAX_BLOCK_S seconds so a broken library cannot hang the
 * test runner. */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

typedef struct { char internal[128]; } ncclUniqueId;
typedef int ncclResult_t;
enum { OK = 0, INTERNAL = 3, INVALID_ARG = 4, INVALID_USAGE = 5, REMOTE = 6, IN_PROGRESS = 7 };
enum { STUB_MAX_BLOCK_S = 20, SLOT_BYTES = 8 << 20, MAX_WORLD = 8 };
enum { T_F32 = 7, T_F64 = 8, T_BF16 = 9 };           /* ncclFloat32 / ncclFloat64 / ncclBfloat16 */
enum { OP_SUM = 0, OP_AVG = 4 };                       /* ncclSum / ncclAvg */

typedef struct {                      /* the leading fields of ncclConfig_t */
  size_t size;
  unsigned int magic, version;
  int blocking;
} stub_config;

typedef struct {                      /* the shared segment of a functional (shm) communicator */
  atomic_int arrived, generation;
  char slot[MAX_WORLD][SLOT_BYTES];
} shm_seg;

typedef struct stub_comm {
  atomic_int aborted, pending;
  int rank, world, nonblocking, magic;
  shm_seg* seg;
} *ncclComm_t;

static atomic_int g_calls_in;   /* calls that entered a blocking entry point */

static int mode_shm(void) {
  const char* m = getenv("STUB_RCCL_MODE");
  return m && strcmp(m, "shm") == 0;
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  memset(id->internal, 0, 128);
  struct timespec t;
  clock_gettime(CLOCK_REALTIME, &t);
  snprintf(id->internal, 64, "/vitmi_stub_%d_%ld", (int)getpid(), (long)t.tv_nsec);
  return OK;
}

/* all ranks of the segment meet here (sense-reversing counter); 0 or a timeout */
static int seg_barrier(ncclComm_t c) {
  shm_seg* s = c->seg;
  const int gen = atomic_load(&s->generation);
  if (atomic_fetch_add(&s->arrived, 1) == c->world - 1) {
    atomic_store(&s->arrived, 0);
    atomic_fetch_add(&s->generation, 1);
    return 0;
  }
  const double t0 = now_s();
  while (atomic_load(&s->generation) == gen) {
    if (atomic_load(&c->aborted) || now_s() - t0 > STUB_MAX_BLOCK_S) return -1;
    struct timespec d = {0, 20000};
    nanosleep(&d, NULL);
  }
  return 0;
}

static ncclResult_t make_comm(ncclComm_t* out, int world, ncclUniqueId id, int rank, int nonblocking) {
  ncclComm_t c = (ncclComm_t)calloc(1, sizeof(*c));
  c->rank = rank;
  c->world = world;
  c->nonblocking = nonblocking;
  c->magic = 0x57ab;
  if (mode_shm() && world > 1) {
    if (world > MAX_WORLD) { free(c); return INVALID_ARG; }
    int fd = shm_open(id.internal, O_CREAT | O_RDWR, 0600);
    if (fd < 0) { free(c); return INTERNAL; }
    if (ftruncate(fd, sizeof(shm_seg)) != 0) { close(fd); free(c); return INTERNAL; }
    c->seg = (shm_seg*)mmap(NULL, sizeof(shm_seg), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (c->seg == MAP_FAILED) { free(c); return INTERNAL; }
    if (seg_barrier(c) != 0) return INTERNAL;      /* every rank mapped the segment */
    if (rank == 0) shm_unlink(id.internal);        /* the mappings keep it: nothing left in /dev/shm */
  }
  *out = c;
  return OK;
}

ncclResult_t ncclCommInitRank(ncclComm_t* c, int world, ncclUniqueId id, int rank) {
  return make_comm(c, world, id, rank, 0);
}

ncclResult_t ncclCommInitRankConfig(ncclComm_t* c, int world, ncclUniqueId id, int rank, stub_config* cfg) {
  const char* e = getenv("STUB_RCCL_NO_CONFIG");
  if (e && *e == '1') return INVALID_ARG;
  if (!cfg || cfg->magic != 0xcafebeef) return INVALID_ARG;
  return make_comm(c, world, id, rank, cfg->blocking == 0);
}

/* ---- block mode */
static ncclResult_t block_until_abort(ncclComm_t c) {
  atomic_fetch_add(&g_calls_in, 1);
  if (c->nonblocking) {               /* the enqueue returns; the state stays in progress */
    atomic_store(&c->pending, 1);
    return IN_PROGRESS;
  }
  const double t0 = now_s();
  for (;;) {
    if (atomic_load(&c->aborted)) return REMOTE;
    if (now_s() - t0 > STUB_MAX_BLOCK_S) return INTERNAL;
    struct timespec d = {0, 1000000};
    nanosleep(&d, NULL);
  }
}

/* ---- shm mode: HIP from the process */
typedef int (*hip_sync_t)(void*);
typedef int (*hip_memcpy_t)(void*, const void*, size_t, int);
static hip_sync_t p_sync;
static hip_memcpy_t p_memcpy;

static int host_sync(void* s) { (void)s; return 0; }
static int host_memcpy(void* d, const void* s, size_t n, int kind) { (void)kind; memcpy(d, s, n); return 0; }

static int bind_hip(void) {
  if (p_sync && p_memcpy) return 0;
  const char* host = getenv("STUB_RCCL_HOST");
  if (host && *host == '1') {
    p_sync = host_sync;
    p_memcpy = host_memcpy;
    return 0;
  }
  /* the HIP runtime the process already mapped (torch's, loaded RTLD_LOCAL), else the global scope */
  void* h = NULL;
  const char* names[] = {"libamdhip64.so.7", "libamdhip64.so", NULL};
  for (int i = 0; names[i] && !h; ++i) h = dlopen(names[i], RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = RTLD_DEFAULT;
  p_sync = (hip_sync_t)dlsym(h, "hipStreamSynchronize");
  p_memcpy = (hip_memcpy_t)dlsym(h, "hipMemcpy");
  return p_sync && p_memcpy ? 0 : -1;
}

static size_t elem_size(int t) { return t == T_F64 ? 8 : t == T_BF16 ? 2 : 4; }

static double load(const char* p, size_t i, int t) {
  if (t == T_F64) return ((const double*)p)[i];
  if (t == T_F32) return ((const float*)p)[i];
  uint32_t u = (uint32_t)((const uint16_t*)p)[i] << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

static void store(char* p, size_t i, int t, double v) {
  if (t == T_F64) { ((double*)p)[i] = v; return; }
  float f = (float)v;
  if (t == T_F32) { ((float*)p)[i] = f; return; }
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);                        /* round to nearest even */
  ((uint16_t*)p)[i] = (uint16_t)(u >> 16);
}

/* chunk by chunk: D2H into this rank's slot, barrier, combine, barrier, H2D */
static ncclResult_t shm_collective(const void* send, void* recv, size_t n, int t, int op, int root, ncclComm_t c,
                                   void* stream) {
  if (bind_hip() != 0) return INTERNAL;
  if (p_sync(stream) != 0) return INTERNAL;
  atomic_fetch_add(&g_calls_in, 1);
  const size_t es = elem_size(t), per = SLOT_BYTES / es;
  char* out = (char*)malloc(SLOT_BYTES);
  if (!out) return INTERNAL;
  for (size_t off = 0; off < n; off += per) {
    const size_t m = n - off < per ? n - off : per;
    if (p_memcpy(c->seg->slot[c->rank], (const char*)send + off * es, m * es, 2 /*D2H*/) != 0) { free(out); return INTERNAL; }
    if (seg_barrier(c) != 0) { free(out); return REMOTE; }
    if (root >= 0) {                                    /* broadcast */
      memcpy(out, c->seg->slot[root], m * es);
    } else {
      for (size_t i = 0; i < m; ++i) {
        double a = 0;
        if (t == T_F32) {                              /* fp32 sum in rank order, as RCCL's fp32 */
          float f = 0.f;
          for (int r = 0; r < c->world; ++r) f += (float)load(c->seg->slot[r], i, t);
          a = op == OP_AVG ? (double)(f / (float)c->world) : (double)f;
        } else {
          for (int r = 0; r < c->world; ++r) a += load(c->seg->slot[r], i, t);
          if (op == OP_AVG) a /= c->world;
        }
        store(out, i, t, a);
      }
    }
    if (seg_barrier(c) != 0) { free(out); return REMOTE; }   /* every rank has read the slots */
    if (p_memcpy((char*)recv + off * es, out, m * es, 1 /*H2D*/) != 0) { free(out); return INTERNAL; }
  }
  free(out);
  return OK;
}

ncclResult_t ncclAllReduce(const void* s, void* r, size_t n, int t, int op, ncclComm_t c, void* stream) {
  if (c->seg) return shm_collective(s, r, n, t, op, -1, c, stream);
  if (mode_shm()) return OK;                           /* world 1: the identity */
  return block_until_abort(c);
}

ncclResult_t ncclBroadcast(const void* s, void* r, size_t n, int t, int root, ncclComm_t c, void* stream) {
  if (c->seg) return shm_collective(s, r, n, t, OP_SUM, root, c, stream);
  if (mode_shm()) return OK;
  return block_until_abort(c);
}

ncclResult_t ncclCommAbort(ncclComm_t c) {
  atomic_store(&c->aborted, 1);
  if (c->nonblocking) {               /* poison and free: a later touch reads freed memory */
    if (c->seg) munmap(c->seg, sizeof(shm_seg));
    memset(c, 0xdd, sizeof(*c));
    free(c);
  }
  return OK;
}

ncclResult_t ncclCommDestroy(ncclComm_t c) {
  atomic_store(&c->aborted, 1);
  if (c->seg) munmap(c->seg, sizeof(shm_seg));
  c->seg = NULL;
  if (c->nonblocking) { memset(c, 0xdd, sizeof(*c)); free(c); }
  return OK;
}

const char* ncclGetErrorString(ncclResult_t r) { return r == REMOTE ? "remote error (stub: aborted)" : "stub error"; }

ncclResult_t ncclCommGetAsyncError(ncclComm_t c, ncclResult_t* a) {
  if (c->magic != 0x57ab) return INTERNAL;             /* a freed (poisoned) communicator */
  if (atomic_load(&c->aborted)) *a = REMOTE;
  else *a = atomic_load(&c->pending) ? IN_PROGRESS : OK;
  return OK;
}

int stub_calls_in(void) { return atomic_load(&g_calls_in); }
