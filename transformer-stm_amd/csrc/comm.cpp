// comm.cpp — RCCL gradient exchange of the data-parallel path.
//
// The reference's only parallel construct is tf.distribute.MirroredStrategy()
// (old_codes/BayConvT(Par)(Muti).py:16-19): synchronous data parallelism whose
// cross-replica gradient reduction TF runs as an NCCL all-reduce on one host.  Here it is
// one process per GPU and one RCCL communicator per process; buckets of the flat gradient
// buffer are all-reduced on a caller-owned side stream, gated by a hipEvent recorded on
// the compute stream, so the exchange overlaps the rest of the backward (vitmi/dp.py).
//
// RCCL is bound at run time (dlopen/dlsym), preferring the copy already mapped into the
// process: PyTorch-ROCm loads its own librccl.so, and two RCCL instances in one process
// would each start their own proxy threads and IPC state.  No RCCL symbol is linked, so
// the library still loads (and every other entry point works) where RCCL is absent.
//
// RCCL is taken from VITMI_RCCL_LIB when that is set (a specific build; the CPU tests' stub).
//
// Thread safety.  The communicator is created NON-BLOCKING (ncclCommInitRankConfig, blocking = 0):
// no RCCL call then waits for a peer (an enqueue returns ncclInProgress and the wait is a poll of
// ncclCommGetAsyncError), so every RCCL call on a communicator runs under g_mu, and the DP
// watchdog's abort (vitmi_comm_destroy(1), from its own thread: vitmi/dp.py CommWatchdog) takes
// g_mu too: ncclCommAbort can never free the handle under another thread's call.  A
// poll drops the lock between two queries and gives up as soon as the communicator is released.
// The Comm wrapper is reference-counted (enqueues in flight hold one), so it outlives the handle.
// Where the RCCL build lacks ncclCommInitRankConfig (or refuses the config) the communicator is
// blocking: calls then run WITHOUT the lock, because an enqueue blocked on a dead peer is what
// the abort must release, and the abort is not serialised with them (the older scheme).
// A graceful vitmi_comm_destroy(0) waits for in-flight calls before ncclCommDestroy.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <condition_variable>
#include <mutex>
#include <stdlib.h>
#include <rccl/rccl.h>
#include <chrono>
#include <thread>
#include <stdio.h>
#include <string.h>
#include "common.h"

namespace vitmi {
namespace {

struct Rccl {
  void* handle = nullptr;
  decltype(&::ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&::ncclCommInitRank) init_rank = nullptr;
  decltype(&::ncclCommInitRankConfig) init_rank_config = nullptr;   // optional (non-blocking init)
  decltype(&::ncclAllReduce) all_reduce = nullptr;
  decltype(&::ncclBroadcast) broadcast = nullptr;
  decltype(&::ncclCommDestroy) destroy = nullptr;
  decltype(&::ncclCommAbort) abort = nullptr;
  decltype(&::ncclGetErrorString) err = nullptr;
  decltype(&::ncclCommGetAsyncError) async_err = nullptr;
};

Rccl g_rccl;
std::mutex g_mu;                 // guards g_rccl loading, g_cur and every Comm's users / detached
std::condition_variable g_idle;  // a Comm's users dropped to 0 (graceful destroy waits for it)

// One communicator and the calls currently inside it.
struct Comm {
  ncclComm_t comm = nullptr;
  int rank = -1, world = 0;
  bool nonblocking = false;  // created with blocking = 0: RCCL calls run under g_mu
  int users = 0;           // enqueues in flight (between acquire and release)
  bool detached = false;   // no longer current: destroy / abort took it
  bool released = false;   // its RCCL handle is gone (aborted or destroyed)
};
Comm* g_cur = nullptr;

// A reference to the current communicator for one RCCL call, or null.
Comm* acquire() {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_cur) return nullptr;
  ++g_cur->users;
  return g_cur;
}

// Drop a reference; the last one out of a detached and released communicator frees it.
void release(Comm* c) {
  bool free_it = false;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    free_it = --c->users == 0 && c->detached && c->released;
    if (c->users == 0) g_idle.notify_all();
  }
  if (free_it) delete c;
}

struct Ref {   // scope guard around acquire / release
  Comm* c;
  Ref() : c(acquire()) {}
  ~Ref() { if (c) release(c); }
};

template <typename F>
bool sym(void* h, const char* name, F& out) {
  out = reinterpret_cast<F>(dlsym(h, name));
  return out != nullptr;
}

int bind_rccl(void* h);

int load_rccl() {
  if (g_rccl.handle) return VITMI_OK;
  const char* pinned = getenv("VITMI_RCCL_LIB");
  if (pinned && *pinned) {
    void* hp = dlopen(pinned, RTLD_NOW | RTLD_LOCAL);
    if (!hp) return fail(VITMI_ERR_COMM, "comm: cannot load VITMI_RCCL_LIB=%s (%s)", pinned, dlerror());
    return bind_rccl(hp);
  }
  // already mapped (torch's bundled copy is loaded by its file name, it has no SONAME)?
  const char* names[] = {"librccl.so", "librccl.so.1"};
  void* h = nullptr;
  for (const char* n : names)
    if ((h = dlopen(n, RTLD_NOW | RTLD_NOLOAD)) != nullptr) break;
  if (!h)
    for (const char* n : names)
      if ((h = dlopen(n, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
  if (!h) return fail(VITMI_ERR_COMM, "comm: cannot load librccl.so (%s)", dlerror());
  return bind_rccl(h);
}

int bind_rccl(void* h) {
  Rccl r;
  r.handle = h;
  if (!sym(h, "ncclGetUniqueId", r.get_unique_id) || !sym(h, "ncclCommInitRank", r.init_rank) ||
      !sym(h, "ncclAllReduce", r.all_reduce) || !sym(h, "ncclBroadcast", r.broadcast) ||
      !sym(h, "ncclCommDestroy", r.destroy) || !sym(h, "ncclCommAbort", r.abort) ||
      !sym(h, "ncclGetErrorString", r.err) || !sym(h, "ncclCommGetAsyncError", r.async_err))
    return fail(VITMI_ERR_COMM, "comm: librccl.so lacks an NCCL 2.x entry point");
  sym(h, "ncclCommInitRankConfig", r.init_rank_config);
  g_rccl = r;
  return VITMI_OK;
}

int nccl_fail(const char* what, ncclResult_t r) {
  return fail(VITMI_ERR_COMM, "comm: %s: %s (%d)", what, g_rccl.err ? g_rccl.err(r) : "?", (int)r);
}

bool dtype_of(int dtype, ncclDataType_t& t) {
  if (dtype == VITMI_F32) t = ncclFloat32;
  else if (dtype == VITMI_BF16) t = ncclBfloat16;
  else if (dtype == VITMI_F64) t = ncclFloat64;
  else return false;
  return true;
}

// Poll a non-blocking communicator until its pending operation (init or an enqueue) has left
// ncclInProgress; the lock is held only around each query, and a released communicator (the
// watchdog's abort) ends the wait.  `deadline_s` > 0 bounds it (init).  -> the final state.
ncclResult_t wait_ready(Comm* c, double deadline_s, bool* released) {
  const auto t0 = std::chrono::steady_clock::now();
  *released = false;
  for (int spin = 0;; ++spin) {
    ncclResult_t a = ncclSuccess, r;
    {
      std::lock_guard<std::mutex> lk(g_mu);
      if (c->released) { *released = true; return ncclInvalidUsage; }
      r = g_rccl.async_err(c->comm, &a);
    }
    if (r != ncclSuccess) return r;
    if (a != ncclInProgress) return a;
    if (deadline_s > 0 &&
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > deadline_s)
      return ncclInProgress;
    if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
    else std::this_thread::yield();
  }
}

// One collective enqueue on the communicator `c` (a reference the caller holds): under g_mu for a
// non-blocking communicator (re-checking that it was not released), then the poll; without the
// lock for a blocking one.
template <typename F>
int enqueue(Comm* c, const char* what, F call) {
  ncclResult_t r;
  if (c->nonblocking) {
    {
      std::lock_guard<std::mutex> lk(g_mu);
      if (c->released) return fail(VITMI_ERR_COMM, "comm: %s: communicator aborted", what);
      r = call(c->comm);
    }
    if (r == ncclInProgress) {
      bool rel = false;
      r = wait_ready(c, 0, &rel);
      if (rel) return fail(VITMI_ERR_COMM, "comm: %s: communicator aborted", what);
    }
  } else {
    r = call(c->comm);   // no lock held: an abort from another thread may release this call
  }
  return r ? nccl_fail(what, r) : VITMI_OK;
}

}  // namespace
}  // namespace vitmi

using namespace vitmi;

extern "C" int vitmi_comm_get_unique_id(char* uid) {
  VITMI_CHECK_ARG(uid != nullptr, "comm_get_unique_id: uid is null");
  std::lock_guard<std::mutex> lk(g_mu);
  if (int rc = load_rccl()) return rc;
  ncclUniqueId id;
  if (ncclResult_t r = g_rccl.get_unique_id(&id)) return nccl_fail("ncclGetUniqueId", r);
  static_assert(sizeof(id.internal) == VITMI_COMM_UID_BYTES, "ncclUniqueId size");
  memcpy(uid, id.internal, VITMI_COMM_UID_BYTES);
  return VITMI_OK;
}

extern "C" int vitmi_comm_init(int rank, int world, const char* uid) {
  VITMI_CHECK_ARG(world >= 1 && rank >= 0 && rank < world, "comm_init: rank %d / world %d", rank, world);
  VITMI_CHECK_ARG(uid != nullptr, "comm_init: uid is null");
  {
    std::lock_guard<std::mutex> lk(g_mu);
    VITMI_CHECK_ARG(g_cur == nullptr, "comm_init: a communicator already exists (vitmi_comm_destroy first)");
    if (int rc = load_rccl()) return rc;
  }
  ncclUniqueId id;
  memcpy(id.internal, uid, VITMI_COMM_UID_BYTES);
  ncclComm_t c = nullptr;
  bool nonblocking = false;
  // the communicator binds to the calling thread's current HIP device; the rendezvous with the
  // other ranks runs without the lock held.  Non-blocking where the library takes a config: the
  // init is then a poll bounded by VITMI_COMM_INIT_TIMEOUT_S (default 600 s), so a rank whose
  // peer never joins fails instead of blocking for ever
  if (g_rccl.init_rank_config) {
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r = g_rccl.init_rank_config(&c, world, id, rank, &cfg);
    if (r == ncclSuccess || r == ncclInProgress) {
      nonblocking = true;
      if (r == ncclInProgress) {
        const char* e = getenv("VITMI_COMM_INIT_TIMEOUT_S");
        const double tmo = e && *e ? atof(e) : 600.0;
        Comm probe;   // not published: only wait_ready's view of the handle
        probe.comm = c;
        bool rel = false;
        r = wait_ready(&probe, tmo > 0 ? tmo : 600.0, &rel);
        if (r != ncclSuccess) {
          g_rccl.abort(c);
          return r == ncclInProgress ? fail(VITMI_ERR_COMM, "comm_init: ncclCommInitRankConfig not done after %g s "
                                                            "(a peer never joined?)", tmo)
                                     : nccl_fail("ncclCommInitRankConfig", r);
        }
      }
    } else if (r != ncclInvalidArgument && r != ncclInvalidUsage) {
      return nccl_fail("ncclCommInitRankConfig", r);
    } else {
      c = nullptr;   // the library refused the config: blocking init below
    }
  }
  if (!nonblocking)
    if (ncclResult_t r = g_rccl.init_rank(&c, world, id, rank)) return nccl_fail("ncclCommInitRank", r);
  std::unique_lock<std::mutex> lk(g_mu);
  if (g_cur != nullptr) {
    lk.unlock();
    g_rccl.destroy(c);
    return fail(VITMI_ERR_INVALID, "comm_init: a communicator was created concurrently");
  }
  Comm* n = new Comm;
  n->comm = c;
  n->rank = rank;
  n->world = world;
  n->nonblocking = nonblocking;
  g_cur = n;
  return VITMI_OK;
}

extern "C" int vitmi_comm_library(char* path, int len) {
  VITMI_CHECK_ARG(path != nullptr && len > 0, "comm_library: bad buffer");
  std::lock_guard<std::mutex> lk(g_mu);
  if (int rc = load_rccl()) return rc;
  Dl_info info;
  if (!dladdr(reinterpret_cast<void*>(g_rccl.all_reduce), &info) || !info.dli_fname)
    return fail(VITMI_ERR_COMM, "comm_library: dladdr(ncclAllReduce) failed");
  snprintf(path, (size_t)len, "%s", info.dli_fname);
  return VITMI_OK;
}

extern "C" int vitmi_comm_info(int* rank, int* world) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (rank) *rank = g_cur ? g_cur->rank : -1;
  if (world) *world = g_cur ? g_cur->world : 0;
  return g_cur ? VITMI_OK : fail(VITMI_ERR_INVALID, "comm_info: no communicator");
}

extern "C" int vitmi_comm_allreduce_async(void* ptr, int64_t count, int dtype, int op, vitmi_stream_t side,
                                          void* ready_event) {
  VITMI_CHECK_ARG(count >= 0, "comm_allreduce_async: negative count");
  VITMI_CHECK_ARG(op == VITMI_REDUCE_SUM || op == VITMI_REDUCE_AVG, "comm_allreduce_async: bad op %d", op);
  ncclDataType_t t;
  VITMI_CHECK_ARG(dtype_of(dtype, t), "comm_allreduce_async: bad dtype %d", dtype);
  Ref ref;
  VITMI_CHECK_ARG(ref.c != nullptr, "comm_allreduce_async: no communicator (never initialised, or aborted)");
  if (count == 0) return VITMI_OK;
  VITMI_CHECK_ARG(ptr != nullptr, "comm_allreduce_async: null buffer");
  hipStream_t s = (hipStream_t)side;
  if (ready_event) {
    hipError_t e = hipStreamWaitEvent(s, (hipEvent_t)ready_event, 0);
    if (e != hipSuccess) return fail(VITMI_ERR_HIP, "comm_allreduce_async: hipStreamWaitEvent: %s", hipGetErrorString(e));
  }
  const ncclRedOp_t rop = op == VITMI_REDUCE_AVG ? ncclAvg : ncclSum;
  return enqueue(ref.c, "ncclAllReduce",
                 [&](ncclComm_t c) { return g_rccl.all_reduce(ptr, ptr, (size_t)count, t, rop, c, s); });
}

extern "C" int vitmi_comm_broadcast(void* ptr, int64_t count, int dtype, int root, vitmi_stream_t stream) {
  ncclDataType_t t;
  VITMI_CHECK_ARG(dtype_of(dtype, t), "comm_broadcast: bad dtype %d", dtype);
  Ref ref;
  VITMI_CHECK_ARG(ref.c != nullptr, "comm_broadcast: vitmi_comm_init first");
  VITMI_CHECK_ARG(root >= 0 && root < ref.c->world, "comm_broadcast: bad root %d", root);
  if (count == 0) return VITMI_OK;
  return enqueue(ref.c, "ncclBroadcast", [&](ncclComm_t c) {
    return g_rccl.broadcast(ptr, ptr, (size_t)count, t, root, c, (hipStream_t)stream);
  });
}

extern "C" int vitmi_comm_check(void) {
  Ref ref;
  if (!ref.c) return VITMI_OK;
  ncclResult_t a = ncclSuccess, r;
  {
    // (a non-blocking communicator's handle is only touched under the lock; see the header)
    std::unique_lock<std::mutex> lk(g_mu, std::defer_lock);
    if (ref.c->nonblocking) {
      lk.lock();
      if (ref.c->released) return fail(VITMI_ERR_COMM, "comm_check: communicator aborted");
    }
    r = g_rccl.async_err(ref.c->comm, &a);
  }
  if (r) return nccl_fail("ncclCommGetAsyncError", r);
  if (a != ncclSuccess && a != ncclInProgress) return nccl_fail("asynchronous error", a);
  return VITMI_OK;
}

extern "C" int vitmi_comm_destroy(int abort) {
  std::unique_lock<std::mutex> lk(g_mu);
  Comm* c = g_cur;
  if (!c) return VITMI_OK;
  g_cur = nullptr;          // new calls see no communicator from here on
  c->detached = true;
  // graceful: ncclCommDestroy must not run under an in-flight call; abort: do not wait
  if (!abort) g_idle.wait(lk, [c] { return c->users == 0; });
  ncclResult_t r;
  if (abort && c->nonblocking) {
    // under the lock: no other thread is inside an RCCL call on this handle (they all take
    // g_mu, and none blocks while holding it), and every later one sees `released` first
    r = g_rccl.abort(c->comm);
    c->released = true;
  } else {
    lk.unlock();
    r = abort ? g_rccl.abort(c->comm) : g_rccl.destroy(c->comm);
    lk.lock();
    c->released = true;
  }
  const bool free_it = c->users == 0;
  lk.unlock();
  if (free_it) delete c;
  return r ? nccl_fail(abort ? "ncclCommAbort" : "ncclCommDestroy", r) : VITMI_OK;
}
