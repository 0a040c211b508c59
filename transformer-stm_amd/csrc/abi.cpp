// abi.cpp — library-level entry points of the C ABI: version, error reporting.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>
#include "../../include/vitmi.h"

namespace vitmi {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

// ---- per-kernel algorithmic work (VITMI_STAT, common.h)
bool g_stats_on = false;
namespace {
struct KStat {
  std::string name;
  int64_t calls = 0;
  double flops = 0, bytes = 0;
};
std::mutex g_stats_mu;
std::unordered_map<const void*, size_t> g_stats_idx;
std::vector<KStat> g_stats;
}  // namespace

void stat_record(const void* kernel, double flops, double bytes) {
  std::lock_guard<std::mutex> lk(g_stats_mu);
  auto it = g_stats_idx.find(kernel);
  size_t i;
  if (it == g_stats_idx.end()) {
    KStat k;
    const char* n = hipKernelNameRefByPtr(kernel, nullptr);   // the mangled device symbol
    k.name = n ? n : "?";
    i = g_stats.size();
    g_stats.push_back(k);
    g_stats_idx[kernel] = i;
  } else {
    i = it->second;
  }
  g_stats[i].calls += 1;
  g_stats[i].flops += flops;
  g_stats[i].bytes += bytes;
}

}  // namespace vitmi

extern "C" int vitmi_stats_enable(int on) {
  std::lock_guard<std::mutex> lk(vitmi::g_stats_mu);
  if (on) {
    vitmi::g_stats.clear();
    vitmi::g_stats_idx.clear();
  }
  vitmi::g_stats_on = on != 0;
  return VITMI_OK;
}

extern "C" int vitmi_stats_count(void) {
  std::lock_guard<std::mutex> lk(vitmi::g_stats_mu);
  return (int)vitmi::g_stats.size();
}

extern "C" int vitmi_stats_get(int i, char* name, int name_len, int64_t* calls, double* flops, double* bytes) {
  std::lock_guard<std::mutex> lk(vitmi::g_stats_mu);
  if (i < 0 || i >= (int)vitmi::g_stats.size()) return vitmi::fail(VITMI_ERR_INVALID, "stats_get: index %d", i);
  const vitmi::KStat& k = vitmi::g_stats[i];
  if (name && name_len > 0) snprintf(name, (size_t)name_len, "%s", k.name.c_str());
  if (calls) *calls = k.calls;
  if (flops) *flops = k.flops;
  if (bytes) *bytes = k.bytes;
  return VITMI_OK;
}

// ---- ROCTx ranges (SURVEY.md §5 profiling: ranges around fwd / bwd / all-reduce / optimizer).
// The ROCm 7 marker library (librocprofiler-sdk-roctx, what `rocprofv3 --marker-trace` records)
// is bound at run time on the first enable, so the library has no link dependency on it; while
// disabled (the default) a push/pop is one branch.
namespace {
typedef int (*roctx_push_t)(const char*);
typedef int (*roctx_pop_t)(void);
roctx_push_t g_roctx_push = nullptr;
roctx_pop_t g_roctx_pop = nullptr;
bool g_trace_on = false;
}  // namespace

extern "C" int vitmi_trace_enable(int on) {
  if (on && !g_roctx_push) {
    void* h = nullptr;
    const char* names[] = {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                           "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1"};
    for (const char* n : names)
      if ((h = dlopen(n, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
    if (!h) return vitmi::fail(VITMI_ERR_UNSUPPORTED, "trace_enable: cannot load the ROCTx library (%s)", dlerror());
    g_roctx_push = (roctx_push_t)dlsym(h, "roctxRangePushA");
    g_roctx_pop = (roctx_pop_t)dlsym(h, "roctxRangePop");
    if (!g_roctx_push || !g_roctx_pop) {
      g_roctx_push = nullptr;
      return vitmi::fail(VITMI_ERR_UNSUPPORTED, "trace_enable: ROCTx library lacks roctxRangePushA/Pop");
    }
  }
  g_trace_on = on != 0;
  return VITMI_OK;
}

extern "C" int vitmi_trace_push(const char* name) {
  if (!g_trace_on) return VITMI_OK;
  g_roctx_push(name ? name : "?");
  return VITMI_OK;
}

extern "C" int vitmi_trace_pop(void) {
  if (!g_trace_on) return VITMI_OK;
  g_roctx_pop();
  return VITMI_OK;
}

#ifndef VITMI_BUILD_ID
#define VITMI_BUILD_ID "unknown"
#endif
#ifndef VITMI_BUILD_FLAGS
#define VITMI_BUILD_FLAGS "unknown"
#endif

extern "C" int vitmi_version(void) { return 300; /* 0.3.0: + §8(b) per-op entry points, flags in the id */ }

extern "C" const char* vitmi_build_id(void) { return VITMI_BUILD_ID; }

extern "C" const char* vitmi_build_flags(void) { return VITMI_BUILD_FLAGS; }

extern "C" const char* vitmi_last_error(void) { return vitmi::g_err; }

extern "C" int vitmi_device_cus(void) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, dev) != hipSuccess) return 0;
  return p.multiProcessorCount;
}
