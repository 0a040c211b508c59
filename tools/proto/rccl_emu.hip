// DIAGNOSTIC (tools/, not the product): a stand-in for one RCCL ring all-reduce kernel on one
// GPU, for the CU-contention sweep of tools/contention.py.  RCCL runs a collective as one block
// per channel, and every channel block must be running at once (each exchanges chunks with the
// peer GPUs in lockstep), so a channel block that finds no free CU holds up the others.  Here
// `nblocks` blocks first meet at an arrival counter (bounded spin: a block that waits longer
// than ~1 s proceeds anyway, so the kernel always drains), then stream their slice of the bucket
// three times through HBM (the 2 x 7/8 read + write volume of a ring all-reduce over 8 ranks).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void emu_allreduce(f32x4* __restrict__ buf, int64_t n4, unsigned* counter,
                                                     unsigned target, float one) {
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int spin = 0; spin < (1 << 18); ++spin) {
      if (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
      __builtin_amdgcn_s_sleep(127);
    }
  }
  __syncthreads();
  const int64_t per = (n4 + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * per, hi = lo + per < n4 ? lo + per : n4;
  // 16 loads in flight per thread (~64 KiB per block, RCCL-like per-channel bandwidth); a
  // runtime 1.0 keeps the load / store pairs from being folded away
  constexpr int U = 16;
  for (int pass = 0; pass < 3; ++pass)
    for (int64_t i0 = lo + threadIdx.x; i0 < hi; i0 += (int64_t)blockDim.x * U) {
      f32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = i0 + (int64_t)u * blockDim.x;
        if (i < hi) v[u] = buf[i];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = i0 + (int64_t)u * blockDim.x;
        if (i < hi) buf[i] = v[u] * one;
      }
    }
}

// counter: device int, zeroed once by the caller; gen = how many launches used it before (the
// arrival target grows by nblocks per launch, so no reset kernel is needed between launches)
extern "C" int emu_allreduce_launch(void* buf, int64_t n, int nblocks, void* counter, unsigned gen, void* stream) {
  if (nblocks < 1 || n % 4) return 1;
  hipLaunchKernelGGL(emu_allreduce, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, (f32x4*)buf, n / 4,
                     (unsigned*)counter, (gen + 1) * (unsigned)nblocks, 1.0f);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
