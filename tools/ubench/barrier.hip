// Micro-benchmark: cost of a device-wide barrier (one atomic counter, agent
// scope, bounded spin) inside one persistent kernel vs. a chain of dependent
// kernel launches on one stream.  Decides whether the per-Gaussian sorts
// (8 launches today) should become one persistent kernel.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench/barrier.hip -o /tmp/ub_barrier
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// arrive + wait; gives up after ~2^22 polls (flags the timeout) so that every
// wave reaches the end of the kernel whatever happens
__device__ __forceinline__ void grid_barrier(uint32_t* ctr, uint32_t target, uint32_t* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t n = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++n > (1u << 22)) { atomicOr(err, 1u); break; }
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_barriers(int nbar, uint32_t* ctr, uint32_t* err, float* sink) {
  float acc = threadIdx.x;
  for (int i = 0; i < nbar; ++i) {
    acc = acc * 1.0001f + 1.f;
    grid_barrier(ctr, (uint32_t)(i + 1) * gridDim.x, err);
  }
  if (acc == -1.f) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_empty(float* sink) {
  if (threadIdx.x == 1000) sink[0] = 1.f;
}

int main() {
  uint32_t *ctr, *err;
  float* sink;
  CHK(hipMalloc(&ctr, 4));
  CHK(hipMalloc(&err, 4));
  CHK(hipMalloc(&sink, 4));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const int nbar = 200;
  for (int grid : {64, 128, 256, 512}) {
    for (int rep = 0; rep < 3; ++rep) {
      CHK(hipMemset(ctr, 0, 4));
      CHK(hipMemset(err, 0, 4));
      CHK(hipDeviceSynchronize());
      CHK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(k_barriers, dim3(grid), dim3(256), 0, 0, nbar, ctr, err, sink);
      CHK(hipEventRecord(b, 0));
      CHK(hipEventSynchronize(b));
      float ms;
      CHK(hipEventElapsedTime(&ms, a, b));
      uint32_t e;
      CHK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
      printf("{\"test\": \"grid_barrier\", \"grid\": %d, \"us_per_barrier\": %.3f, \"timeout\": %u}\n", grid,
             1e3f * ms / nbar, e);
    }
  }
  for (int grid : {64, 512, 2048}) {
    for (int rep = 0; rep < 3; ++rep) {
      CHK(hipDeviceSynchronize());
      const int nl = 200;
      CHK(hipEventRecord(a, 0));
      for (int i = 0; i < nl; ++i) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, 0, sink);
      CHK(hipEventRecord(b, 0));
      CHK(hipEventSynchronize(b));
      float ms;
      CHK(hipEventElapsedTime(&ms, a, b));
      printf("{\"test\": \"launch_chain\", \"grid\": %d, \"us_per_launch\": %.3f}\n", grid, 1e3f * ms / nl);
    }
  }
  return 0;
}
