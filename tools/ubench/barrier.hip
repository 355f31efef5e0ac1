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

// flag barrier: block b stores its epoch into flags[b] (no atomics); wave 0
// of every block polls all flags (nblocks <= 64 * 16) until each is >= epoch
__device__ __forceinline__ void flag_barrier(uint32_t* flags, uint32_t epoch, uint32_t* err) {
  __syncthreads();
  if (threadIdx.x < 64) {
    if (threadIdx.x == 0) __hip_atomic_store(flags + blockIdx.x, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t n = 0;
    while (true) {
      bool ok = true;
      for (uint32_t b = threadIdx.x; b < gridDim.x; b += 64)
        ok = ok && __hip_atomic_load(flags + b, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >= epoch;
      if (__all(ok)) break;
      __builtin_amdgcn_s_sleep(1);
      if (++n > (1u << 22)) { if (threadIdx.x == 0) atomicOr(err, 2u); break; }
    }
  }
  __syncthreads();
}

// two-level: 8 group counters (block % 8), the last arriver of a group bumps
// the top counter; everyone polls the top counter
__device__ __forceinline__ void tree_barrier(uint32_t* ctr, uint32_t epoch, uint32_t* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t g = blockIdx.x & 7, gsize = (gridDim.x - g + 7) / 8;
    const uint32_t old = __hip_atomic_fetch_add(ctr + 16 + 16 * g, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == epoch * gsize) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t n = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < epoch * 8) {
      __builtin_amdgcn_s_sleep(1);
      if (++n > (1u << 22)) { atomicOr(err, 4u); break; }
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_flag_barriers(int nbar, uint32_t* flags, uint32_t* err, float* sink) {
  float acc = threadIdx.x;
  for (int i = 0; i < nbar; ++i) {
    acc = acc * 1.0001f + 1.f;
    flag_barrier(flags, (uint32_t)(i + 1), err);
  }
  if (acc == -1.f) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_tree_barriers(int nbar, uint32_t* ctr, uint32_t* err, float* sink) {
  float acc = threadIdx.x;
  for (int i = 0; i < nbar; ++i) {
    acc = acc * 1.0001f + 1.f;
    tree_barrier(ctr, (uint32_t)(i + 1), err);
  }
  if (acc == -1.f) sink[0] = acc;
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
  CHK(hipMalloc(&ctr, 4096 * 4));
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
  for (int kind = 1; kind <= 2; ++kind) {
    for (int grid : {64, 128, 256, 512}) {
      for (int rep = 0; rep < 2; ++rep) {
        CHK(hipMemset(ctr, 0, 4096 * 4));
        CHK(hipMemset(err, 0, 4));
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(a, 0));
        if (kind == 1)
          hipLaunchKernelGGL(k_flag_barriers, dim3(grid), dim3(256), 0, 0, nbar, ctr, err, sink);
        else
          hipLaunchKernelGGL(k_tree_barriers, dim3(grid), dim3(256), 0, 0, nbar, ctr, err, sink);
        CHK(hipEventRecord(b, 0));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        uint32_t e;
        CHK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
        printf("{\"test\": \"%s\", \"grid\": %d, \"us_per_barrier\": %.3f, \"timeout\": %u}\n",
               kind == 1 ? "flag_barrier" : "tree_barrier", grid, 1e3f * ms / nbar, e);
      }
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
