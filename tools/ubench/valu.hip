// Micro-benchmark: issue throughput of the VALU forms the render kernels are
// built from, with 8 waves per SIMD of independent chains (pure issue rate):
// v_fma_f32, v_pk_fma_f32, v_pk_add_f32, v_pk_mul_f32, v_exp_f32, v_rcp_f32,
// v_cndmask_b32 with an SGPR mask, v_cmp -> SGPR, DPP row adds,
// v_permlane32_swap.  Prints ns per wave-instruction per SIMD and the implied
// cycles at the measured clock-free rate (wave-instr/s per SIMD).
//   hipcc -O3 -fno-slp-vectorize --offload-arch=gfx950 tools/ubench/valu.hip -o tools/ubench/ub_valu
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef float v2f __attribute__((ext_vector_type(2)));
constexpr int kIters = 2048;

template <int OP>
__global__ __launch_bounds__(256) void k_op(float* out, float s) {
  float a[8];
  v2f p[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = threadIdx.x * 0.001f + i;
    p[i] = v2f{a[i], a[i] + 0.5f};
  }
  const v2f ps{s, s * 0.5f};
  const uint64_t msk = 0x5555555555555555ull ^ (uint64_t)blockIdx.x;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (OP == 0) a[i] = fmaf(a[i], s, 0.25f);
      if (OP == 1) p[i] = __builtin_elementwise_fma(p[i], ps, v2f{0.25f, 0.25f});
      if (OP == 2) p[i] = p[i] + ps;
      if (OP == 3) p[i] = p[i] * ps;
      if (OP == 4) a[i] = __builtin_amdgcn_exp2f(a[i]);
      if (OP == 5) a[i] = __builtin_amdgcn_rcpf(a[i]);
      if (OP == 6) a[i] = __builtin_amdgcn_inverse_ballot_w64(msk << (i + it)) ? a[i] : a[(i + 1) & 7];
      if (OP == 7) asm volatile("v_add_f32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a[i]));
      if (OP == 8) {
        auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a[i]), __float_as_uint(a[(i + 1) & 7]), false, false);
        a[i] = __uint_as_float(r[0]);
        a[(i + 1) & 7] = __uint_as_float(r[1]);
      }
      if (OP == 9) a[i] = a[i] + s;
    }
    if (OP == 6) asm volatile("" ::: "memory");
  }
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) acc += a[i] + p[i].x + p[i].y;
  if (acc == 12345.678f) out[threadIdx.x] = acc;
}

template <int OP>
int run(const char* name, float* out, int insts_per_iter) {
  int dev;
  hipDeviceProp_t prop;
  CHK(hipGetDevice(&dev));
  CHK(hipGetDeviceProperties(&prop, dev));
  const int ncu = prop.multiProcessorCount;
  const int blocks = ncu * 8;  // 8 blocks of 4 waves per CU: 8 waves per SIMD
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(k_op<OP>, dim3(blocks), dim3(256), 0, 0, out, 1.0001f);
  CHK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(k_op<OP>, dim3(blocks), dim3(256), 0, 0, out, 1.0001f);
    CHK(hipEventRecord(b, 0));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  const double waves = (double)blocks * 4, insts = waves * kIters * insts_per_iter;
  const double per_simd = insts / (ncu * 4.0);
  printf("{\"op\": \"%s\", \"ms\": %.4f, \"wave_instr_per_simd\": %.0f, \"ns_per_wave_instr_per_simd\": %.4f, "
         "\"cycles_at_2p4GHz\": %.3f}\n",
         name, best, per_simd, 1e6 * best / per_simd, 2.4 * 1e6 * best / per_simd);
  return 0;
}

int main() {
  float* out;
  CHK(hipMalloc(&out, 4096));
  run<0>("v_fma_f32", out, 8);
  run<9>("v_add_f32", out, 8);
  run<1>("v_pk_fma_f32", out, 8);
  run<2>("v_pk_add_f32", out, 8);
  run<3>("v_pk_mul_f32", out, 8);
  run<4>("v_exp_f32", out, 8);
  run<5>("v_rcp_f32", out, 8);
  run<6>("v_cndmask_b32(sgpr)", out, 8);
  run<7>("v_add_f32_dpp", out, 8);
  run<8>("v_permlane32_swap", out, 8);
  return 0;
}
