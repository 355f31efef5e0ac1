// Densification on the device, gfx950:
// GaussianModel.densify_and_prune / prune_points / reset_opacity[_nonvisible]
// (thirdparty/gaussian_splatting/scene/gaussian_model.py:389-420, 526-743) on
// a capacity-preallocated SoA (wgsr/store.py): two banks of parameters + Adam
// moments + keyframe ids / observation counts; a densify reads one bank and
// writes the other, so no torch.cat / boolean-index re-allocation happens.
//
// The reference's composition, row by row:
//   grads = accum / denom (NaN -> 0)
//   clone   sel_c = |g| >= thr && max(exp(s)) <= percent_dense * extent
//           -> rows appended: [P rows | clones]
//   split   sel_s = g >= thr && max(exp(s)) > percent_dense * extent (over the
//           P original rows; the appended clones carry a padded gradient 0)
//           -> rows appended twice (copy A block, copy B block): xyz =
//           R(q) (z * exp(s)) + xyz, scaling = log(exp(s) / (0.8 N)), the rest
//           copied; then the selected originals are pruned
//   prune   sigmoid(o) < min_opacity, or with a screen size:
//           max_radii2D > max_screen_size (max_radii2D was just reset to 0 by
//           densification_postfix, so this term is 0 > max_screen_size) or
//           max(exp(s)) > 0.1 extent
//   new rows get zero Adam moments; accum / denom / max_radii2D end zero.
// So the final table is the stable concatenation of four regions -- kept
// originals, kept clones, kept split copies A, kept split copies B -- each in
// index order: one select kernel (flags + per-block counts of the four
// regions and of the split selection), one scan, one emit kernel.
//
// Split noise: z ~ N(0, 1) of [2 Ns, 3] (Ns = selected split rows) is an
// INPUT (the reference draws torch.normal(0, stds) = z * stds), so parity
// with a composition fed the same z is exact up to the 3x3 product.
#include "wgsr_common.h"
#include "wgsr_internal.h"

namespace wgsr {

namespace {

constexpr int kDenBlock = 256;
constexpr int kDenWaves = kDenBlock / 64;

// flag bits
constexpr uint32_t kKeepOrig = 1u, kKeepClone = 2u, kKeepSplit = 4u, kSelSplit = 8u;

// fp32 ops one at a time (torch's elementwise kernels round every op)
__device__ __forceinline__ float fmul(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float fadd(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float fsub(float a, float b) { return __fsub_rn(a, b); }

__device__ __forceinline__ float sigmoidf_torch(float x) { return 1.0f / (1.0f + expf(-x)); }

struct DenParams {
  float grad_thr, dense_thr, min_opacity, world_thr;
  int screen;          // max_screen_size given (truthy)
  float screen_size;
  int mode;            // 0 densify_and_prune, 1 prune by mask
};

// block-exclusive prefix of a 0/1 predicate per thread, and the block total
__device__ __forceinline__ uint32_t block_prefix(bool p, uint32_t* s_w, uint32_t& total) {
  const int t = threadIdx.x, w = t >> 6;
  const uint64_t m = wave_ballot(p);
  if ((t & 63) == 0) s_w[w] = (uint32_t)__popcll(m);
  __syncthreads();
  uint32_t before = 0;
  total = 0;
#pragma unroll
  for (int k = 0; k < kDenWaves; ++k) {
    const uint32_t v = s_w[k];
    before += k < w ? v : 0u;
    total += v;
  }
  __syncthreads();
  return before + lanes_below(m);
}

__global__ __launch_bounds__(kDenBlock) void k_densify_select(int64_t P, const float* __restrict__ accum,
                                                              const float* __restrict__ denom,
                                                              const float* __restrict__ opacity,
                                                              const float* __restrict__ scaling,
                                                              const uint8_t* __restrict__ prune_mask, DenParams dp,
                                                              uint8_t* __restrict__ flags,
                                                              uint4* __restrict__ bcounts) {
  __shared__ uint32_t s_w[kDenWaves];
  const int64_t i = (int64_t)blockIdx.x * kDenBlock + threadIdx.x;
  uint32_t f = 0;
  if (i < P) {
    if (dp.mode == 1) {
      f = prune_mask[i] ? 0u : kKeepOrig;
    } else {
      float g = accum[i] / denom[i];
      if (g != g) g = 0.f;  // grads[grads.isnan()] = 0
      const float s0 = expf(scaling[3 * i]), s1 = expf(scaling[3 * i + 1]), s2 = expf(scaling[3 * i + 2]);
      const float smax = fmaxf(fmaxf(s0, s1), s2);
      const bool big = fabsf(g) >= dp.grad_thr;
      const bool sel_c = big && smax <= dp.dense_thr;
      const bool sel_s = g >= dp.grad_thr && smax > dp.dense_thr;
      const float o = sigmoidf_torch(opacity[i]);
      const bool p_op = o < dp.min_opacity;
      const bool p_vs = dp.screen && 0.f > dp.screen_size;  // max_radii2D was reset to 0
      const bool prune_o = p_op || p_vs || (dp.screen && smax > dp.world_thr);
      // split copies: scaling log(exp(s) / (0.8 N)) -> exp() again for the test
      const float inv = 1.0f / 1.6f;
      const float n0 = expf(logf(fmul(s0, inv))), n1 = expf(logf(fmul(s1, inv))), n2 = expf(logf(fmul(s2, inv)));
      const bool prune_s = p_op || p_vs || (dp.screen && fmaxf(fmaxf(n0, n1), n2) > dp.world_thr);
      f = (!sel_s && !prune_o ? kKeepOrig : 0u) | (sel_c && !prune_o ? kKeepClone : 0u) |
          (sel_s && !prune_s ? kKeepSplit : 0u) | (sel_s ? kSelSplit : 0u);
    }
    flags[i] = (uint8_t)f;
  }
  uint32_t t0, t1, t2, t3;
  block_prefix(f & kKeepOrig, s_w, t0);
  block_prefix(f & kKeepClone, s_w, t1);
  block_prefix(f & kKeepSplit, s_w, t2);
  block_prefix(f & kSelSplit, s_w, t3);
  if (threadIdx.x == 0) bcounts[blockIdx.x] = make_uint4(t0, t1, t2, t3);
}

// exclusive scan of the per-block counts in place; totals at bcounts[nb]
__global__ __launch_bounds__(1024) void k_densify_scan(uint4* __restrict__ bcounts, uint32_t nb) {
  __shared__ uint4 s_w[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint32_t per = (nb + 1023) / 1024, b0 = min(nb, t * per), b1 = min(nb, b0 + per);
  uint4 acc = make_uint4(0u, 0u, 0u, 0u);
  for (uint32_t b = b0; b < b1; ++b) {
    const uint4 v = bcounts[b];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  const uint32_t ix = wave_incl_scan(acc.x), iy = wave_incl_scan(acc.y), iz = wave_incl_scan(acc.z),
                 iw = wave_incl_scan(acc.w);
  if (lane == 63) s_w[w] = make_uint4(ix, iy, iz, iw);
  __syncthreads();
  uint4 run = make_uint4(ix - acc.x, iy - acc.y, iz - acc.z, iw - acc.w), tot = make_uint4(0u, 0u, 0u, 0u);
  for (int k = 0; k < 16; ++k) {
    const uint4 x = s_w[k];
    if (k < w) { run.x += x.x; run.y += x.y; run.z += x.z; run.w += x.w; }
    tot.x += x.x; tot.y += x.y; tot.z += x.z; tot.w += x.w;
  }
  for (uint32_t b = b0; b < b1; ++b) {
    const uint4 v = bcounts[b];
    bcounts[b] = run;
    run.x += v.x; run.y += v.y; run.z += v.z; run.w += v.w;
  }
  if (t == 0) bcounts[nb] = tot;
}

__device__ __forceinline__ void copy_row(const float* __restrict__ src, float* __restrict__ dst, int64_t from,
                                         int64_t to, int n) {
  for (int k = 0; k < n; ++k) dst[to * n + k] = src[from * n + k];
}
__device__ __forceinline__ void zero_row(float* __restrict__ dst, int64_t to, int n) {
  for (int k = 0; k < n; ++k) dst[to * n + k] = 0.f;
}

// One output row of the bank: params from (src row i) with an optional new
// xyz / scaling, moments copied (kept originals) or zero (new rows).
__device__ void emit_row(const wgsr_gaussian_bank& S, const wgsr_gaussian_bank& D, int F, int64_t i, int64_t r,
                         bool moments, const float* xyz_new, const float* sc_new) {
  const int widths[5] = {3, F, 1, 3, 4};
  const float* sp[5] = {S.xyz, S.features, S.opacity, S.scaling, S.rotation};
  float* dp[5] = {D.xyz, D.features, D.opacity, D.scaling, D.rotation};
  for (int k = 0; k < 5; ++k) {
    if (k == 0 && xyz_new) {
      for (int c = 0; c < 3; ++c) D.xyz[3 * r + c] = xyz_new[c];
    } else if (k == 3 && sc_new) {
      for (int c = 0; c < 3; ++c) D.scaling[3 * r + c] = sc_new[c];
    } else {
      copy_row(sp[k], dp[k], i, r, widths[k]);
    }
    if (moments) {
      copy_row(S.exp_avg[k], D.exp_avg[k], i, r, widths[k]);
      copy_row(S.exp_avg_sq[k], D.exp_avg_sq[k], i, r, widths[k]);
    } else {
      zero_row(D.exp_avg[k], r, widths[k]);
      zero_row(D.exp_avg_sq[k], r, widths[k]);
    }
  }
  if (S.kf_id && D.kf_id) D.kf_id[r] = S.kf_id[i];
  if (S.n_obs && D.n_obs) D.n_obs[r] = S.n_obs[i];
}

// build_rotation (general_utils.py:113-136), op by op
__device__ __forceinline__ void build_rotation(const float* q4, float R[9]) {
  const float a = q4[0], b = q4[1], c = q4[2], d = q4[3];
  const float norm = sqrtf(fadd(fadd(fadd(fmul(a, a), fmul(b, b)), fmul(c, c)), fmul(d, d)));
  const float r = a / norm, x = b / norm, y = c / norm, z = d / norm;
  R[0] = fsub(1.f, fmul(2.f, fadd(fmul(y, y), fmul(z, z))));
  R[1] = fmul(2.f, fsub(fmul(x, y), fmul(r, z)));
  R[2] = fmul(2.f, fadd(fmul(x, z), fmul(r, y)));
  R[3] = fmul(2.f, fadd(fmul(x, y), fmul(r, z)));
  R[4] = fsub(1.f, fmul(2.f, fadd(fmul(x, x), fmul(z, z))));
  R[5] = fmul(2.f, fsub(fmul(y, z), fmul(r, x)));
  R[6] = fmul(2.f, fsub(fmul(x, z), fmul(r, y)));
  R[7] = fmul(2.f, fadd(fmul(y, z), fmul(r, x)));
  R[8] = fsub(1.f, fmul(2.f, fadd(fmul(x, x), fmul(y, y))));
}

__global__ __launch_bounds__(kDenBlock) void k_densify_emit(int64_t P, int F, const uint8_t* __restrict__ flags,
                                                            const uint4* __restrict__ bcounts, uint32_t nb,
                                                            const float* __restrict__ z, wgsr_gaussian_bank S,
                                                            wgsr_gaussian_bank D) {
  __shared__ uint32_t s_w[kDenWaves];
  const int64_t i = (int64_t)blockIdx.x * kDenBlock + threadIdx.x;
  const uint32_t f = i < P ? flags[i] : 0u;
  uint32_t t;
  const uint32_t p0 = block_prefix(f & kKeepOrig, s_w, t);
  const uint32_t p1 = block_prefix(f & kKeepClone, s_w, t);
  const uint32_t p2 = block_prefix(f & kKeepSplit, s_w, t);
  const uint32_t p3 = block_prefix(f & kSelSplit, s_w, t);
  if (i >= P || f == 0u) return;
  const uint4 base = bcounts[blockIdx.x], tot = bcounts[nb];
  if (f & kKeepOrig) emit_row(S, D, F, i, (int64_t)base.x + p0, true, nullptr, nullptr);
  if (f & kKeepClone) emit_row(S, D, F, i, (int64_t)tot.x + base.y + p1, false, nullptr, nullptr);
  if (f & kKeepSplit) {
    const int64_t ns = tot.w, rank = (int64_t)base.w + p3;
    float R[9];
    build_rotation(&S.rotation[4 * i], R);
    const float s[3] = {expf(S.scaling[3 * i]), expf(S.scaling[3 * i + 1]), expf(S.scaling[3 * i + 2])};
    const float inv = 1.0f / 1.6f;
    const float sc_new[3] = {logf(fmul(s[0], inv)), logf(fmul(s[1], inv)), logf(fmul(s[2], inv))};
    const int64_t r0 = (int64_t)tot.x + tot.y + base.z + p2;
    for (int copy = 0; copy < 2; ++copy) {
      const float* zz = z + 3 * (copy * ns + rank);
      // torch.normal(mean=0, std) = z * std + 0; then bmm(R, sample) + xyz
      const float smp[3] = {fadd(fmul(zz[0], s[0]), 0.f), fadd(fmul(zz[1], s[1]), 0.f), fadd(fmul(zz[2], s[2]), 0.f)};
      float xyz[3];
      for (int c = 0; c < 3; ++c)
        xyz[c] = fadd(fadd(fadd(fmul(R[3 * c], smp[0]), fmul(R[3 * c + 1], smp[1])), fmul(R[3 * c + 2], smp[2])),
                      S.xyz[3 * i + c]);
      emit_row(S, D, F, i, r0 + copy * (int64_t)tot.z, false, xyz, sc_new);
    }
  }
}

// reset_opacity / reset_opacity_nonvisible: raw opacity -> value (or, for a
// visible Gaussian, sigmoid(raw): the reference stores get_opacity[filter],
// the ACTIVATED value, into the raw tensor), opacity Adam moments -> 0
__global__ __launch_bounds__(kDenBlock) void k_reset_opacity(int64_t P, float* __restrict__ raw,
                                                             const uint8_t* __restrict__ visible, float value,
                                                             float* __restrict__ m, float* __restrict__ v) {
  const int64_t i = (int64_t)blockIdx.x * kDenBlock + threadIdx.x;
  if (i >= P) return;
  raw[i] = (visible && visible[i]) ? sigmoidf_torch(raw[i]) : value;
  m[i] = 0.f;
  v[i] = 0.f;
}

inline unsigned den_blocks(int64_t n) { return (unsigned)((n + kDenBlock - 1) / kDenBlock); }

}  // namespace

}  // namespace wgsr

using namespace wgsr;

extern "C" {

int64_t wgsr_densify_blocks(int64_t P) { return P > 0 ? (int64_t)den_blocks(P) : 0; }

int wgsr_densify_select(int64_t P, const float* accum, const float* denom, const float* opacity,
                        const float* scaling, const uint8_t* prune_mask, float grad_threshold, float dense_threshold,
                        float min_opacity, float world_threshold, int use_screen_size, float max_screen_size,
                        uint8_t* flags, uint32_t* block_counts, void* stream) {
  if (P < 0 || P > ((int64_t)1 << 31)) return set_error(WGSR_EINVAL, "wgsr_densify_select: bad P");
  if (!block_counts) return set_error(WGSR_EINVAL, "wgsr_densify_select: null block_counts");
  hipStream_t s = (hipStream_t)stream;
  const unsigned nb = den_blocks(P);
  if (P > 0) {
    const int mode = prune_mask ? 1 : 0;
    if (!flags || (!mode && (!accum || !denom || !opacity || !scaling)))
      return set_error(WGSR_EINVAL, "wgsr_densify_select: null pointer");
    if (!mode && !(grad_threshold > 0.f))
      return set_error(WGSR_EINVAL, "wgsr_densify_select: grad_threshold must be > 0 (the appended clones' padded "
                                    "gradient 0 must not select them for a split)");
    DenParams dp{grad_threshold, dense_threshold, min_opacity, world_threshold, use_screen_size ? 1 : 0,
                 max_screen_size, mode};
    hipLaunchKernelGGL(k_densify_select, dim3(nb), dim3(kDenBlock), 0, s, P, accum, denom, opacity, scaling,
                       prune_mask, dp, flags, reinterpret_cast<uint4*>(block_counts));
  }
  hipLaunchKernelGGL(k_densify_scan, dim3(1), dim3(1024), 0, s, reinterpret_cast<uint4*>(block_counts), nb);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(WGSR_EHIP, "wgsr_densify_select: %s", hipGetErrorString(e));
  return WGSR_OK;
}

int wgsr_densify_emit(int64_t P, int M, const uint8_t* flags, const uint32_t* block_counts, const float* z,
                      const wgsr_gaussian_bank* src, const wgsr_gaussian_bank* dst, void* stream) {
  if (P < 0 || M < 1 || M > 16 || !src || !dst) return set_error(WGSR_EINVAL, "wgsr_densify_emit: bad arguments");
  if (P == 0) return WGSR_OK;
  if (!flags || !block_counts) return set_error(WGSR_EINVAL, "wgsr_densify_emit: null pointer");
  const wgsr_gaussian_bank* b[2] = {src, dst};
  for (const wgsr_gaussian_bank* x : b) {
    if (!x->xyz || !x->features || !x->opacity || !x->scaling || !x->rotation)
      return set_error(WGSR_EINVAL, "wgsr_densify_emit: missing parameter pointer");
    for (int k = 0; k < 5; ++k)
      if (!x->exp_avg[k] || !x->exp_avg_sq[k]) return set_error(WGSR_EINVAL, "wgsr_densify_emit: missing moment");
  }
  const unsigned nb = den_blocks(P);
  hipLaunchKernelGGL(k_densify_emit, dim3(nb), dim3(kDenBlock), 0, (hipStream_t)stream, P, 3 * M, flags,
                     reinterpret_cast<const uint4*>(block_counts), nb, z, *src, *dst);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(WGSR_EHIP, "wgsr_densify_emit: %s", hipGetErrorString(e));
  return WGSR_OK;
}

int wgsr_reset_opacity(int64_t P, float* opacity_raw, const uint8_t* visible, float value, float* exp_avg,
                       float* exp_avg_sq, void* stream) {
  if (P < 0) return set_error(WGSR_EINVAL, "wgsr_reset_opacity: bad P");
  if (P == 0) return WGSR_OK;
  if (!opacity_raw || !exp_avg || !exp_avg_sq) return set_error(WGSR_EINVAL, "wgsr_reset_opacity: null pointer");
  hipLaunchKernelGGL(k_reset_opacity, dim3(den_blocks(P)), dim3(kDenBlock), 0, (hipStream_t)stream, P, opacity_raw,
                     visible, value, exp_avg, exp_avg_sq);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(WGSR_EHIP, "wgsr_reset_opacity: %s", hipGetErrorString(e));
  return WGSR_OK;
}

}  // extern "C"
