// Optimizer step and densification compaction for the Gaussian parameters,
// gfx950 (the work that follows the rasteriser in
// every mapping iteration, gaussian_model.py:271-320 and 526-644).
//
//  * wgsr_adam_step: torch.optim.Adam's update (the reference's optimizer,
//    gaussian_model.py:309, lr per parameter group, eps = 1e-15, no weight
//    decay) for all parameter groups in ONE launch.  torch's foreach Adam
//    makes ~7 elementwise passes over every tensor; here each element's
//    (param, grad, exp_avg, exp_avg_sq) is read once and (param, exp_avg,
//    exp_avg_sq) written once: 28 B per element, HBM bound.
//  * wgsr_compact_rows: prune_points / _prune_optimizer's `t[mask]` over the
//    ~21 per-Gaussian tensors (6 params, 12 Adam states, densification stats)
//    in one scan + one gather launch instead of 21 boolean-index kernels.
#include <algorithm>

#include "wgsr_common.h"
#include "wgsr_internal.h"

namespace wgsr {

namespace {

constexpr int kAdamMax = WGSR_ADAM_MAX_TENSORS;

struct AdamBatch {
  wgsr_adam_tensor t[kAdamMax];
  int64_t ustart[kAdamMax + 1];  // first 4-element unit of each tensor (each starts on a unit)
  int n;
  float beta2, w1, w2, eps;  // w1 = 1 - beta1, w2 = 1 - beta2, rounded from double like torch's scalars
  // wgsr_adam_step_dev: per-tensor (step_size, bias_correction2_sqrt,
  // step_size_tail) from device memory, the skip word, the L2 weight decay
  const float* sc;
  const uint32_t* skip;
  float wd;
  // wgsr_adam_step_dev2: tensors [n1, n) are a second optimiser's (its own
  // eps, weight decay and device scalars, indexed from n1)
  int n1;
  float eps2, wd2;
  const float* sc2;
};

// tensor k's step scalars: its own fields, or the device triple
struct AdamScal {
  float neg_step, neg_tail, bc2s;
};
__device__ __forceinline__ AdamScal adam_scal(const AdamBatch& b, int k) {
  const wgsr_adam_tensor& T = b.t[k];
  if (k >= b.n1) {
    const float* q = b.sc2 + 3 * (k - b.n1);
    return {-q[0], -q[2], q[1]};
  }
  if (b.sc) return {-b.sc[3 * k], -b.sc[3 * k + 2], b.sc[3 * k + 1]};
  return {-T.step_size, -T.step_size_tail, T.bias_correction2_sqrt};
}

// Same arithmetic, in the same order, as torch's _multi_tensor_adam (fp32
// opmath): exp_avg.lerp_(grad, 1 - beta1); exp_avg_sq.mul_(beta2)
// .addcmul_(grad, grad, 1 - beta2); denom = sqrt(exp_avg_sq) / sqrt(bc2) + eps;
// param.addcdiv_(exp_avg, denom, -lr / bc1).
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float w1, float beta2, float w2,
                                          float eps, float neg_step, float bc2_sqrt) {
  m = (w1 < 0.5f) ? m + w1 * (g - m) : g - (g - m) * (1.f - w1);  // lerp
  v = v * beta2;
  v = v + w2 * g * g;
  const float denom = sqrtf(v) / bc2_sqrt + eps;
  p = p + neg_step * (m / denom);
}

// -step size of element e (the optional two-rate split, wgsr.h)
__device__ __forceinline__ float neg_step_of(const wgsr_adam_tensor& T, const AdamScal& S, int64_t e) {
  if (T.split_period <= 0) return S.neg_step;
  const int64_t c = (T.numel < (int64_t)1 << 32) ? (int64_t)((uint32_t)e % (uint32_t)T.split_period) : e % T.split_period;
  return c >= T.split_len ? S.neg_tail : S.neg_step;
}

__device__ __forceinline__ void adam_scalar(const wgsr_adam_tensor& T, const AdamScal& S, int64_t e0, float w1,
                                            float beta2, float w2, float eps, float wd) {
  for (int64_t e = e0; e < min(e0 + 4, T.numel); ++e) {
    float p = T.param[e], m = T.exp_avg[e], v = T.exp_avg_sq[e];
    const float g = wd != 0.f ? fmaf(wd, p, T.grad[e]) : T.grad[e];
    adam_elem(p, g, m, v, w1, beta2, w2, eps, neg_step_of(T, S, e), S.bc2s);
    T.param[e] = p;
    T.exp_avg[e] = m;
    T.exp_avg_sq[e] = v;
  }
}

// Grid-stride over tiles of kU x 256 four-element units of the concatenated
// tensors; thread t owns units tile + j*256 + t (coalesced per j).  All kU
// units' loads are issued before any math so each thread keeps 4 kU
// 16-byte loads in flight.  A unit never straddles two tensors (each tensor
// starts on a unit); ragged tails and unaligned tensors take the scalar path.
constexpr int kAdamU = 2;
__global__ __launch_bounds__(256) void k_adam_multi(AdamBatch b) {
  if (b.skip && *b.skip) return;  // (uniform: the whole grid leaves)
  const int64_t units = b.ustart[b.n];
  const float w1 = b.w1, w2 = b.w2, beta2 = b.beta2;
  for (int64_t tile = (int64_t)blockIdx.x * (256 * kAdamU); tile < units; tile += (int64_t)gridDim.x * (256 * kAdamU)) {
    float4 p[kAdamU], g[kAdamU], m[kAdamU], v[kAdamU];
    int ti[kAdamU];
    int64_t e0[kAdamU];
    bool vec[kAdamU];
#pragma unroll
    for (int j = 0; j < kAdamU; ++j) {
      const int64_t u = tile + j * 256 + threadIdx.x;
      int k = 0;
      while (k + 1 < b.n && u >= b.ustart[k + 1]) ++k;
      ti[j] = k;
      const wgsr_adam_tensor& T = b.t[k];
      e0[j] = 4 * (u - b.ustart[k]);
      vec[j] = u < units && e0[j] + 4 <= T.numel &&
               ((reinterpret_cast<uintptr_t>(T.param) | reinterpret_cast<uintptr_t>(T.grad) |
                 reinterpret_cast<uintptr_t>(T.exp_avg) | reinterpret_cast<uintptr_t>(T.exp_avg_sq)) & 15) == 0;
      if (vec[j]) {
        p[j] = *reinterpret_cast<const float4*>(T.param + e0[j]);
        typedef float f4v __attribute__((ext_vector_type(4)));
        const f4v gv = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(T.grad + e0[j]));
        g[j] = make_float4(gv.x, gv.y, gv.z, gv.w);
        m[j] = *reinterpret_cast<const float4*>(T.exp_avg + e0[j]);
        v[j] = *reinterpret_cast<const float4*>(T.exp_avg_sq + e0[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < kAdamU; ++j) {
      const int64_t u = tile + j * 256 + threadIdx.x;
      if (u >= units) continue;
      const wgsr_adam_tensor& T = b.t[ti[j]];
      const AdamScal S = adam_scal(b, ti[j]);
      const bool second = ti[j] >= b.n1;
      const float eps = second ? b.eps2 : b.eps, wd = second ? b.wd2 : b.wd;
      if (!vec[j]) {
        adam_scalar(T, S, e0[j], w1, beta2, w2, eps, wd);
        continue;
      }
      const float bc2s = S.bc2s;
      float ns[4] = {S.neg_step, S.neg_step, S.neg_step, S.neg_step};
      if (T.split_period > 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) ns[k] = neg_step_of(T, S, e0[j] + k);
      }
      if (wd != 0.f) {
        g[j].x = fmaf(wd, p[j].x, g[j].x);
        g[j].y = fmaf(wd, p[j].y, g[j].y);
        g[j].z = fmaf(wd, p[j].z, g[j].z);
        g[j].w = fmaf(wd, p[j].w, g[j].w);
      }
      adam_elem(p[j].x, g[j].x, m[j].x, v[j].x, w1, beta2, w2, eps, ns[0], bc2s);
      adam_elem(p[j].y, g[j].y, m[j].y, v[j].y, w1, beta2, w2, eps, ns[1], bc2s);
      adam_elem(p[j].z, g[j].z, m[j].z, v[j].z, w1, beta2, w2, eps, ns[2], bc2s);
      adam_elem(p[j].w, g[j].w, m[j].w, v[j].w, w1, beta2, w2, eps, ns[3], bc2s);
      *reinterpret_cast<float4*>(T.param + e0[j]) = p[j];
      *reinterpret_cast<float4*>(T.exp_avg + e0[j]) = m[j];
      *reinterpret_cast<float4*>(T.exp_avg_sq + e0[j]) = v[j];
    }
  }
}

// ---- row compaction ---------------------------------------------------------
constexpr int kCompactRows = 4096;  // rows per workgroup (256 threads x 16)
constexpr int kGatherU = 8;

// keep[r0 .. r0+16) as a bit mask (one 16-B load when aligned and in range)
__device__ __forceinline__ uint32_t keep_flags16(const uint8_t* __restrict__ keep, int64_t P, int64_t r0) {
  uint32_t f = 0;
  if (r0 + 16 <= P && (reinterpret_cast<uintptr_t>(keep) & 15) == 0) {
    const uint4 q = *reinterpret_cast<const uint4*>(keep + r0);
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) f |= ((w[i] >> (8 * j)) & 0xffu) ? (1u << (4 * i + j)) : 0u;
  } else {
    for (int j = 0; j < 16; ++j)
      if (r0 + j < P && keep[r0 + j]) f |= 1u << j;
  }
  return f;
}

// per-block count of kept rows
__global__ __launch_bounds__(256) void k_keep_count(const uint8_t* __restrict__ keep, int64_t P,
                                                    uint32_t* __restrict__ bcount) {
  __shared__ uint32_t s_tmp[4];
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * kCompactRows + (int64_t)t * 16;
  const uint32_t c = wave_sum_u32((uint32_t)__popc(keep_flags16(keep, P, r0)));
  if ((t & 63) == 0) s_tmp[t >> 6] = c;
  __syncthreads();
  if (t == 0) bcount[blockIdx.x] = s_tmp[0] + s_tmp[1] + s_tmp[2] + s_tmp[3];
}

struct RowBatch {
  wgsr_row_tensor t[WGSR_COMPACT_MAX_TENSORS];
  int n;
};

// Block (x, y) lists the kept rows of row block x (in order) in LDS, then
// copies tensor y's kept rows to the block's contiguous output range word by
// word (coalesced stores; reads follow the kept rows).
__global__ __launch_bounds__(256) void k_compact_gather(const uint8_t* __restrict__ keep, int64_t P,
                                                        const uint32_t* __restrict__ bbase, RowBatch b) {
  __shared__ uint16_t s_rows[kCompactRows];
  __shared__ uint32_t s_wsum[4];
  const int t = threadIdx.x, w = t >> 6;
  const int64_t blk0 = (int64_t)blockIdx.x * kCompactRows;
  const int64_t r0 = blk0 + (int64_t)t * 16;
  const uint32_t flags = keep_flags16(keep, P, r0);
  const uint32_t c = (uint32_t)__popc(flags);
  const uint32_t inc = wave_incl_scan(c);
  if ((t & 63) == 63) s_wsum[w] = inc;
  __syncthreads();
  uint32_t off = inc - c;
  for (int i = 0; i < w; ++i) off += s_wsum[i];
  const uint32_t total = s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
#pragma unroll
  for (int j = 0; j < 16; ++j)
    if (flags & (1u << j)) s_rows[off++] = (uint16_t)(t * 16 + j);
  __syncthreads();
  const int64_t out0 = bbase[blockIdx.x];
  {  // one tensor per grid row: blocks x tensors workgroups fill the chip
    const wgsr_row_tensor& T = b.t[blockIdx.y];
    const uint32_t wpr = (uint32_t)(T.row_bytes / 4);  // 32-bit words per row
    const uint32_t* src = static_cast<const uint32_t*>(T.src) + blk0 * wpr;
    uint32_t* dst = static_cast<uint32_t*>(T.dst) + out0 * wpr;
    const uint32_t words = total * wpr;  // <= 4096 rows x row words: 32-bit index math
    const float inv_wpr = 1.f / (float)wpr;
    // kGatherU independent loads in flight per thread before the stores
    for (uint32_t k0 = t; k0 < words; k0 += 256 * kGatherU) {
      uint32_t val[kGatherU];
#pragma unroll
      for (int j = 0; j < kGatherU; ++j) {
        const uint32_t k = k0 + 256 * j;
        if (k < words) {
          // k < 2^24: the float quotient is within one of k / wpr
          uint32_t row = (uint32_t)((float)k * inv_wpr);
          if (row * wpr > k) --row;
          else if ((row + 1) * wpr <= k) ++row;
          val[j] = src[(uint32_t)s_rows[row] * wpr + (k - row * wpr)];
        }
      }
#pragma unroll
      for (int j = 0; j < kGatherU; ++j)
        if (k0 + 256 * j < words) dst[k0 + 256 * j] = val[j];
    }
  }
}

// ---- the graph-replayed mapping iteration's small steps (wgsr/online_graph.py) --
constexpr int kGatherMax = WGSR_GATHER_MAX_JOBS;
struct GatherBatch {
  wgsr_gather_job j[kGatherMax];
  int64_t ustart[kGatherMax + 1];  // first unit of each job (units: 4 words when vec, else 1)
  bool vec[kGatherMax];
  int n;
  const int64_t* idx;
};
// dst rows r of job k = src row idx[idx_offset + r] (every job in one launch)
__global__ __launch_bounds__(256) void k_gather_rows(GatherBatch b) {
  const int64_t units = b.ustart[b.n];
  for (int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x; u < units; u += (int64_t)gridDim.x * 256) {
    int k = 0;
    while (k + 1 < b.n && u >= b.ustart[k + 1]) ++k;
    const wgsr_gather_job& J = b.j[k];
    const int64_t v = u - b.ustart[k];
    if (b.vec[k]) {
      const int64_t per = J.row_words / 4, r = v / per, c = v - r * per;
      const int64_t sr = b.idx[J.idx_offset + r];
      reinterpret_cast<uint4*>(J.dst)[r * per + c] =
          reinterpret_cast<const uint4*>(J.src)[sr * (J.src_stride_words / 4) + c];
    } else {
      const int64_t r = v / J.row_words, c = v - r * J.row_words;
      const int64_t sr = b.idx[J.idx_offset + r];
      static_cast<uint32_t*>(J.dst)[r * J.row_words + c] =
          static_cast<const uint32_t*>(J.src)[sr * J.src_stride_words + c];
    }
  }
}

// One keyframe exposure step on its bank row (Adam, torch arithmetic as
// k_adam_multi) unless either skip word is set, plus the overflow
// bookkeeping of the capacity-mode forward: sticky[0] += counts[3],
// sticky[1] = max(sticky[1], counts[0]).
// The gradient is the sum of nparts (a, b) rows (the loss backward's
// per-block partials), added in a fixed order: lane l sums rows l, l + 64,
// ..., then a butterfly over the wave.
__global__ __launch_bounds__(64) void k_exposure_step(float* __restrict__ bank, const int64_t* __restrict__ idx,
                                                      const float* __restrict__ grad, int nparts,
                                                      const float* __restrict__ sc,
                                                      const uint32_t* __restrict__ skip_a,
                                                      const uint32_t* __restrict__ skip_b, float w1, float beta2,
                                                      float w2, float eps, long long* __restrict__ sticky,
                                                      const uint32_t* __restrict__ counts,
                                                      long long* __restrict__ slot_skips) {
  const int l = threadIdx.x;
  float ga = 0.f, gb = 0.f;
  if (nparts == 1) {
    ga = grad[0];
    gb = grad[1];
  } else {
    for (int r = l; r < nparts; r += 64) {
      ga += grad[2 * r];
      gb += grad[2 * r + 1];
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      ga += __shfl_xor(ga, off, 64);
      gb += __shfl_xor(gb, off, 64);
    }
  }
  if (l < 2 && !(*skip_a | *skip_b)) {
    float* row = bank + 6 * idx[0];  // (a, b), exp_avg (a, b), exp_avg_sq (a, b)
    float p = row[l], m = row[2 + l], v = row[4 + l];
    adam_elem(p, l == 0 ? ga : gb, m, v, w1, beta2, w2, eps, -sc[0], sc[1]);
    row[l] = p;
    row[2 + l] = m;
    row[4 + l] = v;
  }
  if (l == 0 && sticky && counts) {
    sticky[0] += (long long)counts[3];
    sticky[1] = max(sticky[1], (long long)counts[0]);
  }
  // a step the host counted (skip_b clear) that the overflow word held back
  if (l == 0 && slot_skips && *skip_a && !*skip_b) slot_skips[idx[0]] += 1;
}

}  // namespace

}  // namespace wgsr

using namespace wgsr;

extern "C" {

static int adam_step_impl(const wgsr_adam_tensor* tensors, int n, double beta1, double beta2, double eps, double wd,
                          const float* scalars, const uint32_t* skip, void* stream, int n1 = -1, double eps2 = 0.0,
                          double wd2 = 0.0, const float* scalars2 = nullptr) {
  if (n < 0 || n > kAdamMax || (n > 0 && !tensors)) return set_error(WGSR_EINVAL, "wgsr_adam_step: 0..%d tensors", kAdamMax);
  AdamBatch b{};
  b.sc = scalars;
  b.skip = skip;
  b.wd = (float)wd;
  b.n = n;
  b.n1 = n1 < 0 ? n : n1;
  b.eps2 = (float)eps2;
  b.wd2 = (float)wd2;
  b.sc2 = scalars2;
  b.beta2 = (float)beta2;
  b.w1 = (float)(1.0 - beta1);
  b.w2 = (float)(1.0 - beta2);
  b.eps = (float)eps;
  b.ustart[0] = 0;
  for (int i = 0; i < n; ++i) {
    b.t[i] = tensors[i];
    if (b.t[i].numel < 0 || (b.t[i].numel > 0 && (!b.t[i].param || !b.t[i].grad || !b.t[i].exp_avg ||
                                                   !b.t[i].exp_avg_sq)))
      return set_error(WGSR_EINVAL, "wgsr_adam_step: tensor %d has null pointers", i);
    b.ustart[i + 1] = b.ustart[i] + (b.t[i].numel + 3) / 4;
  }
  const int64_t units = b.ustart[n];
  if (units == 0) return WGSR_OK;
  const int64_t blocks = std::min<int64_t>((units + 256 * kAdamU - 1) / (256 * kAdamU), 256 * 16);
  hipLaunchKernelGGL(k_adam_multi, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, b);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? WGSR_OK : set_error(WGSR_EHIP, "wgsr_adam_step: %s", hipGetErrorString(e));
}

int wgsr_adam_step(const wgsr_adam_tensor* tensors, int n, double beta1, double beta2, double eps, void* stream) {
  return adam_step_impl(tensors, n, beta1, beta2, eps, 0.0, nullptr, nullptr, stream);
}

int wgsr_adam_step_dev(const wgsr_adam_tensor* tensors, int n, double beta1, double beta2, double eps,
                       double weight_decay, const float* scalars, const uint32_t* skip, void* stream) {
  if (!scalars) return set_error(WGSR_EINVAL, "wgsr_adam_step_dev: missing device scalars");
  return adam_step_impl(tensors, n, beta1, beta2, eps, weight_decay, scalars, skip, stream);
}

int wgsr_adam_step_dev2(const wgsr_adam_tensor* tensors, int n1, int n, double beta1, double beta2, double eps1,
                        double weight_decay1, const float* scalars1, double eps2, double weight_decay2,
                        const float* scalars2, const uint32_t* skip, void* stream) {
  if (!scalars1 || (n > n1 && !scalars2) || n1 < 0 || n1 > n)
    return set_error(WGSR_EINVAL, "wgsr_adam_step_dev2: 0 <= n1 <= n and device scalars for both groups");
  return adam_step_impl(tensors, n, beta1, beta2, eps1, weight_decay1, scalars1, skip, stream, n1, eps2,
                        weight_decay2, scalars2);
}

int wgsr_gather_rows(const wgsr_gather_job* jobs, int n, const int64_t* idx, void* stream) {
  if (n < 0 || n > kGatherMax || (n > 0 && (!jobs || !idx)))
    return set_error(WGSR_EINVAL, "wgsr_gather_rows: 0..%d jobs and an index array", kGatherMax);
  GatherBatch b{};
  b.n = n;
  b.idx = idx;
  b.ustart[0] = 0;
  for (int k = 0; k < n; ++k) {
    const wgsr_gather_job& J = jobs[k];
    if (J.nrows < 0 || J.row_words < 0 || J.src_stride_words < J.row_words || J.idx_offset < 0 ||
        (J.nrows > 0 && J.row_words > 0 && (!J.src || !J.dst)))
      return set_error(WGSR_EINVAL, "wgsr_gather_rows: job %d is malformed", k);
    b.j[k] = J;
    b.vec[k] = J.row_words % 4 == 0 && J.src_stride_words % 4 == 0 &&
               ((reinterpret_cast<uintptr_t>(J.src) | reinterpret_cast<uintptr_t>(J.dst)) & 15) == 0;
    b.ustart[k + 1] = b.ustart[k] + (int64_t)J.nrows * (b.vec[k] ? J.row_words / 4 : J.row_words);
  }
  const int64_t units = b.ustart[n];
  if (units == 0) return WGSR_OK;
  const int64_t blocks = std::min<int64_t>((units + 255) / 256, 4096);
  hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, b);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? WGSR_OK : set_error(WGSR_EHIP, "wgsr_gather_rows: %s", hipGetErrorString(e));
}

int wgsr_exposure_step(float* bank, const int64_t* idx, const float* grad, int nparts, const float* scalars,
                       const uint32_t* skip_a, const uint32_t* skip_b, double beta1, double beta2, double eps,
                       int64_t* sticky, const uint32_t* counts, int64_t* slot_skips, void* stream) {
  if (!bank || !idx || !grad || !scalars || !skip_a || !skip_b || nparts < 1)
    return set_error(WGSR_EINVAL, "wgsr_exposure_step: null pointer or no gradient rows");
  hipLaunchKernelGGL(k_exposure_step, dim3(1), dim3(64), 0, (hipStream_t)stream, bank, idx, grad, nparts, scalars, skip_a,
                     skip_b, (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)eps,
                     reinterpret_cast<long long*>(sticky), counts, reinterpret_cast<long long*>(slot_skips));
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? WGSR_OK : set_error(WGSR_EHIP, "wgsr_exposure_step: %s", hipGetErrorString(e));
}

int wgsr_compact_rows(const uint8_t* keep, int64_t P, const wgsr_row_tensor* tensors, int n,
                      wgsr_alloc_fn scratch_alloc, void* ctx, void* stream) {
  if (P < 0 || n < 0 || n > WGSR_COMPACT_MAX_TENSORS) return set_error(WGSR_EINVAL, "wgsr_compact_rows: bad sizes");
  if (P == 0 || n == 0) return WGSR_OK;
  if (!keep) return set_error(WGSR_EINVAL, "wgsr_compact_rows: null keep mask");
  RowBatch b{};
  b.n = n;
  for (int i = 0; i < n; ++i) {
    b.t[i] = tensors[i];
    if (b.t[i].row_bytes <= 0 || (b.t[i].row_bytes & 3) || !b.t[i].src || !b.t[i].dst)
      return set_error(WGSR_EINVAL, "wgsr_compact_rows: tensor %d needs a positive multiple-of-4 row size", i);
  }
  hipStream_t s = (hipStream_t)stream;
  const uint32_t nb = (uint32_t)((P + kCompactRows - 1) / kCompactRows);
  void* scratch = scratch_alloc(ctx, align256(4 * (size_t)(nb + 1)) + 256);
  if (!scratch) return set_error(WGSR_EALLOC, "wgsr_compact_rows: scratch allocation failed");
  uint32_t* bcount = static_cast<uint32_t*>(scratch);
  hipLaunchKernelGGL(k_keep_count, dim3(nb), dim3(256), 0, s, keep, P, bcount);
  // exclusive scan of the block counts in place (one workgroup)
  hipError_t e = exclusive_scan_gather(bcount, nullptr, nb, bcount, nullptr,
                                       at<uint32_t>(scratch, align256(4 * (size_t)(nb + 1))), nullptr, s);
  if (e != hipSuccess) return set_error(WGSR_EHIP, "wgsr_compact_rows: %s", hipGetErrorString(e));
  hipLaunchKernelGGL(k_compact_gather, dim3(nb, (unsigned)n), dim3(256), 0, s, keep, P, bcount, b);
  e = hipGetLastError();
  return e == hipSuccess ? WGSR_OK : set_error(WGSR_EHIP, "wgsr_compact_rows: %s", hipGetErrorString(e));
}

}  // extern "C"
