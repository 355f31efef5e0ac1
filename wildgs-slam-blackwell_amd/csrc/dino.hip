// DINO feature-similarity regulariser for gfx950 (SURVEY.md 8(f) row f2,
// the uncertainty branch of the mapping loss).
//
// compute_dino_regularization_loss (src/utils/dyn_uncertainty/
// mapping_utils.py:332-389, NeRF-on-the-Go eqs. 2-3): features are
// L2-normalised (torch.nn.functional.normalize: x / max(|x|, 1e-12)), every
// sample i takes the min(128, N) samples of highest cosine similarity
// (torch.topk over the N x N similarity matrix), keeps those above 0.75 and
// contributes the variance of the uncertainty over them:
//   mean_i = sum_sel u_j / (c_i + eps),  var_i = sum_sel (u_j - mean_i)^2 / (c_i + eps),
//   loss   = mean_i var_i.
// The reference runs it as a GEMM + topk + gathers (~15 torch launches, and
// hipBLASLt picks a 256x256 macro tile for the ~300-sample problem, ~100 us).
// Here: one normalisation kernel, one 32x32-tiled similarity kernel, one
// wave per sample for the selection (the samples above the threshold; when
// more than k, a 32-step radix select of the k-th largest similarity, ties
// taken in index order -- torch.topk leaves their order unspecified), the
// mean/variance and d var_i / d u_j, and one fixed-order reduction of the
// loss.  d loss / d u is accumulated with float atomics (one per selected
// (i, j); the order of those adds is not fixed).
#include <math.h>

#include "wgsr_common.h"
#include "wgsr_internal.h"

namespace wgsr {

namespace {

constexpr int kSimTile = 32;  // similarity tile (rows x columns), 256 threads, 2 x 2 outputs each
constexpr int kSimK = 32;     // feature-dimension chunk staged in LDS

// one wave per row: fn[i] = x[i] / max(||x[i]||, 1e-12)
__global__ __launch_bounds__(256) void k_dino_normalize(const float* __restrict__ x, int N, int C,
                                                        float* __restrict__ fn, float* __restrict__ grad_u) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= N) return;
  if (lane == 0) grad_u[i] = 0.f;  // (k_dino_select adds into it: no memset launch)
  const float* xi = x + (size_t)i * C;
  float ss = 0.f;
  for (int c = lane; c < C; c += 64) ss = fmaf(xi[c], xi[c], ss);
  ss = wave_sum(ss);
  const float d = fmaxf(sqrtf(ss), 1e-12f);
  float* fi = fn + (size_t)i * C;
  for (int c = lane; c < C; c += 64) fi[c] = xi[c] / d;
}

// S = fn fn^T (row-major N x N), 32 x 32 output tiles, feature chunks of 32
// staged in LDS for both operands (padded against bank conflicts)
__global__ __launch_bounds__(256) void k_dino_similarity(const float* __restrict__ fn, int N, int C,
                                                         float* __restrict__ S) {
  __shared__ float sa[kSimTile][kSimK + 1], sb[kSimTile][kSimK + 1];
  const int t = threadIdx.x, tx = t & 15, ty = t >> 4;
  const int i0 = blockIdx.y * kSimTile, j0 = blockIdx.x * kSimTile;
  float acc[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
  for (int k0 = 0; k0 < C; k0 += kSimK) {
    for (int e = t; e < kSimTile * kSimK; e += 256) {
      const int r = e / kSimK, k = e % kSimK;
      const bool kin = k0 + k < C;
      sa[r][k] = (i0 + r < N && kin) ? fn[(size_t)(i0 + r) * C + k0 + k] : 0.f;
      sb[r][k] = (j0 + r < N && kin) ? fn[(size_t)(j0 + r) * C + k0 + k] : 0.f;
    }
    __syncthreads();
#pragma unroll 8
    for (int k = 0; k < kSimK; ++k) {
      const float a0 = sa[2 * ty][k], a1 = sa[2 * ty + 1][k], b0 = sb[2 * tx][k], b1 = sb[2 * tx + 1][k];
      acc[0][0] = fmaf(a0, b0, acc[0][0]);
      acc[0][1] = fmaf(a0, b1, acc[0][1]);
      acc[1][0] = fmaf(a1, b0, acc[1][0]);
      acc[1][1] = fmaf(a1, b1, acc[1][1]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int i = i0 + 2 * ty + a, j = j0 + 2 * tx + b;
      if (i < N && j < N) S[(size_t)i * N + j] = acc[a][b];
    }
}

// The same tiles with both 32-row operand blocks streamed into LDS ONCE, over
// the whole feature dimension (LDS-DMA, 16 B per lane, every load in flight
// at once) instead of 12 dependent chunk rounds, and the products on the f32
// matrix cores: wave w owns the 16 x 16 quarter (w >> 1, w & 1) of the tile,
// v_mfma_f32_16x16x4_f32 step m summing k = 4 m + (lane >> 4) -- a k-ordered
// fmaf chain, so the same products in the same k order as k_dino_similarity:
// bit-identical.  Float4 chunk k4 of row r sits at k4 ^ (r & 15), so the 16
// rows x 4 k of a step's b32 reads land on 64 distinct banks.  C % 64 == 0,
// C <= 384 (96 KB of LDS).  (The VALU form, 2 x 2 outputs per thread from
// b128 reads, ran 13.4 us on the mapper's 303-row sample.)
constexpr int kSim2MaxC = 384;
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_dino_similarity2(const float* __restrict__ fn, int N, int C,
                                                         float* __restrict__ S) {
  extern __shared__ float4 s_sim[];  // [2][32][C / 4]
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int i0 = blockIdx.y * kSimTile, j0 = blockIdx.x * kSimTile, C4 = C >> 2;
  {
    typedef __attribute__((address_space(3))) void* lds_ptr;
    const float4* src = reinterpret_cast<const float4*>(fn);
    const int per_op = kSimTile * C4;  // float4 slots per operand (a multiple of 64 when C % 8 == 0)
    for (int b = 64 * w; b < 2 * per_op; b += 256) {  // (uniform) 64 slots per DMA instruction
      const int sl = b + lane;
      const int op = sl >= per_op, s2 = sl - op * per_op, r = s2 / C4, k4 = s2 - r * C4;
      const int row = min((op ? j0 : i0) + r, N - 1);  // rows past N: a valid row, never stored
      __builtin_amdgcn_global_load_lds((const void*)(src + (size_t)row * C4 + (k4 ^ (r & 15))),
                                       (lds_ptr)(s_sim + b), 16, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);
  }
  __syncthreads();
  const int lr = lane & 15, kh = lane >> 4;
  const int ra = 16 * (w >> 1) + lr, rb = 16 * (w & 1) + lr;  // this lane's A row, B row (= output column)
  const float* const fa = reinterpret_cast<const float*>(s_sim) + (size_t)4 * ra * C4;
  const float* const fb = reinterpret_cast<const float*>(s_sim) + (size_t)4 * (kSimTile + rb) * C4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int m = 0; m < C4; ++m) {
    const int o = 4 * (m ^ lr) + kh;  // (ra & 15 == rb & 15 == lr)
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[o], fb[o], acc, 0, 0, 0);
  }
  const int j = j0 + rb;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = i0 + 16 * (w >> 1) + 4 * kh + q;
    if (i < N && j < N) S[(size_t)i * N + j] = acc[q];
  }
}

// one wave per sample i: the selection, its mean / variance and the
// gradient of var_i / rows w.r.t. every selected u_j
__global__ __launch_bounds__(256) void k_dino_select(const float* __restrict__ S, const float* __restrict__ u, int N,
                                                     int K, float thresh, float eps, float inv_rows,
                                                     float* __restrict__ row_var, float* __restrict__ grad_u) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= N) return;
  const float* si = S + (size_t)i * N;
  const uint32_t tb = __float_as_uint(thresh);  // candidates: s > thresh (> 0: bits order as values)
  // number of candidates
  uint32_t cnt = 0;
  for (int j = lane; j < N; j += 64) cnt += si[j] > thresh ? 1u : 0u;
  cnt = wave_sum_u32(cnt);
  // more candidates than k: the k-th largest similarity (as bits), then ties
  // at it taken in index order up to k
  uint32_t vk = tb;   // select s > vk ...
  uint32_t ties = 0;  // ... and the first `ties` samples with s == vk
  if (cnt > (uint32_t)K) {
    uint32_t prefix = 0;
    for (int bit = 31; bit >= 0; --bit) {
      const uint32_t cand = prefix | (1u << bit);
      uint32_t ge = 0;
      for (int j = lane; j < N; j += 64) {
        const float s = si[j];
        ge += (s > thresh && __float_as_uint(s) >= cand) ? 1u : 0u;
      }
      if (wave_sum_u32(ge) >= (uint32_t)K) prefix = cand;
    }
    // prefix = bits of the k-th largest candidate
    uint32_t gt = 0;
    for (int j = lane; j < N; j += 64) gt += __float_as_uint(si[j]) > prefix && si[j] > thresh ? 1u : 0u;
    gt = wave_sum_u32(gt);
    vk = prefix;
    ties = (uint32_t)K - gt;
  }
  // sample j (similarity s) is selected if s > thresh and, when there are
  // more candidates than k, s > vk or s == vk within the first `ties` such
  // samples in index order (tie rank: equal samples at smaller j)
  const bool over = cnt > (uint32_t)K;
  auto selected = [&](float s, uint32_t tie_rank) -> bool {
    if (!(s > thresh)) return false;
    const uint32_t b = __float_as_uint(s);
    return !over || b > vk || (b == vk && tie_rank < ties);
  };
  // pass 1: count and sum of the selected u; ties resolved per 64-sample chunk
  float su = 0.f;
  uint32_t c = 0, tie_base = 0;
  for (int j0 = 0; j0 < N; j0 += 64) {
    const int j = j0 + lane;
    const float s = j < N ? si[j] : 0.f;
    const bool eq = j < N && over && s > thresh && __float_as_uint(s) == vk;
    const uint64_t em = wave_ballot(eq);
    const bool sel = j < N && selected(s, tie_base + lanes_below(em));
    if (sel) {
      su += u[j];
      c += 1;
    }
    tie_base += (uint32_t)__popcll(em);
  }
  su = wave_sum(su);
  c = wave_sum_u32(c);
  const float cn = (float)c + eps;
  const float mean = su / cn;
  // pass 2: variance and sum of deviations
  float sv = 0.f, sdev = 0.f;
  tie_base = 0;
  for (int j0 = 0; j0 < N; j0 += 64) {
    const int j = j0 + lane;
    const float s = j < N ? si[j] : 0.f;
    const bool eq = j < N && over && s > thresh && __float_as_uint(s) == vk;
    const uint64_t em = wave_ballot(eq);
    if (j < N && selected(s, tie_base + lanes_below(em))) {
      const float d = u[j] - mean;
      sv = fmaf(d, d, sv);
      sdev += d;
    }
    tie_base += (uint32_t)__popcll(em);
  }
  sv = wave_sum(sv);
  sdev = wave_sum(sdev);
  if (lane == 0) row_var[i] = sv / cn;
  // pass 3: d var_i / d u_j = (2 (u_j - mean) - 2 sdev / cn) / cn, times 1 / rows
  const float off = 2.f * sdev / cn;
  tie_base = 0;
  for (int j0 = 0; j0 < N; j0 += 64) {
    const int j = j0 + lane;
    const float s = j < N ? si[j] : 0.f;
    const bool eq = j < N && over && s > thresh && __float_as_uint(s) == vk;
    const uint64_t em = wave_ballot(eq);
    if (j < N && selected(s, tie_base + lanes_below(em))) atomicAdd(&grad_u[j], (2.f * (u[j] - mean) - off) / cn * inv_rows);
    tie_base += (uint32_t)__popcll(em);
  }
}

// loss = mean of row_var, fixed order (one workgroup)
__global__ __launch_bounds__(256) void k_dino_mean(const float* __restrict__ row_var, int N, float* __restrict__ loss) {
  __shared__ float s4[4];
  const int t = threadIdx.x;
  float s = 0.f;
  for (int i = t; i < N; i += 256) s += row_var[i];
  s = wave_sum(s);
  if ((t & 63) == 0) s4[t >> 6] = s;
  __syncthreads();
  if (t == 0) loss[0] = ((s4[0] + s4[1]) + (s4[2] + s4[3])) / (float)N;
}

}  // namespace

}  // namespace wgsr

using namespace wgsr;

extern "C" {

int wgsr_dino_reg(const float* u, const float* feat, int N, int C, int top_k, float thresh, float eps,
                  float* fn_scratch, float* sim_scratch, float* row_var, float* grad_u, float* loss, void* stream) {
  if (N <= 0 || C <= 0 || top_k <= 0 || N > 16384)
    return set_error(WGSR_EINVAL, "wgsr_dino_reg: bad shape N=%d C=%d k=%d", N, C, top_k);
  if (!(thresh > 0.f)) return set_error(WGSR_EINVAL, "wgsr_dino_reg: the threshold must be positive");
  if (!u || !feat || !fn_scratch || !sim_scratch || !row_var || !grad_u)
    return set_error(WGSR_EINVAL, "wgsr_dino_reg: null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int K = top_k < N ? top_k : N;
  const unsigned rows4 = (unsigned)((N + 3) / 4), tiles = (unsigned)((N + kSimTile - 1) / kSimTile);
  hipLaunchKernelGGL(k_dino_normalize, dim3(rows4), dim3(256), 0, s, feat, N, C, fn_scratch, grad_u);
  if (C % 64 == 0 && C <= kSim2MaxC)  // (fn_scratch: a 16-byte aligned caller buffer)
    hipLaunchKernelGGL(k_dino_similarity2, dim3(tiles, tiles), dim3(256), sizeof(float) * 2 * kSimTile * (size_t)C, s,
                       fn_scratch, N, C, sim_scratch);
  else
    hipLaunchKernelGGL(k_dino_similarity, dim3(tiles, tiles), dim3(256), 0, s, fn_scratch, N, C, sim_scratch);
  hipLaunchKernelGGL(k_dino_select, dim3(rows4), dim3(256), 0, s, sim_scratch, u, N, K, thresh, eps,
                     1.f / (float)N, row_var, grad_u);
  if (loss) hipLaunchKernelGGL(k_dino_mean, dim3(1), dim3(256), 0, s, row_var, N, loss);  // (NULL: the gradient only)
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? WGSR_OK : set_error(WGSR_EHIP, "wgsr_dino_reg: %s", hipGetErrorString(e));
}

}  // extern "C"
