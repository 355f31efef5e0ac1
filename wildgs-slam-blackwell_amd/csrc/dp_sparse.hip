// Sparse view-sharded exchange for gfx950 (wgsr/dp.py).
//
// In a view's backward most visible Gaussians receive NO gradient: every
// pixel that reaches them has already hit its last contributor (the bench
// scene: 7.5 % of 1M Gaussians per 1080p view, 10.6 % over 8 views;
// profiles/r01/grad_sparsity.json).  Their screen-space records are exactly
// zero and so are their parameter-gradient rows.  These kernels let
// ViewShardedBackward move only the non-zero rows with plain collectives
// (all_gather_into_tensor of equal blocks, all_to_all_single with split
// sizes) and ONE host read of counts per step:
//
//   pack_records      per owner segment [o S, (o+1) S) of a view's records, the
//                     rows with a non-zero partial sum, compacted to the front
//                     of the segment (wave-aggregated atomics; field 10 carries
//                     the row's index inside the segment instead of the
//                     radius), plus a bit per row in the owner's mask words
//   exchange_summary  after the small all-gather of every rank's [camera row |
//                     rows sent per owner | non-zero row masks]: the count
//                     matrix, every owner's UNION row count (the owner's
//                     gradient rows, known before the owners compute them),
//                     the receive offsets of this rank and the camera table
//   unpack_records    the owner scatters every view's received rows back into
//                     its dense [views, S, 12] record table and marks them in a
//                     row mask (the union over views)
//   fill_radius       with densification statistics, the (dense) radius column
//   pack_grads        the owner's gradient rows of the masked Gaussians, one
//                     packed row each: [index, dmean3D(3), dsh(3M), dopacity,
//                     dscale(3), drot(4)]
//   unpack_grads      every rank scatters the gathered packed rows of the other
//                     owners into its (zeroed) gradient tensors
//
// Row order inside a packed segment depends on atomic timing; every consumer
// scatters by index, so the results are bitwise independent of it.
#include "wgsr_common.h"
#include "wgsr_internal.h"

namespace wgsr {

namespace {

constexpr int kSpBlock = 256;

// Wave-aggregated slot allocation: lanes with `take` set get consecutive
// slots of counter[key]; lanes of one wave may carry different keys.
__device__ __forceinline__ uint32_t wave_alloc(bool take, uint32_t key, uint32_t* counter) {
  uint64_t pending = wave_ballot(take);
  uint32_t slot = 0;
  const uint64_t below = (1ull << __lane_id()) - 1ull;
  while (pending) {
    const int leader = __builtin_ctzll(pending);
    const uint32_t k = (uint32_t)__shfl((int)key, leader, 64);
    const uint64_t grp = wave_ballot(take && key == k);
    uint32_t base = 0;
    if (__lane_id() == leader) base = atomicAdd(&counter[k], (uint32_t)__popcll(grp));
    base = (uint32_t)__shfl((int)base, leader, 64);
    if (take && key == k) slot = base + (uint32_t)__popcll(grp & below);
    pending &= ~grp;
  }
  return slot;
}

__global__ __launch_bounds__(kSpBlock) void k_pack_records(const float4* __restrict__ rec, int64_t P_pad, int64_t S,
                                                           uint32_t* __restrict__ counts,
                                                           float4* __restrict__ packed,
                                                           uint32_t* __restrict__ nzmask, int64_t W32) {
  const int64_t i = (int64_t)blockIdx.x * kSpBlock + threadIdx.x;
  float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f), r1 = r0, r2 = r0;
  const bool in = i < P_pad;
  if (in) {
    r0 = rec[3 * i];
    r1 = rec[3 * i + 1];
    r2 = rec[3 * i + 2];
  }
  const bool nz = in && (r0.x != 0.f || r0.y != 0.f || r0.z != 0.f || r0.w != 0.f || r1.x != 0.f || r1.y != 0.f ||
                         r1.z != 0.f || r1.w != 0.f || r2.x != 0.f || r2.y != 0.f);
  const uint32_t o = in ? (uint32_t)(i / S) : 0u;
  const uint32_t slot = wave_alloc(nz, o, counts);
  if (nz) {
    const int64_t j = i - (int64_t)o * S;
    const int64_t k = (int64_t)o * S + slot;
    packed[3 * k] = r0;
    packed[3 * k + 1] = r1;
    packed[3 * k + 2] = make_float4(r2.x, r2.y, __uint_as_float((uint32_t)j), r2.w);
    if (nzmask) atomicOr(&nzmask[(int64_t)o * W32 + (j >> 5)], 1u << (j & 31));
  }
}

// blocks [world][block_words] (uint32): [camera row (kCamFloats) | rows sent to
// each owner (world) | non-zero row mask per owner (world x W32)].  Workgroup
// o: owner o's union row count (popcount of the OR over views); workgroup 0
// also writes the count matrix, this rank's receive offsets and the cameras.
constexpr int kCamFloats = WGSR_VIEW_CAMERA_FLOATS;
__global__ __launch_bounds__(kSpBlock) void k_exchange_summary(const uint32_t* __restrict__ blocks, int world,
                                                               int rank, int64_t W32, int64_t block_words,
                                                               uint32_t* __restrict__ summary,
                                                               uint32_t* __restrict__ offsets,
                                                               float* __restrict__ cams) {
  __shared__ uint32_t s_red[kSpBlock / 64];
  const int o = blockIdx.x, t = threadIdx.x;
  const int64_t mask0 = kCamFloats + world + (int64_t)o * W32;
  uint32_t c = 0;
  for (int64_t w = t; w < W32; w += kSpBlock) {
    uint32_t acc = 0;
    for (int v = 0; v < world; ++v) acc |= blocks[(int64_t)v * block_words + mask0 + w];
    c += (uint32_t)__popc(acc);
  }
  for (int off = 32; off > 0; off >>= 1) c += (uint32_t)__shfl_xor((int)c, off, 64);
  if ((t & 63) == 0) s_red[t >> 6] = c;
  __syncthreads();
  if (t == 0) {
    uint32_t tot = 0;
    for (int k = 0; k < kSpBlock / 64; ++k) tot += s_red[k];
    summary[(int64_t)world * world + o] = tot;
  }
  if (o != 0) return;
  for (int idx = t; idx < world * world; idx += kSpBlock)
    summary[idx] = blocks[(int64_t)(idx / world) * block_words + kCamFloats + idx % world];
  for (int idx = t; idx < world * kCamFloats; idx += kSpBlock)
    cams[idx] = __uint_as_float(blocks[(int64_t)(idx / kCamFloats) * block_words + idx % kCamFloats]);
  if (t == 0) {
    uint32_t run = 0;
    for (int v = 0; v < world; ++v) {
      offsets[v] = run;
      run += blocks[(int64_t)v * block_words + kCamFloats + rank];
    }
    offsets[world] = run;
  }
}

// received: view v's packed rows at [offsets[v], offsets[v + 1]) (contiguous,
// the all_to_all_single output).
__global__ __launch_bounds__(kSpBlock) void k_unpack_records(const float4* __restrict__ recvp,
                                                             const uint32_t* __restrict__ offsets, int64_t S,
                                                             int keep_radius, float4* __restrict__ dense,
                                                             uint8_t* __restrict__ mask) {
  const int v = blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * kSpBlock + threadIdx.x;
  const uint32_t b = offsets[v], e = offsets[v + 1];
  if (j >= (int64_t)(e - b)) return;
  const float4* src = recvp + 3 * ((int64_t)b + j);
  const float4 r0 = src[0], r1 = src[1], r2 = src[2];
  const uint32_t idx = __float_as_uint(r2.z);
  if (idx >= (uint64_t)S) return;  // never produced by k_pack_records
  float4* dst = dense + 3 * ((int64_t)v * S + idx);
  // the owner kernel reads the radius field only as "visible" (> 0) and for
  // the statistics; without statistics any positive value will do
  const float rad = keep_radius ? dst[2].z : 1.f;
  dst[0] = r0;
  dst[1] = r1;
  dst[2] = make_float4(r2.x, r2.y, rad, r2.w);
  mask[idx] = 1;
}

__global__ __launch_bounds__(kSpBlock) void k_fill_radius(const float* __restrict__ radii, int64_t n,
                                                          float4* __restrict__ dense) {
  const int64_t j = (int64_t)blockIdx.x * kSpBlock + threadIdx.x;
  if (j < n) dense[3 * j + 2].z = radii[j];
}

__global__ __launch_bounds__(kSpBlock) void k_pack_grads(int64_t lo, int64_t hi, int M,
                                                         const uint8_t* __restrict__ mask,
                                                         const float* __restrict__ m3d, const float* __restrict__ sh,
                                                         const float* __restrict__ opac, const float* __restrict__ sc,
                                                         const float* __restrict__ rot, uint32_t* __restrict__ count,
                                                         float* __restrict__ packed) {
  const int64_t j = (int64_t)blockIdx.x * kSpBlock + threadIdx.x;  // row inside the shard
  const bool take = lo + j < hi && mask[j];
  const uint32_t slot = wave_alloc(take, 0u, count);
  if (!take) return;
  const int F = 12 + 3 * M;
  const int64_t i = lo + j;
  float* d = packed + (int64_t)slot * F;
  d[0] = __uint_as_float((uint32_t)j);
  for (int k = 0; k < 3; ++k) d[1 + k] = m3d[3 * i + k];
  for (int k = 0; k < 3 * M; ++k) d[4 + k] = sh[3 * M * i + k];
  d[4 + 3 * M] = opac[i];
  for (int k = 0; k < 3; ++k) d[5 + 3 * M + k] = sc[3 * i + k];
  for (int k = 0; k < 4; ++k) d[8 + 3 * M + k] = rot[4 * i + k];
}

// gathered: owner r's rows at gathered + r block_stride (counts[r] rows of F
// floats, at most cap), indices into shard r.  clear: write zeros at those
// rows instead (undoing an earlier step's scatter).
__global__ __launch_bounds__(kSpBlock) void k_unpack_grads(const float* __restrict__ gathered, int64_t block_stride,
                                                           const uint32_t* __restrict__ counts, int rank,
                                                           int64_t cap, int64_t S, int64_t P, int M, int clear,
                                                           float* __restrict__ m3d, float* __restrict__ sh,
                                                           float* __restrict__ opac, float* __restrict__ sc,
                                                           float* __restrict__ rot) {
  const int r = blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * kSpBlock + threadIdx.x;
  if (r == rank || j >= (int64_t)min((uint32_t)cap, counts[r])) return;
  const int F = 12 + 3 * M;
  const float* s = gathered + (int64_t)r * block_stride + j * F;
  const uint32_t idx = __float_as_uint(s[0]);
  const int64_t i = (int64_t)r * S + idx;
  if (idx >= (uint64_t)S || i >= P) return;  // padding rows are never packed; guard anyway
  const float keep = clear ? 0.f : 1.f;  // (x * 0 would keep NaN / inf)
  auto val = [&](int k) { return keep != 0.f ? s[k] : 0.f; };
  for (int k = 0; k < 3; ++k) m3d[3 * i + k] = val(1 + k);
  for (int k = 0; k < 3 * M; ++k) sh[3 * M * i + k] = val(4 + k);
  opac[i] = val(4 + 3 * M);
  for (int k = 0; k < 3; ++k) sc[3 * i + k] = val(5 + 3 * M + k);
  for (int k = 0; k < 4; ++k) rot[4 * i + k] = val(8 + 3 * M + k);
}

inline unsigned blocks_for(int64_t n) { return (unsigned)((n + kSpBlock - 1) / kSpBlock); }

}  // namespace

}  // namespace wgsr

using namespace wgsr;

#define SPCHK(name)                                                                          \
  do {                                                                                       \
    const hipError_t _e = hipGetLastError();                                                 \
    if (_e != hipSuccess) return set_error(WGSR_EHIP, "%s: %s", name, hipGetErrorString(_e)); \
  } while (0)

extern "C" {

int wgsr_sparse_grad_row_floats(int M) { return M >= 0 ? 12 + 3 * M : -1; }

int64_t wgsr_sparse_mask_words(int64_t S) { return S > 0 ? (S + 31) / 32 : 0; }

int wgsr_sparse_pack_records(const float* records, int64_t P_pad, int64_t S, uint32_t* counts, float* packed,
                             uint32_t* nzmask, void* stream) {
  if (P_pad < 0 || S <= 0 || P_pad % S != 0) return set_error(WGSR_EINVAL, "wgsr_sparse_pack_records: bad P_pad / S");
  if (P_pad == 0) return WGSR_OK;
  if (!records || !counts || !packed) return set_error(WGSR_EINVAL, "wgsr_sparse_pack_records: null pointer");
  hipLaunchKernelGGL(k_pack_records, dim3(blocks_for(P_pad)), dim3(kSpBlock), 0, (hipStream_t)stream,
                     reinterpret_cast<const float4*>(records), P_pad, S, counts, reinterpret_cast<float4*>(packed),
                     nzmask, wgsr_sparse_mask_words(S));
  SPCHK("wgsr_sparse_pack_records");
  return WGSR_OK;
}

int64_t wgsr_sparse_summary_block_words(int world, int64_t S) {
  return world > 0 && S >= 0 ? WGSR_VIEW_CAMERA_FLOATS + world + (int64_t)world * wgsr_sparse_mask_words(S) : -1;
}

int wgsr_sparse_exchange_summary(const uint32_t* blocks, int world, int rank, int64_t S, uint32_t* summary,
                                 uint32_t* offsets, float* cams, void* stream) {
  if (world < 1 || world > 65535 || rank < 0 || rank >= world || S <= 0)
    return set_error(WGSR_EINVAL, "wgsr_sparse_exchange_summary: bad arguments");
  if (!blocks || !summary || !offsets || !cams) return set_error(WGSR_EINVAL, "wgsr_sparse_exchange_summary: null pointer");
  hipLaunchKernelGGL(k_exchange_summary, dim3(world), dim3(kSpBlock), 0, (hipStream_t)stream, blocks, world, rank,
                     wgsr_sparse_mask_words(S), wgsr_sparse_summary_block_words(world, S), summary, offsets, cams);
  SPCHK("wgsr_sparse_exchange_summary");
  return WGSR_OK;
}

int wgsr_sparse_unpack_records(const float* received, const uint32_t* offsets, int n_views, int64_t S,
                               int keep_radius, float* records, uint8_t* mask, void* stream) {
  if (n_views < 0 || n_views > 65535 || S < 0) return set_error(WGSR_EINVAL, "wgsr_sparse_unpack_records: bad sizes");
  if (n_views == 0 || S == 0) return WGSR_OK;
  if (!received || !offsets || !records || !mask)
    return set_error(WGSR_EINVAL, "wgsr_sparse_unpack_records: null pointer");
  hipLaunchKernelGGL(k_unpack_records, dim3(blocks_for(S), n_views), dim3(kSpBlock), 0, (hipStream_t)stream,
                     reinterpret_cast<const float4*>(received), offsets, S, keep_radius,
                     reinterpret_cast<float4*>(records), mask);
  SPCHK("wgsr_sparse_unpack_records");
  return WGSR_OK;
}

int wgsr_sparse_fill_radius(const float* radii, int64_t n, float* records, void* stream) {
  if (n < 0) return set_error(WGSR_EINVAL, "wgsr_sparse_fill_radius: negative size");
  if (n == 0) return WGSR_OK;
  if (!radii || !records) return set_error(WGSR_EINVAL, "wgsr_sparse_fill_radius: null pointer");
  hipLaunchKernelGGL(k_fill_radius, dim3(blocks_for(n)), dim3(kSpBlock), 0, (hipStream_t)stream, radii, n,
                     reinterpret_cast<float4*>(records));
  SPCHK("wgsr_sparse_fill_radius");
  return WGSR_OK;
}

int wgsr_sparse_pack_grads(int64_t lo, int64_t hi, int M, const uint8_t* mask, const float* dL_dmeans3D,
                           const float* dL_dsh, const float* dL_dopacity, const float* dL_dscales,
                           const float* dL_drotations, uint32_t* count, float* packed, void* stream) {
  if (lo < 0 || hi < lo || M < 1 || M > 16) return set_error(WGSR_EINVAL, "wgsr_sparse_pack_grads: bad arguments");
  if (hi == lo) return WGSR_OK;
  if (!mask || !dL_dmeans3D || !dL_dsh || !dL_dopacity || !dL_dscales || !dL_drotations || !count || !packed)
    return set_error(WGSR_EINVAL, "wgsr_sparse_pack_grads: null pointer");
  hipLaunchKernelGGL(k_pack_grads, dim3(blocks_for(hi - lo)), dim3(kSpBlock), 0, (hipStream_t)stream, lo, hi, M, mask,
                     dL_dmeans3D, dL_dsh, dL_dopacity, dL_dscales, dL_drotations, count, packed);
  SPCHK("wgsr_sparse_pack_grads");
  return WGSR_OK;
}

int wgsr_sparse_unpack_grads(const float* gathered, int64_t block_stride, const uint32_t* counts, int world, int rank,
                             int64_t cap, int64_t S, int64_t P, int M, float* dL_dmeans3D, float* dL_dsh,
                             float* dL_dopacity, float* dL_dscales, float* dL_drotations, int clear, void* stream) {
  if (world < 1 || world > 65535 || rank < 0 || rank >= world || cap < 0 || S < 0 || P < 0 || M < 1 || M > 16 ||
      block_stride < cap * (12 + 3 * M))
    return set_error(WGSR_EINVAL, "wgsr_sparse_unpack_grads: bad arguments");
  if (cap == 0) return WGSR_OK;
  if (!gathered || !counts || !dL_dmeans3D || !dL_dsh || !dL_dopacity || !dL_dscales || !dL_drotations)
    return set_error(WGSR_EINVAL, "wgsr_sparse_unpack_grads: null pointer");
  hipLaunchKernelGGL(k_unpack_grads, dim3(blocks_for(cap), world), dim3(kSpBlock), 0, (hipStream_t)stream, gathered,
                     block_stride, counts, rank, cap, S, P, M, clear, dL_dmeans3D, dL_dsh, dL_dopacity, dL_dscales,
                     dL_drotations);
  SPCHK("wgsr_sparse_unpack_grads");
  return WGSR_OK;
}

}  // extern "C"
