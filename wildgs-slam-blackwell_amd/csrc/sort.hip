// Stable LSD radix sort of (u32 key, u32 value) pairs and exclusive scans, gfx950.
//
// Replaces the CUB primitives upstream's rasteriser and simple-knn lean on
// (cub::DeviceRadixSort::SortPairs, cub::DeviceScan::InclusiveSum: SURVEY.md
// 2 "Kernel inventory").  8-bit digits; a workgroup owns 4096 keys (2048 for
// sorts of <= 2M keys, so a per-Gaussian pass still fills the chip).
// Reduce-then-scan: per pass, block histograms (which also add into 16-block
// superblock sums) -> stable scatter whose blocks derive their digit bases
// from the superblock sums.  (A decoupled look-back "onesweep" schedule
// measured 1.3-2x slower here -- look-back chains through ~700 resident
// blocks -- and was removed in round 5.)
// Block-local stable ranking uses 64-bit ballots to find the lanes that share
// a digit; the scatter stages the block's keys in LDS in digit order so that
// runs of one digit leave as contiguous (coalesced) stores.  Each wave of the
// scatter owns a contiguous run of 64 I keys that it walks 64 at a time, so
// ranks follow input order.
#include <stdlib.h>
#include <string.h>

#include "wgsr_common.h"
#include "wgsr_internal.h"

namespace wgsr {

namespace {

// exclusive scan of one value per thread over a 256-thread block
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* s_tmp4, uint32_t* total) {
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  uint32_t inc = wave_incl_scan(v);
  if (lane == 63) s_tmp4[w] = inc;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint32_t x = s_tmp4[i];
    base += (i < w) ? x : 0u;
    tot += x;
  }
  __syncthreads();
  if (total) *total = tot;
  return base + inc - v;
}

// ---- digit counting ----------------------------------------------------------
// Histogram kernels give thread t of a block the I CONTIGUOUS keys
// [I t, I t + I) of the block's 256 I and count them one LDS atomic per run
// of equal digits: the sort inputs here (depth bits, tile ids in duplicate
// order, Morton codes) have long runs in their high digits, which would
// otherwise serialise as same-address LDS atomics.

template <int I>
__device__ __forceinline__ int load_run(const uint32_t* __restrict__ keys, size_t n, size_t e0, uint32_t (&k)[I]) {
  static_assert(I % 4 == 0, "load_run reads uint4s");
  if (e0 + I <= n) {
    const uint4* p = reinterpret_cast<const uint4*>(keys + e0);
#pragma unroll
    for (int q = 0; q < I / 4; ++q) {
      const uint4 v = p[q];
      k[4 * q] = v.x; k[4 * q + 1] = v.y; k[4 * q + 2] = v.z; k[4 * q + 3] = v.w;
    }
    return I;
  }
  const int nv = e0 < n ? (int)(n - e0) : 0;
#pragma unroll
  for (int j = 0; j < I; ++j) k[j] = j < nv ? keys[e0 + j] : 0u;
  return nv;
}

template <int I>
__device__ __forceinline__ void add_runs(uint32_t* h, const uint32_t (&k)[I], int nv, int shift, uint32_t mask) {
  if (nv <= 0) return;
  uint32_t cur = (k[0] >> shift) & mask, run = 0;
#pragma unroll
  for (int j = 0; j < I; ++j) {
    if (j < nv) {
      const uint32_t d = (k[j] >> shift) & mask;
      if (d != cur) {
        atomicAdd(&h[cur], run);
        cur = d;
        run = 0;
      }
      ++run;
    }
  }
  atomicAdd(&h[cur], run);
}

// Reduce-then-scan mode, step 1: per-block histogram of one pass, stored
// digit-major: hist[d * nb + block].
// With `sup` (superblock mode), each block also adds its counts into its
// superblock's (kSupBlocks consecutive blocks) per-digit sums, so the scatter
// can find its offsets without a row-scan kernel in between.
constexpr uint32_t kSupBlocks = kSortSupBlocks;
template <int I>
__global__ __launch_bounds__(256) void k_radix_hist(const uint32_t* __restrict__ keys, uint32_t n, int shift,
                                                    int bits, uint32_t nb, uint32_t* __restrict__ hist,
                                                    uint32_t* __restrict__ sup, uint32_t nsup,
                                                    const uint32_t* __restrict__ ndev) {
  __shared__ uint32_t s_h[256];
  const int t = threadIdx.x;
  if (ndev) n = min(n, *ndev);  // capacity mode: the live key count from the device
  s_h[t] = 0;
  uint32_t k[I];
  const int nv = load_run<I>(keys, n, (size_t)blockIdx.x * (256 * I) + (size_t)t * I, k);
  __syncthreads();
  add_runs(s_h, k, nv, shift, (1u << bits) - 1u);
  __syncthreads();
  const uint32_t c = s_h[t];
  if (sup) {  // block-major [nb][256] and [nsup][256]: coalesced both ways
    hist[(size_t)blockIdx.x * 256 + t] = c;
    if (c) atomicAdd(&sup[(size_t)(blockIdx.x / kSupBlocks) * 256 + t], c);
  } else {
    hist[(size_t)t * nb + blockIdx.x] = c;
  }
}

// Superblock mode: digit t's global base for block bid = (exclusive scan of
// the digit totals) + (earlier superblocks' counts) + (earlier blocks of its
// own superblock), every term read straight from the hist kernel's output
// (block-major layouts: thread t's loads are coalesced across the block).
__device__ __forceinline__ uint32_t sup_digit_base(const uint32_t* __restrict__ hist,
                                                   const uint32_t* __restrict__ sup, uint32_t nb, uint32_t nsup,
                                                   uint32_t bid, int t, uint32_t* s_tmp, uint2* bounds,
                                                   uint32_t mask) {
  const uint32_t sb = bid / kSupBlocks;
  // every load of a 32-superblock chunk (and the own superblock's earlier
  // blocks) is issued before the first add: one round trip per chunk
  uint32_t h[kSupBlocks - 1];
#pragma unroll
  for (uint32_t k = 0; k < kSupBlocks - 1; ++k) {
    const uint32_t b = sb * kSupBlocks + k;
    h[k] = b < bid ? hist[(size_t)b * 256 + t] : 0u;
  }
  uint32_t total = 0, pre = 0;
  for (uint32_t q0 = 0; q0 < nsup; q0 += 32) {
    uint32_t v[32];
#pragma unroll
    for (uint32_t k = 0; k < 32; ++k) v[k] = q0 + k < nsup ? sup[(size_t)(q0 + k) * 256 + t] : 0u;
#pragma unroll
    for (uint32_t k = 0; k < 32; ++k) {
      total += v[k];
      pre += q0 + k < sb ? v[k] : 0u;
    }
  }
  uint32_t intra = 0;
#pragma unroll
  for (uint32_t k = 0; k < kSupBlocks - 1; ++k) intra += h[k];
  const uint32_t start = block_excl_scan256(total, s_tmp, nullptr);
  // a one-pass sort hands back every digit's [start, end) of the output
  if (bounds && bid == 0 && (uint32_t)t <= mask) bounds[t] = make_uint2(start, start + total);
  return start + pre + intra;
}

// Reduce-then-scan mode, step 2: exclusive scan of hist row d (over blocks)
// in place; totals[d] = row sum.
__global__ __launch_bounds__(256) void k_radix_rowscan(uint32_t* __restrict__ hist, uint32_t nb,
                                                       uint32_t* __restrict__ totals) {
  __shared__ uint32_t s_tmp[4];
  uint32_t* row = hist + (size_t)blockIdx.x * nb;
  const int t = threadIdx.x;
  const uint32_t per = (nb + 255) / 256;
  const uint32_t b0 = t * per, b1 = min(nb, b0 + per);
  uint32_t s = 0;
  for (uint32_t b = b0; b < b1; ++b) s += row[b];
  uint32_t tot;
  uint32_t run = block_excl_scan256(s, s_tmp, &tot);
  for (uint32_t b = b0; b < b1; ++b) {
    const uint32_t x = row[b];
    row[b] = run;
    run += x;
  }
  if (t == 0) totals[blockIdx.x] = tot;
}

// ---- scatter -----------------------------------------------------------------
constexpr uint32_t kStCount = (1u << 30) - 1u;  // largest key count a sort takes

// One stable digit pass over a block of 256 I keys.  Keys/payloads are loaded
// up front (in flight while ranking); ranks come from LDS atomics-with-return
// issued by each peer group's lowest lane (a wave's LDS atomics execute in
// issue order, so the returned counts are the sequential ones and the 16
// atomics pipeline instead of forming a read-wait-write chain); keys and
// payloads are staged as (key, value) pairs through one 32 KB LDS buffer in digit order so that each
// digit's run leaves as contiguous stores.  The block's digit offsets come
// from the superblock sums (sup) or, without them, from the row-scanned
// per-block histogram (hist: [256][nb], totals: digit totals).
template <int I>
__global__ __launch_bounds__(256) void k_radix_scatter(
    const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin, int iota, uint32_t n, int shift, int bits,
    uint32_t nb, const uint32_t* __restrict__ hist, const uint32_t* __restrict__ totals, uint32_t* __restrict__ kout,
    uint32_t* __restrict__ vout, const uint32_t* __restrict__ sup, uint32_t nsup, uint2* __restrict__ bounds,
    const uint32_t* __restrict__ ndev) {
  constexpr int kTile = 256 * I;
  if (ndev) {  // capacity mode: blocks past the live keys have nothing to move
    n = min(n, *ndev);
    if ((size_t)blockIdx.x * kTile >= n && !(blockIdx.x == 0 && bounds)) return;
  }
  __shared__ uint2 s_buf[kTile];  // (key, value) pairs in digit order (32 KB at I = 16)
  __shared__ uint32_t s_wcnt[4][256];
  __shared__ uint32_t s_lbase[256];
  __shared__ uint32_t s_gbase[256];
  __shared__ uint32_t s_tmp[4];
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const uint32_t mask = (1u << bits) - 1u;
#pragma unroll
  for (int i = 0; i < 4; ++i) s_wcnt[i][t] = 0;
  const uint32_t bid = blockIdx.x;
  const size_t blk0 = (size_t)bid * kTile;
  const size_t base = blk0 + (size_t)w * (64 * I);
  uint32_t key[I], val[I], rank[I];
#pragma unroll
  for (int j = 0; j < I; ++j) {
    const size_t e = base + (size_t)j * 64 + lane;
    const bool valid = e < n;
    key[j] = valid ? kin[e] : 0u;
    val[j] = iota ? (uint32_t)e : (valid ? vin[e] : 0u);
  }
  uint32_t gdig = 0;  // this block's global base of digit t (the scans' barriers publish s_wcnt = 0)
  if (sup) {
    gdig = sup_digit_base(hist, sup, nb, nsup, bid, t, s_tmp, bounds, mask);
  } else {
    const uint32_t ex = block_excl_scan256(totals[t], s_tmp, nullptr);
    gdig = ex + hist[(size_t)t * nb + bid];
  }
#pragma unroll
  for (int j = 0; j < I; ++j) {
    const size_t e = base + (size_t)j * 64 + lane;
    const bool valid = e < n;
    const uint32_t d = (key[j] >> shift) & mask;
    const uint64_t peers = match_digit(d, bits, wave_ballot(valid));
    const int leader = __ffsll((unsigned long long)peers) - 1;
    uint32_t old = 0;
    if (valid && lane == leader) old = atomicAdd(&s_wcnt[w][d], (uint32_t)__popcll(peers));
    old = (uint32_t)__shfl((int)old, leader & 63, 64);
    rank[j] = old + lanes_below(peers);
  }
  __syncthreads();
  {
    const uint32_t c0 = s_wcnt[0][t], c1 = s_wcnt[1][t], c2 = s_wcnt[2][t], c3 = s_wcnt[3][t];
    const uint32_t cnt_d = c0 + c1 + c2 + c3;
    // per-digit: exclusive prefix over waves, then over digits (block-local)
    s_wcnt[0][t] = 0;
    s_wcnt[1][t] = c0;
    s_wcnt[2][t] = c0 + c1;
    s_wcnt[3][t] = c0 + c1 + c2;
    s_lbase[t] = block_excl_scan256(cnt_d, s_tmp, nullptr);
    s_gbase[t] = gdig;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < I; ++j) {
    const size_t e = base + (size_t)j * 64 + lane;
    const uint32_t d = (key[j] >> shift) & mask;
    const uint32_t slot = s_lbase[d] + s_wcnt[w][d] + rank[j];  // block-local slot in digit order
    if (e < n) s_buf[slot] = make_uint2(key[j], val[j]);
  }
  __syncthreads();
  const uint32_t cnt = (size_t)n > blk0 ? (uint32_t)min((size_t)kTile, (size_t)n - blk0) : 0u;
#pragma unroll
  for (int r = 0; r < I; ++r) {
    const uint32_t i = (uint32_t)t + 256u * r;
    if (i < cnt) {
      const uint2 kv = s_buf[i];
      const uint32_t d = (kv.x >> shift) & mask;
      const uint32_t dst = s_gbase[d] + (i - s_lbase[d]);
      kout[dst] = kv.x;
      vout[dst] = kv.y;
    }
  }
}

// ---- wide single pass (9-10 bit digits) ------------------------------------
// A sort on 9 or 10 bits (the 510 sort bins of a 1080p frame) in ONE
// stable pass instead of two 8-bit-or-less passes: the same reduce-then-scan
// structure with DIG digits, each thread owning DIG / 256 consecutive digits
// in the per-digit steps.
template <int DIG, int I>
__global__ __launch_bounds__(256) void k_radix_hist_wide(const uint32_t* __restrict__ keys, uint32_t n, int shift,
                                                         int bits, uint32_t nb, uint32_t* __restrict__ hist,
                                                         const uint32_t* __restrict__ ndev) {
  __shared__ uint32_t s_h[DIG];
  const int t = threadIdx.x;
  if (ndev) n = min(n, *ndev);
#pragma unroll
  for (int k = 0; k < DIG / 256; ++k) s_h[t + 256 * k] = 0;
  uint32_t key[I];
  const int nv = load_run<I>(keys, n, (size_t)blockIdx.x * (256 * I) + (size_t)t * I, key);
  __syncthreads();
  add_runs(s_h, key, nv, shift, (1u << bits) - 1u);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < DIG / 256; ++k) hist[(size_t)(t + 256 * k) * nb + blockIdx.x] = s_h[t + 256 * k];
}

template <int DIG, int I>
__global__ __launch_bounds__(256) void k_radix_scatter_wide(
    const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin, int iota, uint32_t n, int shift, int bits,
    uint32_t nb, const uint32_t* __restrict__ hist, const uint32_t* __restrict__ totals, uint32_t* __restrict__ kout,
    uint32_t* __restrict__ vout, uint2* __restrict__ digit_bounds, const uint32_t* __restrict__ ndev) {
  constexpr int kT = 256 * I, DPT = DIG / 256;
  if (ndev) {
    n = min(n, *ndev);
    if ((size_t)blockIdx.x * kT >= n && !(blockIdx.x == 0 && digit_bounds)) return;
  }
  __shared__ uint2 s_buf[kT];  // (key, value) in digit order
  __shared__ uint32_t s_wcnt[4][DIG];
  __shared__ uint32_t s_lbase[DIG];
  __shared__ uint32_t s_gbase[DIG];
  __shared__ uint32_t s_tmp[4];
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const uint32_t mask = (1u << bits) - 1u;
#pragma unroll
  for (int i = 0; i < 4 * DPT; ++i) (&s_wcnt[0][0])[t + 256 * i] = 0;
  const uint32_t bid = blockIdx.x;
  const size_t blk0 = (size_t)bid * kT;
  const size_t base = blk0 + (size_t)w * (64 * I);
  uint32_t key[I], val[I], rank[I];
#pragma unroll
  for (int j = 0; j < I; ++j) {
    const size_t e = base + (size_t)j * 64 + lane;
    const bool valid = e < n;
    key[j] = valid ? kin[e] : 0u;
    val[j] = iota ? (uint32_t)e : (valid ? vin[e] : 0u);
  }
  {  // global base of this block's digits: digit start (scan of totals) + block offset
    uint32_t tot[DPT], s = 0;
#pragma unroll
    for (int k = 0; k < DPT; ++k) { tot[k] = totals[t * DPT + k]; s += tot[k]; }
    uint32_t run = block_excl_scan256(s, s_tmp, nullptr);  // (its barriers publish s_wcnt = 0)
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
      const int d = t * DPT + k;
      s_gbase[d] = run + hist[(size_t)d * nb + bid];
      // the sorted output's [start, end) of every digit (the key is the
      // whole digit: e.g. the bin ranges k_expand_bins needs)
      if (digit_bounds && bid == 0) digit_bounds[d] = make_uint2(run, run + tot[k]);
      run += tot[k];
    }
  }
#pragma unroll
  for (int j = 0; j < I; ++j) {
    const size_t e = base + (size_t)j * 64 + lane;
    const bool valid = e < n;
    const uint32_t d = (key[j] >> shift) & mask;
    const uint64_t peers = match_digit(d, bits, wave_ballot(valid));
    const int leader = __ffsll((unsigned long long)peers) - 1;
    uint32_t old = 0;
    if (valid && lane == leader) old = atomicAdd(&s_wcnt[w][d], (uint32_t)__popcll(peers));
    old = (uint32_t)__shfl((int)old, leader & 63, 64);
    rank[j] = old + lanes_below(peers);
  }
  __syncthreads();
  {  // per digit: exclusive prefix over waves, then over digits (block-local)
    uint32_t cnt[DPT], s = 0;
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
      const int d = t * DPT + k;
      const uint32_t c0 = s_wcnt[0][d], c1 = s_wcnt[1][d], c2 = s_wcnt[2][d], c3 = s_wcnt[3][d];
      cnt[k] = c0 + c1 + c2 + c3;
      s += cnt[k];
      s_wcnt[0][d] = 0;
      s_wcnt[1][d] = c0;
      s_wcnt[2][d] = c0 + c1;
      s_wcnt[3][d] = c0 + c1 + c2;
    }
    uint32_t run = block_excl_scan256(s, s_tmp, nullptr);
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
      s_lbase[t * DPT + k] = run;
      run += cnt[k];
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < I; ++j) {
    const size_t e = base + (size_t)j * 64 + lane;
    const uint32_t d = (key[j] >> shift) & mask;
    const uint32_t slot = s_lbase[d] + s_wcnt[w][d] + rank[j];
    if (e < n) s_buf[slot] = make_uint2(key[j], val[j]);
  }
  __syncthreads();
  const uint32_t cnt = (size_t)n > blk0 ? (uint32_t)min((size_t)kT, (size_t)n - blk0) : 0u;
#pragma unroll
  for (int r = 0; r < I; ++r) {
    const uint32_t i = (uint32_t)t + 256u * r;
    if (i < cnt) {
      const uint2 kv = s_buf[i];
      const uint32_t d = (kv.x >> shift) & mask;
      const uint32_t dst = s_gbase[d] + (i - s_lbase[d]);
      kout[dst] = kv.x;
      vout[dst] = kv.y;
    }
  }
}

// ---- depth sort over the visible key range (DepthKeyPlan, wgsr_common.h) -----
// Three stable passes over key'' (the first maps the raw keys); each kernel
// derives the passes' digit widths from the range words k_preprocess left in
// the counter block, so the host queues the passes before it knows the range.
// Same reduce-then-scan structure as the 8-bit passes (superblock sums, no
// row-scan launch), with up to 1024 digits: thread t owns digits
// [t dpt, t dpt + dpt), dpt = ceil(digits / 256).
static_assert(kRectPairLanes == 64, "one range word per lane");
__device__ __forceinline__ int bitlen32(uint32_t x) {
  return x ? 32 - __clz((int)x) : 0;
}
// The range words: one per lane, max-reduced across the wave.  Every kernel
// issues its key loads (and the scatter its first digit-sum loads) before it
// needs the plan, so this adds no round trip of its own.
// wave max into a scalar: DPP within each 16-lane row (shifted-in lanes
// read 0), then the four rows' lane 15 by readlane
__device__ __forceinline__ uint32_t wave_max_u32_uniform(uint32_t x) {
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xf, 0xf, true));   // quad_perm [1,0,3,2]
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xf, 0xf, true));   // quad_perm [2,3,0,1]
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true));  // row_shr:4
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true));  // row_shr:8
  const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)x, 15), b = (uint32_t)__builtin_amdgcn_readlane((int)x, 31);
  const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)x, 47), d = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
  return max(max(a, b), max(c, d));
}
// The first kernel (pass 0's histogram) reduces k_preprocess's 2 x 64 range
// words and its workgroup 0 leaves the result in two words (the counter
// block's pad words) that every later kernel reads with one scalar load,
// whose wait does not hold up the vector loads issued before the plan is
// needed.
__device__ __forceinline__ uint2 depth_range_reduce(const uint32_t* __restrict__ range) {
  const int lane = threadIdx.x & 63;
  return make_uint2(wave_max_u32_uniform(range[lane]), wave_max_u32_uniform(range[kRectPairLanes + lane]));
}
__device__ __forceinline__ DepthKeyPlan depth_plan_from2(const uint32_t* __restrict__ range2) {
  return depth_key_plan(range2[0], ~range2[1]);
}

template <int I, int PASS>
__global__ __launch_bounds__(256) void k_depth_hist(const uint32_t* __restrict__ keys, uint32_t n,
                                                    const uint32_t* __restrict__ range, uint32_t* __restrict__ range2,
                                                    uint32_t* __restrict__ hist, uint32_t* __restrict__ sup) {
  __shared__ uint32_t s_h[kDepthMaxDigits];
  const int t = threadIdx.x;
  uint32_t k[I];
  const int nv = load_run<I>(keys, n, (size_t)blockIdx.x * (256 * I) + (size_t)t * I, k);
#pragma unroll
  for (int q = 0; q < kDepthMaxDigits / 256; ++q) s_h[t + 256 * q] = 0;
  DepthKeyPlan pl;
  if (PASS == 0) {
    const uint2 r = depth_range_reduce(range);
    if (blockIdx.x == 0 && t == 0) {
      range2[0] = r.x;
      range2[1] = r.y;
    }
    pl = depth_key_plan(r.x, ~r.y);
  } else {
    pl = depth_plan_from2(range2);
  }
  const int shift = pl.shift[PASS], bits = pl.bits[PASS];
  const uint32_t ndig = 1u << bits;
  if (PASS == 0) {
#pragma unroll
    for (int j = 0; j < I; ++j) k[j] = depth_key_xform(pl, k[j]);
  }
  __syncthreads();
  add_runs(s_h, k, nv, shift, ndig - 1u);
  __syncthreads();
  uint32_t* hrow = hist + (size_t)blockIdx.x * kDepthMaxDigits;
  uint32_t* srow = sup + (size_t)(blockIdx.x / kSupBlocks) * kDepthMaxDigits;
  for (uint32_t d = t; d < ndig; d += 256) {
    const uint32_t c = s_h[d];
    hrow[d] = c;
    if (c) atomicAdd(&srow[d], c);
  }
}

// digit d: its total over all blocks, over the superblocks before block
// bid's, and over the blocks before bid in its own superblock (every load
// of a 32-superblock chunk issued before the first add)
__device__ __forceinline__ void depth_digit_sums(const uint32_t* __restrict__ hist, const uint32_t* __restrict__ sup,
                                                 uint32_t nsup, uint32_t bid, uint32_t d, uint32_t& total,
                                                 uint32_t& pre, uint32_t& intra) {
  const uint32_t sb = bid / kSupBlocks;
  uint32_t h[kSupBlocks - 1];
#pragma unroll
  for (uint32_t k = 0; k < kSupBlocks - 1; ++k) {
    const uint32_t b = sb * kSupBlocks + k;
    h[k] = b < bid ? hist[(size_t)b * kDepthMaxDigits + d] : 0u;
  }
  // the first 32 superblocks' loads go out with the row loads (no loop in
  // between to wait at)
  uint32_t v0[32];
#pragma unroll
  for (uint32_t k = 0; k < 32; ++k) v0[k] = k < nsup ? sup[(size_t)k * kDepthMaxDigits + d] : 0u;
  total = 0;
  pre = 0;
  for (uint32_t q0 = 32; q0 < nsup; q0 += 32) {
    uint32_t v[32];
#pragma unroll
    for (uint32_t k = 0; k < 32; ++k) v[k] = q0 + k < nsup ? sup[(size_t)(q0 + k) * kDepthMaxDigits + d] : 0u;
#pragma unroll
    for (uint32_t k = 0; k < 32; ++k) {
      total += v[k];
      pre += q0 + k < sb ? v[k] : 0u;
    }
  }
#pragma unroll
  for (uint32_t k = 0; k < 32; ++k) {
    total += v0[k];
    pre += k < sb ? v0[k] : 0u;
  }
  intra = 0;
#pragma unroll
  for (uint32_t k = 0; k < kSupBlocks - 1; ++k) intra += h[k];
}

// Thread t owns digits t + 256 q (q < dpt = ceil(digits / 256)), so the
// q = 0 sums are loaded before the plan is known: a column beyond this
// pass's digits holds zeros (superblock sums) or stale counts (block rows)
// and only ever feeds the bases of digits no key has.
template <int I, int PASS>
__global__ __launch_bounds__(256) void k_depth_scatter(const uint32_t* __restrict__ kin,
                                                       const uint32_t* __restrict__ vin, uint32_t n,
                                                       const uint32_t* __restrict__ range2,
                                                       const uint32_t* __restrict__ hist,
                                                       const uint32_t* __restrict__ sup, uint32_t nsup,
                                                       uint32_t* __restrict__ kout, uint32_t* __restrict__ vout) {
  constexpr int kTile = 256 * I, kQ = kDepthMaxDigits / 256;
  __shared__ uint2 s_buf[kTile];
  __shared__ uint32_t s_wcnt[4][kDepthMaxDigits];
  __shared__ uint32_t s_lbase[kDepthMaxDigits];
  __shared__ uint32_t s_gbase[kDepthMaxDigits];
  __shared__ uint32_t s_tmp[4];
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const uint32_t bid = blockIdx.x;
  const size_t blk0 = (size_t)bid * kTile;
  const size_t base = blk0 + (size_t)w * (64 * I);
  uint32_t key[I], val[I], rank[I];
#pragma unroll
  for (int j = 0; j < I; ++j) {
    const size_t e = base + (size_t)j * 64 + lane;
    const bool valid = e < n;
    key[j] = valid ? kin[e] : 0u;
    val[j] = PASS == 0 ? (uint32_t)e : (valid ? vin[e] : 0u);
  }
  uint32_t tot[kQ], pre[kQ], intra[kQ];
  depth_digit_sums(hist, sup, nsup, bid, (uint32_t)t, tot[0], pre[0], intra[0]);
#pragma unroll
  for (int q = 0; q < kQ; ++q) {
    s_wcnt[0][t + 256 * q] = 0;
    s_wcnt[1][t + 256 * q] = 0;
    s_wcnt[2][t + 256 * q] = 0;
    s_wcnt[3][t + 256 * q] = 0;
  }
  const DepthKeyPlan pl = depth_plan_from2(range2);
  const int shift = pl.shift[PASS], bits = pl.bits[PASS];
  const uint32_t ndig = 1u << bits, mask = ndig - 1u;
  const int dpt = (int)((ndig + 255u) >> 8);
#pragma unroll
  for (int q = 1; q < kQ; ++q) {
    tot[q] = pre[q] = intra[q] = 0u;
    if (q < dpt) depth_digit_sums(hist, sup, nsup, bid, (uint32_t)t + 256u * q, tot[q], pre[q], intra[q]);
  }
  if (PASS == 0) {
#pragma unroll
    for (int j = 0; j < I; ++j) key[j] = depth_key_xform(pl, key[j]);
  }
  {  // global base of this block's digits (the scans' barriers publish s_wcnt = 0)
    uint32_t carry = 0;
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      if (q < dpt) {
        uint32_t all;
        const uint32_t ex = block_excl_scan256(tot[q], s_tmp, &all);
        s_gbase[t + 256 * q] = carry + ex + pre[q] + intra[q];
        carry += all;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < I; ++j) {
    const size_t e = base + (size_t)j * 64 + lane;
    const bool valid = e < n;
    const uint32_t d = (key[j] >> shift) & mask;
    const uint64_t peers = match_digit(d, bits, wave_ballot(valid));
    const int leader = __ffsll((unsigned long long)peers) - 1;
    uint32_t old = 0;
    if (valid && lane == leader) old = atomicAdd(&s_wcnt[w][d], (uint32_t)__popcll(peers));
    old = (uint32_t)__shfl((int)old, leader & 63, 64);
    rank[j] = old + lanes_below(peers);
  }
  __syncthreads();
  {  // per digit: exclusive prefix over waves, then over digits (block-local)
    uint32_t carry = 0;
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      if (q < dpt) {
        const uint32_t d = (uint32_t)t + 256u * q;
        const uint32_t c0 = s_wcnt[0][d], c1 = s_wcnt[1][d], c2 = s_wcnt[2][d], c3 = s_wcnt[3][d];
        s_wcnt[0][d] = 0;
        s_wcnt[1][d] = c0;
        s_wcnt[2][d] = c0 + c1;
        s_wcnt[3][d] = c0 + c1 + c2;
        uint32_t all;
        const uint32_t ex = block_excl_scan256(c0 + c1 + c2 + c3, s_tmp, &all);
        s_lbase[d] = carry + ex;
        carry += all;
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < I; ++j) {
    const size_t e = base + (size_t)j * 64 + lane;
    const uint32_t d = (key[j] >> shift) & mask;
    const uint32_t slot = s_lbase[d] + s_wcnt[w][d] + rank[j];
    if (e < n) s_buf[slot] = make_uint2(key[j], val[j]);
  }
  __syncthreads();
  // the last pass writes keys only when a fix-up pass over extra_bits follows
  const bool wkeys = PASS < kDepthPasses - 1 || pl.extra_bits > 0;
  const uint32_t cnt = (size_t)n > blk0 ? (uint32_t)min((size_t)kTile, (size_t)n - blk0) : 0u;
#pragma unroll
  for (int r = 0; r < I; ++r) {
    const uint32_t i = (uint32_t)t + 256u * r;
    if (i < cnt) {
      const uint2 kv = s_buf[i];
      const uint32_t d = (kv.x >> shift) & mask;
      const uint32_t dst = s_gbase[d] + (i - s_lbase[d]);
      if (wkeys) kout[dst] = kv.x;
      vout[dst] = kv.y;
    }
  }
}

// ---- exclusive scan of u32 values gathered as vals[idx[i]] (idx may be null)
__global__ __launch_bounds__(256) void k_scan_reduce(const uint32_t* __restrict__ vals, uint32_t stride,
                                                     const uint32_t* __restrict__ idx, uint32_t n,
                                                     uint32_t* __restrict__ bsum) {
  __shared__ uint32_t s_tmp[4];
  const int t = threadIdx.x;
  const size_t b0 = (size_t)blockIdx.x * kScanTile + (size_t)t * (kScanTile / 256);
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < kScanTile / 256; ++j) {
    const size_t i = b0 + j;
    if (i < n) s += vals[(size_t)(idx ? idx[i] : i) * stride];
  }
  uint32_t tot;
  block_excl_scan256(s, s_tmp, &tot);
  if (t == 0) bsum[blockIdx.x] = tot;
}

// single workgroup: exclusive scan of nbs block sums in place, total -> bsum[nbs], *total_out
__global__ __launch_bounds__(256) void k_scan_bsum(uint32_t* __restrict__ bsum, uint32_t nbs,
                                                   uint32_t* __restrict__ total_out) {
  __shared__ uint32_t s_tmp[4];
  const int t = threadIdx.x;
  const uint32_t per = (nbs + 255) / 256;
  const uint32_t b0 = t * per, b1 = min(nbs, b0 + per);
  uint32_t s = 0;
  for (uint32_t b = b0; b < b1; ++b) s += bsum[b];
  uint32_t tot;
  uint32_t run = block_excl_scan256(s, s_tmp, &tot);
  for (uint32_t b = b0; b < b1; ++b) {
    uint32_t x = bsum[b];
    bsum[b] = run;
    run += x;
  }
  if (t == 0) {
    bsum[nbs] = tot;
    if (total_out) *total_out = tot;
  }
}

// out[i] = exclusive prefix; if scatter_out: scatter_out[idx[i]] = prefix
__global__ __launch_bounds__(256) void k_scan_down(const uint32_t* __restrict__ vals, uint32_t stride,
                                                   const uint32_t* __restrict__ idx, uint32_t n,
                                                   const uint32_t* __restrict__ bsum, uint32_t* __restrict__ out,
                                                   uint32_t* __restrict__ scatter_out) {
  __shared__ uint32_t s_tmp[4];
  constexpr int PER = kScanTile / 256;
  const int t = threadIdx.x;
  const size_t b0 = (size_t)blockIdx.x * kScanTile + (size_t)t * PER;
  uint32_t v[PER];
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const size_t i = b0 + j;
    v[j] = (i < n) ? vals[(size_t)(idx ? idx[i] : i) * stride] : 0u;
    s += v[j];
  }
  uint32_t run = block_excl_scan256(s, s_tmp, nullptr) + bsum[blockIdx.x];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const size_t i = b0 + j;
    if (i < n) {
      out[i] = run;
      if (scatter_out) scatter_out[idx[i]] = run;
    }
    run += v[j];
  }
  if (blockIdx.x == gridDim.x - 1 && t == 255) out[n] = run;  // grand total at out[n]
}

// ---- exclusive scan of packed pairs (lo 16 | hi 16 bits) gathered by index --
// (the exact tile-list length and the bin count of each Gaussian, in depth
// order: one gather of one word for both sums; sums kept as two u32s)
template <int PER>
__global__ __launch_bounds__(256) void k_scan2_reduce(const uint32_t* __restrict__ packed, uint32_t stride,
                                                      const uint32_t* __restrict__ idx, uint32_t n,
                                                      uint2* __restrict__ bsum, uint2* __restrict__ bsup,
                                                      const PublishJob pub) {
  __shared__ uint2 s_tmp[4];
  const int t = threadIdx.x;
  if (pub.counter && blockIdx.x == 0 && t < 64) publish_counts(pub, t);  // (the forward's counts to the host)
  const size_t b0 = (size_t)blockIdx.x * (256 * PER) + (size_t)t * PER;
  uint2 acc = make_uint2(0u, 0u);
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const size_t i = b0 + j;
    if (i < n) {
      const uint32_t v = packed[(size_t)(idx ? idx[i] : (uint32_t)i) * stride];
      acc.x += v & 0xFFFFu;
      acc.y += v >> 16;
    }
  }
  uint2 tot;
  block_excl_scan256_2(acc, s_tmp, &tot);
  if (t == 0) {
    bsum[blockIdx.x] = tot;
    if (bsup) {  // (superblock mode: bsum keeps the raw block sums)
      uint32_t* sp = reinterpret_cast<uint32_t*>(&bsup[(size_t)(blockIdx.x / kScanSupBlocks) * kScanSupStride]);
      if (tot.x) atomicAdd(sp, tot.x);
      if (tot.y) atomicAdd(sp + 1, tot.y);
    }
  }
}

// single workgroup of 1024 threads: exclusive scan of the nbs block sums in
// place, total -> bsum[nbs].  Each thread owns a contiguous run of `per`
// sums, loaded up front in chunks of 8 (independent loads in flight).
__global__ __launch_bounds__(1024) void k_scan2_bsum(uint2* __restrict__ bsum, uint32_t nbs) {
  constexpr int NW = 16;
  __shared__ uint2 s_w[NW];
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const uint32_t per = (nbs + 1023) / 1024;
  const uint32_t b0 = min(nbs, t * per), b1 = min(nbs, b0 + per);
  uint2 acc = make_uint2(0u, 0u);
  for (uint32_t b = b0; b < b1; b += 8) {
    uint2 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = b + u < b1 ? bsum[b + u] : make_uint2(0u, 0u);
#pragma unroll
    for (int u = 0; u < 8; ++u) { acc.x += v[u].x; acc.y += v[u].y; }
  }
  const uint32_t ia = wave_incl_scan(acc.x), ib = wave_incl_scan(acc.y);
  if (lane == 63) s_w[w] = make_uint2(ia, ib);
  __syncthreads();
  uint2 run = make_uint2(ia - acc.x, ib - acc.y), tot = make_uint2(0u, 0u);
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const uint2 x = s_w[k];
    if (k < w) { run.x += x.x; run.y += x.y; }
    tot.x += x.x;
    tot.y += x.y;
  }
  for (uint32_t b = b0; b < b1; b += 8) {
    uint2 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = b + u < b1 ? bsum[b + u] : make_uint2(0u, 0u);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (b + u < b1) bsum[b + u] = run;
      run.x += v[u].x;
      run.y += v[u].y;
    }
  }
  if (t == 0) bsum[nbs] = tot;
}

}  // namespace

// 9 or 10 key bits sort in one wide pass
static bool wide_pass(int bits) { return bits > 8 && bits <= 10; }

int radix_passes(int begin_bit, int end_bit) {
  const int bits = end_bit - begin_bit;
  if (bits <= 0) return 0;
  return wide_pass(bits) ? 1 : (bits + 7) / 8;
}

// Superblock sums of a reduce-then-scan sort of n keys over [begin_bit,
// end_bit): their place in `status` (words) and size (words); 0 words when the
// sort does not use them (wide pass).  A caller
// that zeroes this range itself passes sup_zeroed to radix_sort_pairs.
size_t sort_sup_words(size_t n, int begin_bit, int end_bit, size_t* offset_words) {
  const int bits = end_bit - begin_bit;
  if (offset_words) *offset_words = 0;
  if (n == 0 || bits <= 0 || wide_pass(bits)) return 0;
  const uint32_t nb = sort_blocks(n);
  if (offset_words) *offset_words = 256 * (size_t)nb;
  return 256 * (size_t)((nb + kSupBlocks - 1) / kSupBlocks) * ((bits + 7) / 8);
}

// one sort with I keys per thread (workgroup tile 256 I)
template <int I>
static hipError_t radix_sort_tiled(uint32_t* keys, uint32_t* keys_alt, uint32_t* vals, uint32_t* vals_alt,
                                   bool vals_iota, size_t n, int begin_bit, int end_bit, uint32_t* status,
                                   uint32_t* totals, hipStream_t stream, bool* result_in_alt, uint2* digit_bounds,
                                   bool* bounds_done, bool sup_zeroed, const uint32_t* ndev) {
  const uint32_t nb = sort_blocks(n);
  if (wide_pass(end_bit - begin_bit) && n <= (size_t)kStCount) {
    const int bits = end_bit - begin_bit;
    // status doubles as the [DIG][nb] per-block histogram (DIG <= 1024 <= 256 x kMaxSortPasses rows)
    if (bits <= 9) {
      hipLaunchKernelGGL((k_radix_hist_wide<512, I>), dim3(nb), dim3(256), 0, stream, keys, (uint32_t)n, begin_bit,
                         bits, nb, status, ndev);
      hipLaunchKernelGGL(k_radix_rowscan, dim3(512), dim3(256), 0, stream, status, nb, totals);
      hipLaunchKernelGGL((k_radix_scatter_wide<512, I>), dim3(nb), dim3(256), 0, stream, keys, vals,
                         vals_iota ? 1 : 0, (uint32_t)n, begin_bit, bits, nb, status, totals, keys_alt, vals_alt,
                         begin_bit == 0 ? digit_bounds : nullptr, ndev);
    } else {
      hipLaunchKernelGGL((k_radix_hist_wide<1024, I>), dim3(nb), dim3(256), 0, stream, keys, (uint32_t)n, begin_bit,
                         bits, nb, status, ndev);
      hipLaunchKernelGGL(k_radix_rowscan, dim3(1024), dim3(256), 0, stream, status, nb, totals);
      hipLaunchKernelGGL((k_radix_scatter_wide<1024, I>), dim3(nb), dim3(256), 0, stream, keys, vals,
                         vals_iota ? 1 : 0, (uint32_t)n, begin_bit, bits, nb, status, totals, keys_alt, vals_alt,
                         begin_bit == 0 ? digit_bounds : nullptr, ndev);
    }
    *result_in_alt = true;
    if (bounds_done) *bounds_done = digit_bounds && begin_bit == 0;
    return hipGetLastError();
  }
  const int passes = (end_bit - begin_bit + 7) / 8;
  if (passes > kMaxSortPasses || n > (size_t)kStCount) return hipErrorInvalidValue;
  uint32_t* ghist = totals;  // digit totals (row-scan path only)
  // superblock sums: one memset of every pass's sums (or none: the caller
  // zeroed them) replaces a row-scan launch per pass
  const uint32_t nsup = (nb + kSupBlocks - 1) / kSupBlocks;
  uint32_t* sup = status + 256 * (size_t)nb;  // (sort_status_bytes reserves 256 nb + kMaxSortPasses x 256 nsup words)
  if (!sup_zeroed) {
    hipError_t e = hipMemsetAsync(sup, 0, 4 * 256 * (size_t)nsup * passes, stream);
    if (e != hipSuccess) return e;
  }
  uint32_t *ki = keys, *ko = keys_alt, *vi = vals, *vo = vals_alt;
  bool iota = vals_iota;
  // balanced digits (13 tile-id bits -> 7 + 6, not 8 + 5): wider per-block
  // digit runs leave as longer contiguous stores in every pass
  const int per = (end_bit - begin_bit + passes - 1) / passes;
  for (int p = 0; p < passes; ++p) {
    const int shift = begin_bit + per * p;
    const int bits = min(per, end_bit - shift);
    // status doubles as the [256][nb] per-block histogram, followed by the
    // passes' [256][nsup] superblock sums
    uint32_t* sp = sup + (size_t)p * 256 * nsup;
    hipLaunchKernelGGL(k_radix_hist<I>, dim3(nb), dim3(256), 0, stream, ki, (uint32_t)n, shift, bits, nb, status,
                       sp, nsup, ndev);
    // a single pass over bits [0, end_bit) also writes the digit bounds
    uint2* db = (passes == 1 && begin_bit == 0) ? digit_bounds : nullptr;
    hipLaunchKernelGGL(k_radix_scatter<I>, dim3(nb), dim3(256), 0, stream, ki, vi, iota ? 1 : 0, (uint32_t)n, shift,
                       bits, nb, status, ghist, ko, vo, sp, nsup, db, ndev);
    if (db && bounds_done) *bounds_done = true;
    iota = false;
    uint32_t* tk = ki; ki = ko; ko = tk;
    uint32_t* tv = vi; vi = vo; vo = tv;
    *result_in_alt = !*result_in_alt;
  }
  return hipGetLastError();
}

hipError_t radix_sort_pairs(uint32_t* keys, uint32_t* keys_alt, uint32_t* vals, uint32_t* vals_alt, bool vals_iota,
                            size_t n, int begin_bit, int end_bit, uint32_t* status, uint32_t* totals,
                            hipStream_t stream, bool* result_in_alt, uint2* digit_bounds, bool* bounds_done,
                            bool sup_zeroed, const uint32_t* ndev) {
  *result_in_alt = false;
  if (bounds_done) *bounds_done = false;
  if (n == 0 || end_bit <= begin_bit) {
    if (vals_iota && n > 0) {
      // a zero-pass sort still has to materialise the identity permutation
      return hipErrorInvalidValue;
    }
    return hipSuccess;
  }
  switch (sort_items(n)) {
    case kTinySortItems:
      return radix_sort_tiled<kTinySortItems>(keys, keys_alt, vals, vals_alt, vals_iota, n, begin_bit, end_bit, status,
                                              totals, stream, result_in_alt, digit_bounds, bounds_done, sup_zeroed,
                                              ndev);
    case kSmallSortItems:
      return radix_sort_tiled<kSmallSortItems>(keys, keys_alt, vals, vals_alt, vals_iota, n, begin_bit, end_bit,
                                               status, totals, stream, result_in_alt, digit_bounds, bounds_done,
                                               sup_zeroed, ndev);
    default:
      return radix_sort_tiled<kSortItems>(keys, keys_alt, vals, vals_alt, vals_iota, n, begin_bit, end_bit, status,
                                          totals, stream, result_in_alt, digit_bounds, bounds_done, sup_zeroed,
                                          ndev);
  }
}

template <int I>
static hipError_t depth_sort_tiled(uint32_t* keys, uint32_t* keys_alt, uint32_t* vals, uint32_t* vals_alt, size_t n,
                                   const uint32_t* range, uint32_t* range2, uint32_t* scratch, hipStream_t s) {
  const uint32_t nb = (uint32_t)((n + 256 * I - 1) / (256 * I)), nsup = (nb + kSupBlocks - 1) / kSupBlocks;
  uint32_t* hist = scratch;
  uint32_t* sup = scratch + depth_sort_sup_offset_words(n);
  const size_t sup_pass = (size_t)kDepthMaxDigits * nsup;
  const uint32_t un = (uint32_t)n;
  hipLaunchKernelGGL((k_depth_hist<I, 0>), dim3(nb), dim3(256), 0, s, keys, un, range, range2, hist, sup);
  hipLaunchKernelGGL((k_depth_scatter<I, 0>), dim3(nb), dim3(256), 0, s, keys, vals, un, range2, hist, sup, nsup,
                     keys_alt, vals_alt);
  hipLaunchKernelGGL((k_depth_hist<I, 1>), dim3(nb), dim3(256), 0, s, keys_alt, un, range, range2, hist,
                     sup + sup_pass);
  hipLaunchKernelGGL((k_depth_scatter<I, 1>), dim3(nb), dim3(256), 0, s, keys_alt, vals_alt, un, range2, hist,
                     sup + sup_pass, nsup, keys, vals);
  hipLaunchKernelGGL((k_depth_hist<I, 2>), dim3(nb), dim3(256), 0, s, keys, un, range, range2, hist,
                     sup + 2 * sup_pass);
  hipLaunchKernelGGL((k_depth_scatter<I, 2>), dim3(nb), dim3(256), 0, s, keys, vals, un, range2, hist,
                     sup + 2 * sup_pass, nsup, keys_alt, vals_alt);
  return hipGetLastError();
}

hipError_t launch_depth_sort(uint32_t* keys, uint32_t* keys_alt, uint32_t* vals, uint32_t* vals_alt, size_t n,
                             const uint32_t* range, uint32_t* range2, uint32_t* scratch, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (n > (size_t)kStCount) return hipErrorInvalidValue;
  switch (sort_items(n)) {
    case kTinySortItems:
      return depth_sort_tiled<kTinySortItems>(keys, keys_alt, vals, vals_alt, n, range, range2, scratch, s);
    case kSmallSortItems:
      return depth_sort_tiled<kSmallSortItems>(keys, keys_alt, vals, vals_alt, n, range, range2, scratch, s);
    default:
      return depth_sort_tiled<kSortItems>(keys, keys_alt, vals, vals_alt, n, range, range2, scratch, s);
  }
}

hipError_t exclusive_scan_gather(const uint32_t* vals, const uint32_t* idx, size_t n, uint32_t* out,
                                 uint32_t* scatter_out, uint32_t* bsum, uint32_t* total_out, hipStream_t stream,
                                 uint32_t stride) {
  const uint32_t nbs = (uint32_t)((n + kScanTile - 1) / kScanTile);
  if (n == 0) {
    hipError_t e = hipMemsetAsync(out, 0, sizeof(uint32_t), stream);
    if (e == hipSuccess && total_out) e = hipMemsetAsync(total_out, 0, sizeof(uint32_t), stream);
    return e;
  }
  hipLaunchKernelGGL(k_scan_reduce, dim3(nbs), dim3(256), 0, stream, vals, stride, idx, (uint32_t)n, bsum);
  hipLaunchKernelGGL(k_scan_bsum, dim3(1), dim3(256), 0, stream, bsum, nbs, total_out);
  hipLaunchKernelGGL(k_scan_down, dim3(nbs), dim3(256), 0, stream, vals, stride, idx, (uint32_t)n, bsum, out,
                     scatter_out);
  return hipGetLastError();
}

hipError_t packed_scan_blocks(const uint32_t* packed, uint32_t stride, const uint32_t* idx, size_t n, void* bsum,
                              hipStream_t stream, void* bsup, const PublishJob& pub) {
  const uint32_t nbs = (uint32_t)((n + kPackedScanTile - 1) / kPackedScanTile);
  if (n == 0) return hipMemsetAsync(bsum, 0, sizeof(uint2), stream);
  uint2* bs = static_cast<uint2*>(bsum);
  hipLaunchKernelGGL(k_scan2_reduce<kPackedScanTile / 256>, dim3(nbs), dim3(256), 0, stream, packed, stride, idx,
                     (uint32_t)n, bs, static_cast<uint2*>(bsup), pub);
  if (!bsup) hipLaunchKernelGGL(k_scan2_bsum, dim3(1), dim3(1024), 0, stream, bs, nbs);
  return hipGetLastError();
}

}  // namespace wgsr
