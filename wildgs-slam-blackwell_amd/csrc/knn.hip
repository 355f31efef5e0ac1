// simple_knn._C.distCUDA2 for gfx950.
//
// out[i] = mean of the squared distances from point i to its 3 nearest other
// points -- exact, like upstream's box-pruned search.  Pipeline:
//   bbox (min/max, seeded with 0 as upstream's cub::DeviceReduce init)
//   -> 30-bit Morton codes -> radix sort of their top 24 bits (sort.hip) -> points gathered into
//   Morton order -> bounds of 64-point leaf boxes and of 64-leaf super-boxes
//   -> per point: seed a reject bound from the +-3 Morton neighbours, scan
//      the wave's own leaf, then every 8-point mini-box whose distance to the
//      point is within the current 3rd-best distance.  A wave scans a
//      mini-box when ANY of its lanes needs it (staged through LDS, read as
//      broadcasts); scanning one a lane did not need cannot change its exact
//      answer.
// Distances are evaluated unfused (dx*dx + dy*dy + dz*dz) so results are
// bitwise identical to the CPU restatement (oracle/cpu_raster.cpp).
#include <cfloat>

#include "wgsr_common.h"
#include "wgsr_internal.h"

namespace wgsr {

namespace {

constexpr int kBox = 64;  // points per leaf box == one k_knn wave
constexpr int kSuper = 64;  // boxes per super-box
constexpr int kMini = 8;  // points per mini-box (8 per leaf)
// The search is exact in any point order; the order only decides how compact
// the leaves are.  Sorting the codes' top 24 bits (256^3 cells, 3 radix
// passes) keeps the leaves as compact as the full 30 bits for a fourth less.
constexpr int kMortonSortLo = 6;

struct KnnLayout {
  size_t part, bbox, codes, codes_alt, idx, idx_alt, spts, boxes, minis, supers, hist, totals, total;
  KnnLayout(size_t P) {
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o = align256(o + bytes); return r; };
    const size_t nbox = (P + kBox - 1) / kBox, nsup = (nbox + kSuper - 1) / kSuper;
    part = take(6 * 4 * 1024);
    bbox = take(6 * 4);
    codes = take(4 * P);
    codes_alt = take(4 * P);
    idx = take(4 * P);
    idx_alt = take(4 * P);
    spts = take(16 * P);
    boxes = take(32 * nbox);
    minis = take(32 * nbox * (kBox / kMini));
    supers = take(32 * nsup);
    hist = take(sort_status_bytes(P));
    totals = take(kSortTotalsBytes);
    total = o;
  }
};

__global__ __launch_bounds__(256) void k_bbox_partial(int P, const float* __restrict__ pts, float* __restrict__ part) {
  __shared__ float s[6][256];
  const int t = threadIdx.x;
  float mn[3] = {0.f, 0.f, 0.f}, mx[3] = {0.f, 0.f, 0.f};  // upstream reduce init {0,0,0}
  for (int i = blockIdx.x * 256 + t; i < P; i += gridDim.x * 256)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float v = pts[3 * (size_t)i + k];
      mn[k] = fminf(mn[k], v);
      mx[k] = fmaxf(mx[k], v);
    }
#pragma unroll
  for (int k = 0; k < 3; ++k) { s[k][t] = mn[k]; s[3 + k][t] = mx[k]; }
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (t < off)
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        s[k][t] = fminf(s[k][t], s[k][t + off]);
        s[3 + k][t] = fmaxf(s[3 + k][t], s[3 + k][t + off]);
      }
    __syncthreads();
  }
  if (t < 6) part[6 * blockIdx.x + t] = s[t][0];
}

__global__ __launch_bounds__(256) void k_bbox_final(int nparts, const float* __restrict__ part,
                                                    float* __restrict__ bbox) {
  // thread t folds partials t, t + 256, ... (partial 0 seeds every thread);
  // then one LDS tree over the 256 threads per component
  __shared__ float sm[6][256];
  const int t = threadIdx.x;
  float v[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) v[k] = part[k];
  for (int b = t; b < nparts; b += 256)
#pragma unroll
    for (int k = 0; k < 6; ++k) v[k] = (k < 3) ? fminf(v[k], part[6 * b + k]) : fmaxf(v[k], part[6 * b + k]);
#pragma unroll
  for (int k = 0; k < 6; ++k) sm[k][t] = v[k];
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (t < off)
#pragma unroll
      for (int k = 0; k < 6; ++k)
        sm[k][t] = (k < 3) ? fminf(sm[k][t], sm[k][t + off]) : fmaxf(sm[k][t], sm[k][t + off]);
    __syncthreads();
  }
  if (t < 6) bbox[t] = sm[t][0];
}

__device__ __forceinline__ uint32_t prep_morton(uint32_t x) {
  x = (x | (x << 16)) & 0x030000FF;
  x = (x | (x << 8)) & 0x0300F00F;
  x = (x | (x << 4)) & 0x030C30C3;
  x = (x | (x << 2)) & 0x09249249;
  return x;
}

__global__ __launch_bounds__(256) void k_morton(int P, const float* __restrict__ pts, const float* __restrict__ bbox,
                                                uint32_t* __restrict__ codes) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= P) return;
  uint32_t c[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float v = ((pts[3 * (size_t)i + k] - bbox[k]) / (bbox[3 + k] - bbox[k])) * ((1 << 10) - 1);
    c[k] = prep_morton(v == v ? (uint32_t)fmaxf(v, 0.f) : 0u);
  }
  codes[i] = c[0] | (c[1] << 1) | (c[2] << 2);
}

__global__ __launch_bounds__(256) void k_gather_sorted(int P, const float* __restrict__ pts,
                                                       const uint32_t* __restrict__ idx, float4* __restrict__ spts) {
  const int s = blockIdx.x * 256 + threadIdx.x;
  if (s >= P) return;
  const uint32_t i = idx[s];
  spts[s] = make_float4(pts[3 * (size_t)i], pts[3 * (size_t)i + 1], pts[3 * (size_t)i + 2], 0.f);
}

// bounds of `per` consecutive items (float4 points, or (min,max) float4 pairs)
__global__ __launch_bounds__(256) void k_bounds(int n, int per, const float4* __restrict__ src, int src_is_box,
                                                float4* __restrict__ dst) {
  __shared__ float s[6][256];
  const int t = threadIdx.x;
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int j = t; j < per; j += 256) {
    const int i = blockIdx.x * per + j;
    if (i >= n) break;
    const float4 lo = src_is_box ? src[2 * (size_t)i] : src[i];
    const float4 hi = src_is_box ? src[2 * (size_t)i + 1] : lo;
    mn[0] = fminf(mn[0], lo.x); mn[1] = fminf(mn[1], lo.y); mn[2] = fminf(mn[2], lo.z);
    mx[0] = fmaxf(mx[0], hi.x); mx[1] = fmaxf(mx[1], hi.y); mx[2] = fmaxf(mx[2], hi.z);
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) { s[k][t] = mn[k]; s[3 + k][t] = mx[k]; }
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (t < off)
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        s[k][t] = fminf(s[k][t], s[k][t + off]);
        s[3 + k][t] = fmaxf(s[3 + k][t], s[3 + k][t + off]);
      }
    __syncthreads();
  }
  if (t == 0) {
    dst[2 * (size_t)blockIdx.x] = make_float4(s[0][0], s[1][0], s[2][0], 0.f);
    dst[2 * (size_t)blockIdx.x + 1] = make_float4(s[3][0], s[4][0], s[5][0], 0.f);
  }
}

// leaf (64-point) and mini (8-point) box bounds of the Morton-ordered
// points: one wave per leaf, butterfly min/max over 8 then 64 lanes
__global__ __launch_bounds__(256) void k_leaf_bounds(int P, const float4* __restrict__ spts, float4* __restrict__ boxes,
                                                     float4* __restrict__ minis) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  if (blockIdx.x * 256 + (threadIdx.x & ~63) >= P) return;  // whole wave past the end
  float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  if (i < P) {
    const float4 q = spts[i];
    lo[0] = hi[0] = q.x; lo[1] = hi[1] = q.y; lo[2] = hi[2] = q.z;
  }
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      lo[k] = fminf(lo[k], __shfl_xor(lo[k], off, 64));
      hi[k] = fmaxf(hi[k], __shfl_xor(hi[k], off, 64));
    }
    if (off == kMini / 2 && (lane & (kMini - 1)) == 0) {  // this lane's mini-box is complete
      const size_t m = (size_t)i / kMini;
      minis[2 * m] = make_float4(lo[0], lo[1], lo[2], 0.f);
      minis[2 * m + 1] = make_float4(hi[0], hi[1], hi[2], 0.f);
    }
  }
  if (lane == 0) {
    const size_t b = (size_t)i / kBox;
    boxes[2 * b] = make_float4(lo[0], lo[1], lo[2], 0.f);
    boxes[2 * b + 1] = make_float4(hi[0], hi[1], hi[2], 0.f);
  }
}

// (dx*dx + dy*dy) + dz*dz with x, y as packed pairs (the same unfused,
// correctly rounded operations in the same order)
__device__ __forceinline__ float sqdist(float4 a, float4 b) {
#pragma clang fp contract(off)
  const v2f dxy = v2f{b.x, b.y} - v2f{a.x, a.y};
  const float dz = b.z - a.z;
  const v2f sq = dxy * dxy;
  return (sq.x + sq.y) + dz * dz;
}

// squared distance from p to a box, for pruning: it never exceeds sqdist(p,
// q) of a point q inside the box (per-axis gaps are differences of the same
// operands and correctly rounded subtraction is monotone; same unfused sums)
__device__ __forceinline__ float box_dist(float4 lo, float4 hi, float4 p) {
#pragma clang fp contract(off)
  const float dx = fmaxf(fmaxf(lo.x - p.x, p.x - hi.x), 0.f);
  const float dy = fmaxf(fmaxf(lo.y - p.y, p.y - hi.y), 0.f);
  const float dz = fmaxf(fmaxf(lo.z - p.z, p.z - hi.z), 0.f);
  return dx * dx + dy * dy + dz * dz;
}

// squared gap between two boxes: never exceeds box_dist(b, p) for a point p
// inside box a (same monotonicity argument)
__device__ __forceinline__ float box_box(float4 alo, float4 ahi, float4 blo, float4 bhi) {
#pragma clang fp contract(off)
  const float dx = fmaxf(fmaxf(blo.x - ahi.x, alo.x - bhi.x), 0.f);
  const float dy = fmaxf(fmaxf(blo.y - ahi.y, alo.y - bhi.y), 0.f);
  const float dz = fmaxf(fmaxf(blo.z - ahi.z, alo.z - bhi.z), 0.f);
  return dx * dx + dy * dy + dz * dz;
}

// fold d into the ascending 3 best (b0 <= b1 <= b2): two medians and a min
__device__ __forceinline__ void update3(float d, float& b0, float& b1, float& b2) {
  b2 = __builtin_amdgcn_fmed3f(b1, b2, d);
  b1 = __builtin_amdgcn_fmed3f(b0, b1, d);
  b0 = fminf(b0, d);
}

// LDS written by some lanes of a wave and read by others: a wave's LDS
// operations complete in order, so a compiler-level fence is all it takes.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Staged leaves are read back from the wave's LDS slots as broadcasts.
// Distances from p to the n staged points of a leaf starting at sorted index
// i0 (self excluded by index), folded into the running 3 best; branch-free
// and unrolled so the broadcast LDS reads of a group issue together
__device__ __forceinline__ void scan_leaf(const float4* pts, int i0, int n, int s, float4 p, float& b0, float& b1,
                                          float& b2) {
  if (n == 64) {
#pragma unroll 8
    for (int j = 0; j < 64; ++j) {
      const float d = sqdist(p, pts[j]);
      update3(i0 + j == s ? FLT_MAX : d, b0, b1, b2);
    }
  } else {
    for (int j = 0; j < n; ++j) {
      const float d = sqdist(p, pts[j]);
      update3(i0 + j == s ? FLT_MAX : d, b0, b1, b2);
    }
  }
}

struct KnnWaveLds {
  float4 pts[64];
  float4 mini[2 * (kBox / kMini)];  // (lo, hi) of the staged leaf's mini-boxes
  float4 own[2 * (kBox / kMini)];  // (lo, hi) of the wave's own mini-boxes
  float ownR[kBox / kMini];  // the largest bound among each own mini-box's lanes
  float4 qp[64];  // the wave's own points (lane order)
  float qb[64];  // and their current search radii
  float4 leaf_lo[64], leaf_hi[64];
};

// refresh ownR / qb from the lanes' current radii; returns the wave's largest
__device__ __forceinline__ float own_bounds(KnnWaveLds& L, float bound, int lane) {
  const float mine = bound;
#pragma unroll
  for (int off = 1; off < kMini; off <<= 1) bound = fmaxf(bound, __shfl_xor(bound, off, 64));
  wave_lds_sync();
  L.qb[lane] = mine;
  if ((lane & (kMini - 1)) == 0) L.ownR[lane / kMini] = bound;
  wave_lds_sync();
#pragma unroll
  for (int off = kMini; off < 64; off <<= 1) bound = fmaxf(bound, __shfl_xor(bound, off, 64));
  return bound;
}

// can any lane need a point of box (lo, hi)?  Tested against each own
// mini-box grown by its lanes' largest bound: box_box(own mini, box) never
// exceeds box_dist(p, box) for a lane p inside that mini-box, so this is a
// superset of the per-lane test.  An own mini-box much larger than its
// lanes' radii (its 8 Morton-consecutive points straddle a jump of the curve:
// bit m of split_m) would pass a whole slab of the scene, so its lanes are
// tested one by one instead.
__device__ __forceinline__ bool near_own(const KnnWaveLds& L, uint32_t split_m, float4 lo, float4 hi) {
  bool r = false;
#pragma unroll
  for (int m = 0; m < kBox / kMini; ++m) {
    if (split_m >> m & 1) {
      for (int j = m * kMini; j < (m + 1) * kMini; ++j) r |= box_dist(lo, hi, L.qp[j]) <= L.qb[j];
    } else {
      r |= box_box(L.own[2 * m], L.own[2 * m + 1], lo, hi) <= L.ownR[m];
    }
  }
  return r;
}

// a non-own leaf: only its mini-boxes some lane still needs (the own leaf
// holds every lane's self; no other leaf does, so no self test here)
// mmask: the mini-boxes that pass the wave-level (grown own box) test
__device__ __forceinline__ void scan_minis(const KnnWaveLds& L, uint32_t mmask, int n, float lim, float4 p,
                                           float& b0, float& b1, float& b2) {
  while (mmask) {
    const int m = __builtin_ctz(mmask);
    mmask &= mmask - 1;
    if (!__any(box_dist(L.mini[2 * m], L.mini[2 * m + 1], p) <= fminf(lim, b2))) continue;
    if (n - m * kMini >= kMini) {
#pragma unroll
      for (int j = 0; j < kMini; ++j) update3(sqdist(p, L.pts[m * kMini + j]), b0, b1, b2);
    } else {
      for (int j = m * kMini; j < n; ++j) update3(sqdist(p, L.pts[j]), b0, b1, b2);
    }
  }
}

// Every leaf but the own one, pruned coarse-to-fine with each lane's search
// radius fminf(lim, b2): super-boxes and a super-box's leaves one per lane
// against the grown own mini-boxes, the surviving leaves per lane (any lane
// within its radius), and inside a staged leaf its 8-point mini-boxes (first
// against the own leaf box grown by the wave's largest radius, then per lane).
__device__ __forceinline__ void walk(KnnWaveLds& L, int P, const float4* __restrict__ spts,
                                     const float4* __restrict__ boxes, int nbox, const float4* __restrict__ minis,
                                     const float4* __restrict__ supers, int nsup, int own, float4 olo, float4 ohi,
                                     float4 p, int lane, float lim, uint32_t split_m, float& b0, float& b1,
                                     float& b2) {
  constexpr int kM = kBox / kMini;
  for (int c = 0; c < nsup; c += 64) {
    uint64_t smask;
    {
      own_bounds(L, fminf(lim, b2), lane);
      const int k = c + lane;
      bool cand = false;
      if (k < nsup) cand = near_own(L, split_m, supers[2 * k], supers[2 * k + 1]);
      smask = __ballot(cand);
    }
    while (smask) {
      const int sb = c + __builtin_ctzll(smask);
      smask &= smask - 1;
      const int l0 = sb * kSuper, nl = min(kSuper, nbox - l0);
      uint64_t lmask;
      // (R stays valid for this super-box's leaves and mini-boxes: the
      // radii only shrink)
      const float R = own_bounds(L, fminf(lim, b2), lane);
      {
        const int k = l0 + min(lane, nl - 1);
        const float4 lo = boxes[2 * k], hi = boxes[2 * k + 1];
        lmask = __ballot(lane < nl && k != own && near_own(L, split_m, lo, hi));
        wave_lds_sync();
        L.leaf_lo[lane] = lo;
        L.leaf_hi[lane] = hi;
        wave_lds_sync();
      }
      // the next leaf any lane needs (tested with the radii as they stand)
      auto next_leaf = [&]() -> int {
        while (lmask) {
          const int jl = __builtin_ctzll(lmask);
          lmask &= lmask - 1;
          if (__any(box_dist(L.leaf_lo[jl], L.leaf_hi[jl], p) <= fminf(lim, b2))) return jl;
        }
        return -1;
      };
      // a leaf's points (one per lane) and its mini-box bounds (lanes 0..15:
      // lo, hi of mini 0, lo, hi of mini 1, ...) are fetched one leaf ahead,
      // so their load overlaps the scan of the previous leaf
      float4 q = make_float4(0.f, 0.f, 0.f, 0.f), mb = q;
      auto fetch = [&](int jl) {
        const int b = l0 + jl;
        q = spts[min(b * kBox + lane, P - 1)];
        mb = minis[2 * (size_t)b * kM + min(lane, 2 * kM - 1)];
      };
      int jl = next_leaf();
      if (jl >= 0) fetch(jl);
      while (jl >= 0) {
        const int b = l0 + jl, n = min(kBox, P - b * kBox);
        wave_lds_sync();  // every lane is done reading the previous leaf
        L.pts[lane] = q;
        if (lane < 2 * kM) L.mini[lane] = mb;
        wave_lds_sync();
        // chosen before this leaf's scan shrinks the radii: a superset of
        // the leaves still needed, whose mini-boxes are re-tested below
        jl = next_leaf();
        if (jl >= 0) fetch(jl);
        // lanes 0..7: one mini-box each, tested against the grown own box
        const int mi = min(lane, kM - 1);
        const uint32_t mmask = (uint32_t)__ballot(lane < kM && lane * kMini < n &&
                                                  box_box(olo, ohi, L.mini[2 * mi], L.mini[2 * mi + 1]) <= R);
        scan_minis(L, mmask, n, lim, p, b0, b1, b2);
      }
    }
  }
}

// One wave = 64 consecutive Morton-ordered points = one leaf.  Each wave
// scans its own leaf first; its bound prunes almost every other leaf.  A
// lane whose own leaf and +-3 Morton neighbours lie far from it (a jump of
// the curve) would keep a radius many times its answer and drag its wave
// through a large part of the scene, so the walk runs in two phases:
//   1. radii capped at `cap` (16x the smallest own mini-box bound): a lane
//      that ends with b2 <= cap is exact (every mini-box skipped lay beyond
//      min(radius, cap) >= its final b2);
//   2. only if some lane ended above the cap: those lanes restart from their
//      own-leaf state with radius min(reject, phase-1 b2) (still an upper
//      bound of the answer), the finished lanes search nothing (radius -1)
//      and keep their phase-1 result.
__global__ __launch_bounds__(256) void k_knn(int P, const float4* __restrict__ spts,
                                             const uint32_t* __restrict__ idx, const float4* __restrict__ boxes,
                                             int nbox, const float4* __restrict__ minis,
                                             const float4* __restrict__ supers, int nsup, float* __restrict__ out) {
  __shared__ KnnWaveLds sl[4];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int s0 = blockIdx.x * 256 + threadIdx.x;
  if (blockIdx.x * 256 + w * 64 >= P) return;  // whole wave past the end (wave-uniform)
  const bool valid = s0 < P;
  const int s = valid ? s0 : P - 1;
  const float4 p = spts[s];
  float b0 = FLT_MAX, b1 = FLT_MAX, b2 = FLT_MAX;
  for (int i = max(0, s - 3); i <= min(P - 1, s + 3); ++i)
    if (i != s) update3(sqdist(p, spts[i]), b0, b1, b2);
  const float reject = b2;
  b0 = b1 = b2 = FLT_MAX;
  KnnWaveLds& L = sl[w];
  const int own = (blockIdx.x * 256 + w * 64) / kBox;
  const float4 olo = boxes[2 * own], ohi = boxes[2 * own + 1];
  L.pts[lane] = p;  // invalid lanes' copies lie past P and are never read
  if (lane < 2 * (kBox / kMini)) L.own[lane] = minis[2 * (size_t)own * (kBox / kMini) + lane];
  wave_lds_sync();
  scan_leaf(L.pts, own * kBox, min(kBox, P - own * kBox), s, p, b0, b1, b2);
  const float o0 = b0, o1 = b1, o2 = b2;  // own-leaf state (phase 2 restarts here)
  L.qp[lane] = p;
  own_bounds(L, fminf(reject, b2), lane);
  float cap = L.ownR[0];
#pragma unroll
  for (int m = 1; m < kBox / kMini; ++m) cap = fminf(cap, L.ownR[m]);
  cap *= 16.f;
  uint32_t split_m;
  {
    const int m = min(lane, kBox / kMini - 1);
    const float4 lo = L.own[2 * m], hi = L.own[2 * m + 1];
    const float ex = hi.x - lo.x, ey = hi.y - lo.y, ez = hi.z - lo.z;
    // (an empty mini-box of a partial last leaf has negative extents)
    split_m = (uint32_t)__ballot(lane < kBox / kMini && ex >= 0.f &&
                                 ex * ex + ey * ey + ez * ez > 36.f * fminf(L.ownR[m], cap));
  }
  // (one loop body for both phases keeps a single copy of the walk)
  float lim = fminf(reject, cap);
  bool done = false;
#pragma clang loop unroll(disable)
  for (int phase = 0;; ++phase) {
    float c0 = o0, c1 = o1, c2 = o2;
    walk(L, P, spts, boxes, nbox, minis, supers, nsup, own, olo, ohi, p, lane, lim, split_m, c0, c1, c2);
    if (!done) { b0 = c0; b1 = c1; b2 = c2; }
    if (phase == 1) break;
    done = b2 <= cap;
    if (!__any(!done)) break;
    lim = done ? -1.f : fminf(reject, b2);
  }
  if (valid) out[idx[s]] = (b0 + b1 + b2) / 3.0f;
}

}  // namespace

size_t knn_scratch_bytes(int P) { return KnnLayout((size_t)P).total; }

hipError_t launch_dist_cuda2(int P, const float* points, float* out, void* scratch, hipStream_t s) {
  if (P <= 0) return hipSuccess;
  const KnnLayout L((size_t)P);
  const int nparts = min(1024, (P + 255) / 256);
  hipLaunchKernelGGL(k_bbox_partial, dim3(nparts), dim3(256), 0, s, P, points, at<float>(scratch, L.part));
  hipLaunchKernelGGL(k_bbox_final, dim3(1), dim3(256), 0, s, nparts, at<float>(scratch, L.part),
                     at<float>(scratch, L.bbox));
  hipLaunchKernelGGL(k_morton, dim3((P + 255) / 256), dim3(256), 0, s, P, points, at<float>(scratch, L.bbox),
                     at<uint32_t>(scratch, L.codes));
  bool in_alt = false;
  hipError_t e = radix_sort_pairs(at<uint32_t>(scratch, L.codes), at<uint32_t>(scratch, L.codes_alt),
                                  at<uint32_t>(scratch, L.idx), at<uint32_t>(scratch, L.idx_alt), true, (size_t)P,
                                  kMortonSortLo, 30, at<uint32_t>(scratch, L.hist), at<uint32_t>(scratch, L.totals), s, &in_alt);
  if (e != hipSuccess) return e;
  const uint32_t* sidx = at<uint32_t>(scratch, in_alt ? L.idx_alt : L.idx);
  float4* spts = at<float4>(scratch, L.spts);
  hipLaunchKernelGGL(k_gather_sorted, dim3((P + 255) / 256), dim3(256), 0, s, P, points, sidx, spts);
  const int nbox = (P + kBox - 1) / kBox, nsup = (nbox + kSuper - 1) / kSuper;
  float4* boxes = at<float4>(scratch, L.boxes);
  float4* minis = at<float4>(scratch, L.minis);
  float4* supers = at<float4>(scratch, L.supers);
  hipLaunchKernelGGL(k_leaf_bounds, dim3((P + 255) / 256), dim3(256), 0, s, P, spts, boxes, minis);
  hipLaunchKernelGGL(k_bounds, dim3(nsup), dim3(256), 0, s, nbox, kSuper, boxes, 1, supers);
  hipLaunchKernelGGL(k_knn, dim3((P + 255) / 256), dim3(256), 0, s, P, spts, sidx, boxes, nbox, minis, supers, nsup,
                     out);
  return hipGetLastError();
}

}  // namespace wgsr
