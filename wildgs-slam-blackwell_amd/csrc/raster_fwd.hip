// Forward rasteriser stages for gfx950.
//
//   preprocess   one lane per Gaussian: cull, cov3D -> EWA cov2D -> conic,
//                radius + tile rectangle, SH -> RGB; writes a 48-byte splat
//                record per Gaussian (the only thing the tile loops read).
//   [depth sort] visible Gaussians by depth (stable by id)      -- sort.hip
//   [scan]       duplicate-slot offsets in depth order           -- sort.hip
//   duplicate    wave-cooperative expansion of every Gaussian's tile
//                rectangle into (tile, slot) pairs: each lane writes one pair,
//                so the writes of a wave are contiguous.
//   [tile sort]  stable sort of the pairs by tile id             -- sort.hip
//   ranges       per-tile [start, end) by binary search.
//   render       one wave64 per 16x16 tile (4 pixels per lane), splat records
//                staged in LDS 64 at a time and prefetched one batch ahead,
//                front-to-back alpha blending.
//
// Sorting by depth first and then stably by tile yields exactly upstream's
// (tile << 32 | depth) order (ties broken by Gaussian index) while the
// N-sized sort only moves tile ids.
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "wgsr_common.h"
#include "wgsr_internal.h"

namespace wgsr {

namespace {

constexpr float SH_C0 = 0.28209479177387814f;
constexpr float SH_C1 = 0.4886025119029199f;
__constant__ float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
__constant__ float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f,  -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

__device__ __forceinline__ f3 ldc(const float* sh, int k) { return mk3(sh[3 * k], sh[3 * k + 1], sh[3 * k + 2]); }

// SH -> RGB (upstream computeColorFromSH forward), clamp flags in bits 0..2.
// Every product and sum is written here, under contract(off) (the local
// lambdas included): no multiply-add of the colour can be fused, whatever the
// inlining context, so every preprocess kernel rounds the colour alike.
__device__ __forceinline__ f3 sh_to_rgb(int deg, const float* sh, f3 dir, uint32_t& clamp_bits) {
#pragma clang fp contract(off)
  auto term = [](float c, const float* v) -> f3 { return {c * v[0], c * v[1], c * v[2]}; };
  auto plus = [](f3 a, f3 b) -> f3 { return {a.x + b.x, a.y + b.y, a.z + b.z}; };
  auto minus = [](f3 a, f3 b) -> f3 { return {a.x - b.x, a.y - b.y, a.z - b.z}; };
  f3 r = term(SH_C0, sh);
  if (deg > 0) {
    const float x = dir.x, y = dir.y, z = dir.z;
    r = minus(plus(minus(r, term(SH_C1 * y, sh + 3)), term(SH_C1 * z, sh + 6)), term(SH_C1 * x, sh + 9));
    if (deg > 1) {
      const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
      r = plus(r, term(SH_C2[0] * xy, sh + 12));
      r = plus(r, term(SH_C2[1] * yz, sh + 15));
      r = plus(r, term(SH_C2[2] * (2.f * zz - xx - yy), sh + 18));
      r = plus(r, term(SH_C2[3] * xz, sh + 21));
      r = plus(r, term(SH_C2[4] * (xx - yy), sh + 24));
      if (deg > 2) {
        r = plus(r, term(SH_C3[0] * y * (3.f * xx - yy), sh + 27));
        r = plus(r, term(SH_C3[1] * xy * z, sh + 30));
        r = plus(r, term(SH_C3[2] * y * (4.f * zz - xx - yy), sh + 33));
        r = plus(r, term(SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy), sh + 36));
        r = plus(r, term(SH_C3[4] * x * (4.f * zz - xx - yy), sh + 39));
        r = plus(r, term(SH_C3[5] * z * (xx - yy), sh + 42));
        r = plus(r, term(SH_C3[6] * x * (xx - 3.f * yy), sh + 45));
      }
    }
  }
  r = plus(r, f3{0.5f, 0.5f, 0.5f});
  clamp_bits = (r.x < 0 ? 1u : 0u) | (r.y < 0 ? 2u : 0u) | (r.z < 0 ? 4u : 0u);
  return mk3(fmaxf(r.x, 0.f), fmaxf(r.y, 0.f), fmaxf(r.z, 0.f));
}

// compile-time loop: f(std::integral_constant<int, I>) for I in [I0, N)
template <int I0, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I0 < N) {
    f(std::integral_constant<int, I0>{});
    static_for<I0 + 1, N>(f);
  }
}

// One Gaussian of k_preprocess2; returns (rect area, exact list length, bins
// touched), 0 if culled.  The per-Gaussian words every Gaussian gets (radius,
// list length, tb, depth key) are returned in `w` (radius, cnt, tb, key) and
// stored once by the caller; the splat record, rect, row table and clamp bits
// only for visible Gaussians.
__device__ __forceinline__ uint3 preprocess_one(
    int P, int D, int M, const float* __restrict__ means, const float* __restrict__ scales,
    const float* __restrict__ rots, const float* __restrict__ opac, const float* __restrict__ shs,
    const float* __restrict__ colors, const float* __restrict__ cov_pre, float scale_mod,
    const float* __restrict__ viewm, const float* __restrict__ projm, const float* __restrict__ campos_p, int W,
    int H, float tanx, float tany, int gx, int gy, int prefiltered, float4* __restrict__ splat,
    ListRec* __restrict__ lrec, uint32_t* __restrict__ clamped,
    uint32_t* __restrict__ err_flag, int bshift,
    int i, const Cam& c, const f3 p, const f3 sc, const float4 q, const float o, const f3 sh_rgb,
    uint32_t sh_cbits, uint4& w, uint2& rcw, bool write_color = true, float4* ab = nullptr) {
#pragma clang fp contract(off)
  w = make_uint4(0u, 0u, 0u, 0xFFFFFFFFu);  // culled: radius 0, no list, key sorts last
  rcw = make_uint2(0u, 0u);

  const float4 hom = xform44(c.proj, p);
  const float pw = 1.0f / (hom.w + 0.0000001f);
  const f3 pproj = mk3(hom.x * pw, hom.y * pw, hom.z * pw);
  const f3 pv = xform43(c.view, p);
  if (pv.z <= kNearZ) {
    if (prefiltered) atomicOr(err_flag, 1u);
    return make_uint3(0u, 0u, 0u);
  }
  float cv[6];
  if (cov_pre) {
#pragma unroll
    for (int k = 0; k < 6; ++k) cv[k] = cov_pre[6 * (size_t)i + k];
  } else {
    cov3d_from(sc, scale_mod, q, cv);
  }
  float S[3][3];
  sym3(cv, S);
  float T[2][3];
  f3 tc;
  float xm, ym;
  ewa_T(c, pv, T, tc, xm, ym);
  float a, b, cc;
  cov2d(T, S, a, b, cc);
  const float det = a * cc - b * b;
  if (det == 0.0f) return make_uint3(0u, 0u, 0u);
  const float det_inv = 1.f / det;
  const float mid = 0.5f * (a + cc);
  const float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
  const float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
  const float my_radius = ceilf(3.f * sqrtf(fmaxf(l1, l2)));
  const float px = ndc2pix(pproj.x, W), py = ndc2pix(pproj.y, H);
  const int r = (int)my_radius;
  const int x0 = min(gx, max(0, (int)((px - r) / kTile)));
  const int y0 = min(gy, max(0, (int)((py - r) / kTile)));
  const int x1 = min(gx, max(0, (int)((px + r + kTile - 1) / kTile)));
  const int y1 = min(gy, max(0, (int)((py + r + kTile - 1) / kTile)));
  if ((x1 - x0) * (y1 - y0) == 0) return make_uint3(0u, 0u, 0u);

  f3 rgb = sh_rgb;  // (colours given: read below; SH colours: k_preprocess2 evaluates them after the geometry)
  uint32_t cbits = sh_cbits;
  if (colors) {
    rgb = mk3(colors[3 * i], colors[3 * i + 1], colors[3 * i + 2]);
    cbits = 0;
  }
  // Reach of the splat: o G >= 1/255  <=>  d^T conic d <= lim = 2 ln(255 o)
  // (G = exp(-d^T conic d / 2) <= 1, so lim < 0 means "reaches no pixel").
  // The render loops test each entry's ellipse against a wave's pixel
  // rectangle and skip entries that cannot reach it (pure culling).
  const float lim = (o >= kMinAlpha) ? 2.f * logf(255.f * o) : -1.f;
  // record: A = (mean x, mean y, conic xx, conic yy), B = (conic xy, opacity,
  // lim, 0), C = (r, g, b, depth) -- pairs laid out for packed math
  const float4 A = make_float4(px, py, kConicSq * (cc * det_inv), kConicSq * (a * det_inv));
  const float4 B = make_float4(kConicXY * (-b * det_inv), o, lim, 0.f);
  if (ab) {  // (the caller writes the whole record with its colour)
    ab[0] = A;
    ab[1] = B;
  } else {
    splat[3 * (size_t)i + 0] = A;
    splat[3 * (size_t)i + 1] = B;
  }
  if (write_color) splat[3 * (size_t)i + 2] = make_float4(rgb.x, rgb.y, rgb.z, pv.z);
  rcw = make_uint2((uint32_t)x0 | ((uint32_t)y0 << 16), (uint32_t)x1 | ((uint32_t)y1 << 16));
  // exact tile list length (row_span); upstream's num_rendered counts the rect
  const Reach rr = reach_of(A, B);
  uint32_t cnt = 0;
  uint4 tab = make_uint4(0u, 0u, 0u, 0u);
  for (int ty = y0; ty < y1; ++ty) {
    int xa;
    const uint32_t len = (uint32_t)row_span(rr, ty, x0, x1, xa);
    const int k = ty - y0;
    if (k < 4) {
      tab.x |= len << (8 * k);
      tab.z |= (uint32_t)(xa - x0) << (8 * k);
    } else if (k < kRowTab) {
      tab.y |= len << (8 * (k - 4));
      tab.w |= (uint32_t)(xa - x0) << (8 * (k - 4));
    }
    cnt += len;
  }
  lrec[i].tab = tab;
  if (write_color) clamped[i] = cbits;
  // bins of the rect (exact lists are per tile; a bin list holds every
  // Gaussian whose rect meets the bin, and the render waves cull the rest)
  const uint32_t nb = cnt == 0 ? 0u
                               : (uint32_t)((((x1 - 1) >> bshift) - (x0 >> bshift) + 1) *
                                            (((y1 - 1) >> bshift) - (y0 >> bshift) + 1));
  // tb: both < 2^16 (bin_shift() requires <= 65535 tiles); the key: pv.z > 0.2 > 0,
  // so float bits sort like the floats
  w = make_uint4((uint32_t)r, cnt, cnt | (nb << 16), __float_as_uint(pv.z));
  return make_uint3((uint32_t)((x1 - x0) * (y1 - y0)), cnt, nb);
}

// A preprocess wave's pair counts (upstream's num_rendered, exact pairs, bin
// pairs) and visible depth-key range into the counter block: one atomic per
// wave each, spread over kRectPairLanes words.  The wave sums / maxima are
// DPP row reductions + four readlanes (SGPR results, no LDS round trips);
// per-lane rect areas of 2^26 or more (images beyond ~17 Gpixel) take the
// 64-bit shuffle path.
__device__ __forceinline__ void wave_pair_counts(const uint3 ac, uint32_t khi, uint32_t knlo,
                                                 unsigned long long* __restrict__ rect_pairs,
                                                 unsigned long long* __restrict__ list_pairs,
                                                 unsigned long long* __restrict__ bin_pairs,
                                                 uint32_t* __restrict__ drange) {
  const uint32_t slot = blockIdx.x % kRectPairLanes;
  unsigned long long area, cnt, nbin;
  if (wave_any(ac.x >= (1u << 26))) {
    area = ac.x;
    cnt = ac.y;
    nbin = ac.z;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      area += __shfl_xor(area, off, 64);
      cnt += __shfl_xor(cnt, off, 64);
      nbin += __shfl_xor(nbin, off, 64);
    }
  } else {  // (list and bin counts never exceed the rect area)
    area = wave_total_u32(ac.x);
    cnt = wave_total_u32(ac.y);
    nbin = wave_total_u32(ac.z);
  }
  const uint32_t kh = wave_maximum_u32(khi), kn = wave_maximum_u32(knlo);
  if (threadIdx.x % 64 == 0) {
    atomicAdd(&rect_pairs[slot], area);
    atomicAdd(&list_pairs[slot], cnt);
    atomicAdd(&bin_pairs[slot], nbin);
    // the depth sort's key range (DepthKeyPlan): max key, max complement
    if (kh) atomicMax(&drange[slot], kh);
    if (kn) atomicMax(&drange[kRectPairLanes + slot], kn);
  }
}

constexpr int kPreWave = 64;

// ---- k_preprocess2: the SH slab streams into LDS while the geometry runs ----
// One wave of 64 Gaussians per workgroup.  The wave loads its parameters
// (one round trip for all four arrays), then queues its 64 rows' evaluated
// SH coefficients as LDS-DMA loads (global_load_lds: no VGPR holds them in
// flight), in a chunk-major layout [chunk][lane] (chunk = 4 floats when rows
// are 16-byte aligned, else 1) so that each lane later reads its own row
// conflict-free; runs the projection / covariance / rectangle / row-table
// work and writes the geometry records while the slab is in flight; only
// then does it wait for the slab and evaluate the colour -- for visible
// Gaussians only.  (The order matters: vmcnt retires in issue order, so with
// the slab queued first every parameter use waited for the whole slab.)
// Measured alternatives (all bit-identical): the slab staged before the
// geometry (k_preprocess, 90 us when this one was 86), SH coefficients in
// VGPRs (150 vs 103 us), the coalesced row-major slab (112 vs 102; round 5:
// 109.3 vs 102.5 us, and again 107.2 vs 101.1 with the parameters first and
// XOR-swizzled conflict-free LDS rows, although tools/ubench/pre_copy.hip's
// copy of this access shape runs 62 us row-major vs 92 chunk-major; a
// 16-row-group slab -- each load 16 rows x 64 contiguous bytes, rotated for
// conflict-free reads -- 103.7-108.0 vs 101.1-102.0 over three A/B pairs), one
// memory round trip per wave (106.7 vs 103.4), records staged through LDS
// for contiguous stores (115.8 vs 106.7).
template <int kD, int kCh>
__device__ __forceinline__ f3 sh_rgb_lds(const float* __restrict__ s_sh, int lane, f3 dir, uint32_t& cbits) {
  constexpr int K = (kD + 1) * (kD + 1), NF = 3 * K, NCH = (NF + kCh - 1) / kCh;
  float sh[NCH * kCh];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    if constexpr (kCh >= 4) {
      const float4 v = reinterpret_cast<const float4*>(s_sh)[k * 64 + lane];
      sh[4 * k] = v.x;
      sh[4 * k + 1] = v.y;
      sh[4 * k + 2] = v.z;
      sh[4 * k + 3] = v.w;
    } else {
      sh[k] = s_sh[k * 64 + lane];
    }
  }
  return sh_to_rgb(kD, sh, dir, cbits);
}

// kD: the evaluated SH degree (-1: no slab -- colours given, or no SH).  The
// degree is a template parameter so that the slab is a compile-time number of
// loads queued AFTER the parameter loads: vmcnt retires in issue order, and
// with the slab queued first (or a run-time trip count) the first parameter
// use waited for the whole slab, so nothing overlapped it.
// WGSR_PRE_LATE_SH (default 1): the SH slab is loaded after the geometry, by
// the visible rows only -- culled rows read no SH (17 % of the bench scene's
// rows; 1M / 1080p / SH3: 103.6 -> 102.3 us over two A/B pairs).  0: the slab
// is issued with the parameter loads, for every row, in flight during the
// geometry.
#ifndef WGSR_PRE_LATE_SH
#define WGSR_PRE_LATE_SH 1
#endif
// WGSR_PRE_AB_LATE (default 1): with SH colours, a visible row's whole 48-byte
// splat record is stored after its colour, in three back-to-back stores.  The
// geometry half used to be stored before the slab wait and the colour after
// it: by then many of the record's lines had left the L2, so they were
// written to HBM twice (write counters ~40 MB above the model at 1M).
#ifndef WGSR_PRE_AB_LATE
#define WGSR_PRE_AB_LATE 1
#endif
template <int kCh, int kD>
__global__ __launch_bounds__(kPreWave) void k_preprocess2(
    int P, int D, int M, const float* __restrict__ means, const float* __restrict__ scales,
    const float* __restrict__ rots, const float* __restrict__ opac, const float* __restrict__ shs,
    const float* __restrict__ colors, const float* __restrict__ cov_pre, float scale_mod,
    const float* __restrict__ viewm, const float* __restrict__ projm, const float* __restrict__ campos_p, int W,
    int H, float tanx, float tany, int gx, int gy, int prefiltered, float4* __restrict__ splat,
    ListRec* __restrict__ lrec, uint32_t* __restrict__ clamped,
    uint32_t* __restrict__ dkey, int32_t* __restrict__ radii, int32_t* __restrict__ n_touched,
    uint32_t* __restrict__ err_flag, unsigned long long* __restrict__ rect_pairs,
    unsigned long long* __restrict__ list_pairs, unsigned long long* __restrict__ bin_pairs, int bshift,
    uint32_t* __restrict__ tb, uint8_t* __restrict__ gflag, uint32_t* __restrict__ drange, const ZeroJob zero,
    uint32_t* __restrict__ meta) {
  extern __shared__ float s_sh[];  // nch x 64 x kCh floats (chunk-major)
  const int lane = threadIdx.x;
  const int i0 = blockIdx.x * kPreWave, i = i0 + lane;
  constexpr bool sh_on = kD >= 0;
  // the parameters first, in one basic block (clamped rows; with cov_pre the
  // scale / rotation loads read its first words and are discarded)
  const int ic = min(i, P - 1);
  const int ir = cov_pre ? 0 : ic;
  const float* __restrict__ sp = cov_pre ? cov_pre : scales;
  const float* __restrict__ rp = cov_pre ? cov_pre : rots;
  const f3 pl = mk3(means[3 * ic], means[3 * ic + 1], means[3 * ic + 2]);
  const f3 sl = mk3(sp[3 * ir], sp[3 * ir + 1], sp[3 * ir + 2]);
  const float4 ql = make_float4(rp[4 * ir], rp[4 * ir + 1], rp[4 * ir + 2], rp[4 * ir + 3]);
  const float ol = opac[ic];
  // an opaque use of every parameter: the four loads share one round trip
  // (none sinks into the branch below), completed before the slab is queued
  asm volatile("" ::"v"(pl.x), "v"(pl.y), "v"(pl.z), "v"(sl.x), "v"(sl.y), "v"(sl.z), "v"(ql.x), "v"(ql.y),
               "v"(ql.z), "v"(ql.w), "v"(ol));
  auto load_slab = [&]() {
    using lds_t = __attribute__((address_space(3))) void*;
    constexpr int kNch = (3 * ((kD < 0 ? 0 : kD) + 1) * ((kD < 0 ? 0 : kD) + 1) + kCh - 1) / kCh;
    const float* src = shs + (size_t)ic * (3 * M);
#pragma unroll
    for (int k = 0; k < kNch; ++k) {
      if constexpr (kCh == 4)
        __builtin_amdgcn_global_load_lds((const void*)(src + 4 * k), (lds_t)(s_sh + 256 * k), 16, 0, 0);
      else
        __builtin_amdgcn_global_load_lds((const void*)(src + k), (lds_t)(s_sh + 64 * k), 4, 0, 0);
    }
  };
  if constexpr (sh_on && !WGSR_PRE_LATE_SH) load_slab();  // then the slab, in flight while the geometry runs
  const f3 p = i < P ? pl : mk3(0.f, 0.f, 1.f);
  const float o = i < P ? ol : 0.f;
  const f3 sc = cov_pre ? mk3(1.f, 1.f, 1.f) : sl;
  const float4 q = cov_pre ? make_float4(1.f, 0.f, 0.f, 0.f) : ql;
  Cam c;
  load_cam(c, viewm, projm, W, H, tanx, tany);
  uint3 ac = make_uint3(0u, 0u, 0u);
  uint32_t khi = 0u, knlo = 0u;
  uint4 w = make_uint4(0u, 0u, 0u, 0xFFFFFFFFu);
  constexpr bool ab_late = sh_on && WGSR_PRE_AB_LATE;
  float4 ab[2];
  if (i < P) {
    uint2 rcw;
    ac = preprocess_one(P, D, M, means, scales, rots, opac, shs, colors, cov_pre, scale_mod, viewm, projm, campos_p,
                        W, H, tanx, tany, gx, gy, prefiltered, splat, lrec, clamped, err_flag, bshift, i, c, p,
                        sc, q, o, mk3(0.f, 0.f, 0.f), 0u, w, rcw, !sh_on, ab_late ? ab : nullptr);
    radii[i] = (int32_t)w.x;
    lrec[i].w = make_uint4(rcw.x, rcw.y, w.z, w.y);
    if (bshift) tb[i] = w.z;
    dkey[i] = w.w;
    if (w.w != 0xFFFFFFFFu) {
      khi = w.w;
      knlo = ~w.w;
    }
    n_touched[i] = 0;
    gflag[i] = 0;
  }
  if constexpr (sh_on && WGSR_PRE_LATE_SH) {
    if (i < P && w.x != 0u) load_slab();  // (visible rows only: culled rows read no SH)
  }
  if constexpr (sh_on) {
    __builtin_amdgcn_s_waitcnt(0);  // the slab has landed (one wave per workgroup)
    __syncthreads();
    if (i < P && w.x != 0u) {  // visible: the colour record
#pragma clang fp contract(off)
      f3 dir = sub3(p, mk3(campos_p[0], campos_p[1], campos_p[2]));
      const float len = sqrtf(dot3(dir, dir));
      dir = mk3(dir.x / len, dir.y / len, dir.z / len);
      uint32_t cbits = 0;
      const f3 rgb = sh_rgb_lds<(kD < 0 ? 0 : kD), kCh>(s_sh, lane, dir, cbits);
      if constexpr (ab_late) {
        splat[3 * (size_t)i + 0] = ab[0];
        splat[3 * (size_t)i + 1] = ab[1];
      }
      splat[3 * (size_t)i + 2] = make_float4(rgb.x, rgb.y, rgb.z, __uint_as_float(w.w));
      clamped[i] = cbits;
    }
  }
  wave_pair_counts(ac, khi, knlo, rect_pairs, list_pairs, bin_pairs, drange);
  zero_share(zero, blockIdx.x, gridDim.x, lane, kPreWave);
  if (blockIdx.x == 0 && lane == 0) {
    meta[1] = 0u;  // no capacity overflow (ImageLayout::meta)
    meta[2] = 0u;  // slots not (yet) known to follow the index order (k_duplicate_bins)
  }
}

// Expand the exact tile lists (row_span) of depth ranks [r0, r0 + 64) (one
// wave) into pairs: lane <-> pair, so the writes are contiguous.
__global__ __launch_bounds__(256) void k_duplicate(uint32_t P, int gx, const uint32_t* __restrict__ offs,
                                                   const uint32_t* __restrict__ sorted_g,
                                                   const ListRec* __restrict__ lrec,
                                                   const float4* __restrict__ splat, uint32_t* __restrict__ keys,
                                                   uint32_t* __restrict__ slot_g, uint8_t* __restrict__ pflag) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t r0 = (blockIdx.x * blockDim.x + threadIdx.x) - lane;
  if (r0 >= P) return;
  const uint32_t r = r0 + lane;
  const uint32_t my_off = offs[min(r, P)];
  const uint32_t start = offs[r0];
  const uint32_t end = offs[min(r0 + 64, P)];
  uint32_t g = 0, rlo = 0, rhi = 0;
  uint4 tab = make_uint4(0u, 0u, 0u, 0u);
  bool tall = false;  // rows beyond the row table (or a rect too wide for it)
  if (r < P) {
    g = sorted_g[r];
    if (offs[r + 1] > my_off) {
      const uint4 lw = lrec[g].w;
      const ushort4 rc = lr_rect(lw);
      rlo = lw.x;
      rhi = lw.y;
      tab = lrec[g].tab;
      tall = rc.w - rc.y > kRowTab || !rowtab_ok(rc);
    }
  }
  // rare: some Gaussian of the wave needs spans beyond its row table
  const bool any_tall = wave_any(tall);
  Reach rr{};
  if (any_tall && tall) rr = reach_of(splat[3 * (size_t)g], splat[3 * (size_t)g + 1]);
  for (uint32_t base = start; base < end; base += 64) {
    const uint32_t k = base + lane;
    const uint32_t kk = min(k, end - 1);
    int lo = 0, hi = 64;
#pragma unroll
    for (int it = 0; it < 6; ++it) {
      const int mid = (lo + hi) >> 1;
      const uint32_t v = __shfl(my_off, mid, 64);
      if (v <= kk) lo = mid; else hi = mid;
    }
    const uint32_t local = kk - __shfl(my_off, lo, 64);
    const uint32_t gg = __shfl(g, lo, 64);
    const uint32_t a = __shfl(rlo, lo, 64), b = __shfl(rhi, lo, 64);
    const int x0 = (int)(a & 0xFFFF), y0 = (int)(a >> 16), x1 = (int)(b & 0xFFFF), y1 = (int)(b >> 16);
    const uint4 tb = make_uint4(__shfl(tab.x, lo, 64), __shfl(tab.y, lo, 64), __shfl(tab.z, lo, 64),
                                __shfl(tab.w, lo, 64));
    // walk the table rows to the one holding list entry `local`
    const bool use_tab = x1 - x0 <= 255;
    const int nt = use_tab ? min(y1 - y0, kRowTab) : 0;
    uint32_t acc = 0, tx = 0, ty = 0;
    bool found = false;
    for (int row = 0; row < nt; ++row) {
      const uint32_t len = rowtab_len(tb, row);
      if (!found && local < acc + len) {
        ty = (uint32_t)(y0 + row);
        tx = (uint32_t)x0 + rowtab_x(tb, row) + (local - acc);
        found = true;
      }
      if (!found) acc += len;
    }
    if (any_tall) {  // wave-uniform: the shuffles need every lane
      Reach rg;
      rg.mx = __shfl(rr.mx, lo, 64); rg.my = __shfl(rr.my, lo, 64); rg.ca = __shfl(rr.ca, lo, 64);
      rg.cb = __shfl(rr.cb, lo, 64); rg.L = __shfl(rr.L, lo, 64); rg.det = __shfl(rr.det, lo, 64);
      rg.ey = __shfl(rr.ey, lo, 64); rg.dya = __shfl(rr.dya, lo, 64); rg.ica = __shfl(rr.ica, lo, 64);
      rg.ok = __shfl(rr.ok, lo, 64);
      for (int row = y0 + nt; !found && row < y1; ++row) {
        int xa;
        const uint32_t len = (uint32_t)row_span(rg, row, x0, x1, xa);
        if (local < acc + len) {
          ty = (uint32_t)row;
          tx = (uint32_t)xa + (local - acc);
          found = true;
        }
        acc += len;
      }
    }
    if (k < end) {
      keys[k] = ty * (uint32_t)gx + tx;
      slot_g[k] = gg;
      pflag[k] = 0;  // the backward's "record written" flag of this slot
    }
  }
}

// Exact tile mask of the splat inside bin (bx, by): bit rr 2^s + c for the
// tile (bx 2^s + c, by 2^s + rr) of its exact list (the row table, or
// row_span past it: the same spans k_duplicate enumerates).
__device__ __forceinline__ uint32_t bin_mask(int bx, int by, int bshift, int x0, int y0, int x1, int y1,
                                             const uint4& tab, bool tall, const Reach& rg) {
  const int B = 1 << bshift;
  const bool use_tab = x1 - x0 <= 255;
  uint32_t mask = 0;
  for (int rr = 0; rr < B; ++rr) {
    const int ty = (by << bshift) + rr;
    if (ty < y0 || ty >= y1) continue;
    const int kr = ty - y0;
    int xa, len;
    if (!tall || (use_tab && kr < kRowTab)) {
      xa = x0 + (int)rowtab_x(tab, kr);
      len = (int)rowtab_len(tab, kr);
    } else {
      len = row_span(rg, ty, x0, x1, xa);
    }
    const int cl = max(xa, bx << bshift), ch = min(xa + len, (bx << bshift) + B);
    if (ch > cl) mask |= ((1u << (ch - cl)) - 1u) << (rr * B + (cl - (bx << bshift)));
  }
  return mask;
}

// Exact tile mask inside bin (bx, by) of a splat whose rect rows all sit in
// its row table (not `tall`): the bin's 2^S rows' spans come out of the
// table as one byte run (rows above the rect shift in zeros, rows below it
// are zero in the table), each row a bit field of the mask.
template <int S>
__device__ __forceinline__ uint32_t bin_mask_tab(int bx, int by, int x0, int y0, const uint4& tab) {
  constexpr int B = 1 << S;
  const int kr0 = (by << S) - y0;  // in [-(B - 1), kRowTab - 1]
  const uint64_t L64 = ((uint64_t)tab.y << 32) | tab.x, X64 = ((uint64_t)tab.w << 32) | tab.z;
  // branch-free: one of the two shifts is by zero
  const uint32_t sr = 8u * (uint32_t)max(kr0, 0), sl = 8u * (uint32_t)max(-kr0, 0);
  const uint32_t lens = (uint32_t)((L64 >> sr) << sl);
  const uint32_t xs = (uint32_t)((X64 >> sr) << sl);
  const int d0 = x0 - (bx << S);  // the rect's left edge relative to the bin's
  uint32_t mask = 0;
#pragma unroll
  for (int rr = 0; rr < B; ++rr) {
    // row rr covers bin columns [lo, hi) (clamped to the bin; len >= 0 so
    // hi >= lo, and an empty or outside row gives lo == hi)
    const int xa = d0 + (int)((xs >> (8 * rr)) & 0xFFu);
    const int xe = xa + (int)((lens >> (8 * rr)) & 0xFFu);
    const int lo = min(max(xa, 0), B), hi = min(max(xe, 0), B);  // (v_med3_i32)
    mask |= (((1u << hi) - 1u) ^ ((1u << lo) - 1u)) << (rr * B);
  }
  return mask;
}

// Sort bins, after the dual scan's block sums (packed_scan_blocks: bsum[b]
// = exclusive prefix of (exact list length, bins touched) over the 256-rank
// blocks in depth order): each 256-thread workgroup finishes the scan for its
// ranks (thread <-> rank) -- slot_start[g], the backward's record slots, and
// the ranks' first bin pair -- zeroes the "record written" flags of its slots,
// and every wave expands its 64 ranks' bin rectangles into (key, Gaussian)
// pairs: lane <-> pair, contiguous writes.  key = bin id (low 16 bits: the
// sort's digits) | the Gaussian's exact tile list inside the bin as a
// 2^s x 2^s tile mask (bin_mask; high 16 bits, carried through the sort).  A
// Gaussian's pairs in row-major bin order (the stable sort by bin keeps the
// depth order inside each bin).
// A pair's owner (the rank whose rectangle it belongs to) is found without a
// search: each rank with bins writes its lane id at its first pair's place
// in a 64-entry LDS row, and an inclusive max-scan over the row (DPP) hands
// every pair its owner -- the last rank starting at or before it; the
// owner's record (rect, first pair, Gaussian, row table) is read
// from LDS where every rank staged it (three LDS reads per pair instead of a
// six-step shuffle search and ten shuffles).
constexpr int kDupScanThreads = kPackedScanTile;  // one rank per thread
template <int S>
__global__ __launch_bounds__(kDupScanThreads) void k_duplicate_bins(
    uint32_t P, int gbx, const ListRec* __restrict__ lrec, const uint32_t* __restrict__ sorted_g,
    const uint2* __restrict__ bsum, const uint2* __restrict__ bsup, const float4* __restrict__ splat,
    uint32_t* __restrict__ slot_start, uint8_t* __restrict__ pflag, uint32_t* __restrict__ keys,
    uint32_t* __restrict__ vals, const ZeroJob zero, uint32_t* __restrict__ meta, uint32_t cap_slots,
    uint32_t cap_pairs) {
  // (cap_slots / cap_pairs: the capacity-mode forward's buffer sizes -- writes
  // past them are dropped and the forward flags the overflow; ~0 otherwise)
  constexpr int NW = kDupScanThreads / 64;
  constexpr int bshift = S;
  __shared__ uint2 s_w[NW], s_p[NW];
  __shared__ uint4 s_ra[NW][64];    // per rank: rect lo | hi, first bin pair, Gaussian
  __shared__ uint4 s_rt[NW][64];    // per rank: row table
  __shared__ uint2 s_rw[NW][64];    // per rank: bin columns of the rect, their reciprocal (float bits)
  __shared__ uint32_t s_own[NW][64];
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const uint32_t r = blockIdx.x * kDupScanThreads + t;
  const bool in = r < P;
  // ranks in index order: Gaussian g's slots are [slot_start[g], slot_start[g + 1]) (ImageLayout::meta[2])
  if (blockIdx.x == 0 && t == 0) meta[2] = sorted_g ? 0u : 1u;
  // (unconditional loads of a clamped rank, the selects after: a load under
  // `in` would be waited for at its join.)
  const uint32_t rc = min(r, P - 1u);
  const uint32_t g0 = sorted_g ? sorted_g[rc] : rc;  // (null: index order)
  // the whole 32-byte list record in one round trip (row table + rect, tb,
  // list length: one cache line)
  uint4 lw = lrec[g0].w, tab = lrec[g0].tab;
  // the block prefix's inputs, issued behind the record loads (the scans
  // below wait for the records only; vmcnt counts in order): the earlier
  // superblocks' sums plus the earlier blocks of its own superblock
  uint2 pre = make_uint2(0u, 0u);
  if (bsup) {
    const uint32_t b = blockIdx.x, sb = b / kScanSupBlocks;
    for (uint32_t q = (uint32_t)t; q < sb; q += kDupScanThreads) {
      const uint2 x = bsup[(size_t)q * kScanSupStride];
      pre.x += x.x;
      pre.y += x.y;
    }
    if ((uint32_t)t < kScanSupBlocks && sb * kScanSupBlocks + t < b) {
      const uint2 x = bsum[sb * kScanSupBlocks + t];
      pre.x += x.x;
      pre.y += x.y;
    }
  } else {
    pre = bsum[blockIdx.x];
  }
  const uint32_t g = in ? g0 : 0u;
  if (!in) {
    lw = make_uint4(0u, 0u, 0u, 0u);
    tab = lw;
  }
  const uint32_t v = lw.z;
  const uint32_t cnt = v & 0xFFFFu, nb = v >> 16;
  uint32_t rlo = 0, rhi = 0;
  bool tall = false;
  if (nb) {
    const ushort4 rc = lr_rect(lw);
    rlo = lw.x;
    rhi = lw.y;  // exclusive
    tall = rc.w - rc.y > kRowTab || !rowtab_ok(rc);
  } else {
    tab = make_uint4(0u, 0u, 0u, 0u);
  }
  const uint32_t ic = wave_incl_scan(cnt), ib = wave_incl_scan(nb);
  if (lane == 63) s_w[w] = make_uint2(ic, ib);
  uint2 wb;  // this block's first slot / first bin pair
  if (bsup) {
    pre.x = wave_sum_u32(pre.x);
    pre.y = wave_sum_u32(pre.y);
    if (lane == 0) s_p[w] = pre;
    __syncthreads();
    wb = make_uint2(0u, 0u);
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      wb.x += s_p[k].x;
      wb.y += s_p[k].y;
    }
  } else {
    __syncthreads();
    wb = pre;
  }
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const uint2 x = s_w[k];
    if (k < w) { wb.x += x.x; wb.y += x.y; }
  }
  const uint2 wt = s_w[w];  // the wave's totals
  if (in) slot_start[g] = wb.x + ic - cnt;
  // the wave's slots are contiguous: dword stores for the aligned interior,
  // byte stores for the (< 4-byte) head and tail
  {
    const uint32_t f0 = wb.x, f1 = min(wb.x + wt.x, cap_slots);
    const uint32_t a0 = min((f0 + 3u) & ~3u, max(f1, f0)), a1 = max(f1 & ~3u, a0);
    if (lane < (int)(a0 - f0)) pflag[f0 + lane] = 0;
    if (lane < (int)(f1 - a1)) pflag[a1 + lane] = 0;
    uint32_t* pw = reinterpret_cast<uint32_t*>(pflag);
    for (uint32_t k = (a0 >> 2) + lane; k < (a1 >> 2); k += 64) pw[k] = 0u;
  }
  // scratch the bin sort needs zeroed (its superblock sums)
  zero_share(zero, blockIdx.x, gridDim.x, t, kDupScanThreads);
  if (wt.y == 0) return;  // wave-uniform; no barrier below
  const uint32_t my_off = wb.y + ib - nb;  // first bin pair of this rank
  const uint32_t start = wb.y, end = wb.y + wt.y;
  const bool any_tall = wave_any(tall);
  Reach rr{};
  if (any_tall && tall) rr = reach_of(splat[3 * (size_t)g], splat[3 * (size_t)g + 1]);
  // every rank's record, for its pairs' lanes
  s_ra[w][lane] = make_uint4(rlo, rhi, my_off, g);
  s_rt[w][lane] = tab;
  {  // the rect's bin-column count and its reciprocal, once per rank
    const int bw = (((int)(rhi & 0xFFFFu) - 1) >> bshift) - ((int)(rlo & 0xFFFFu) >> bshift) + 1;
    s_rw[w][lane] = make_uint2((uint32_t)bw, __float_as_uint(__builtin_amdgcn_rcpf((float)bw)));
  }
  uint32_t carry = 0;  // owner of the chunk's first pair (the first chunk: a rank starts there)
  for (uint32_t base = start; base < end; base += 64) {
    const uint32_t k = base + lane;
    const uint32_t kk = min(k, end - 1);
    // owner of pair kk: the highest lane with bins whose first pair is <= kk
    // (lanes without bins share their successor's offset: they do not write)
    s_own[w][lane] = lane == 0 ? carry : 0u;
    __builtin_amdgcn_wave_barrier();
    if (nb && my_off >= base && my_off < base + 64) s_own[w][my_off - base] = (uint32_t)lane;
    __builtin_amdgcn_wave_barrier();
    const uint32_t lo = wave_incl_max(s_own[w][lane]);
    carry = (uint32_t)__builtin_amdgcn_readlane((int)lo, 63);
    const uint4 ra = s_ra[w][lo];
    const uint32_t local = kk - ra.z;
    const uint32_t gg = ra.w;
    const int x0 = (int)(ra.x & 0xFFFFu), y0 = (int)(ra.x >> 16), x1 = (int)(ra.y & 0xFFFFu), y1 = (int)(ra.y >> 16);
    const uint4 tq = s_rt[w][lo];
    const uint2 rw = s_rw[w][lo];
    const int bx0 = x0 >> bshift, bw = (int)rw.x;
    // local / bw without the integer-division sequence: local < 2^16 (a
    // Gaussian's bins), so the float estimate is within one of the quotient
    int row = (int)((float)local * __uint_as_float(rw.y));
    int col = (int)local - row * bw;
    {  // (selects, not branches)
      const int dn = col < 0 ? 1 : 0, up = col >= bw ? 1 : 0;
      row += up - dn;
      col += (dn - up) * bw;
    }
    const int bx = bx0 + col, by = (y0 >> bshift) + row;
    uint32_t mask;
    if (!any_tall) {  // (wave-uniform) every owner's rows sit in its row table
      mask = bin_mask_tab<S>(bx, by, x0, y0, tq);
    } else {
      const bool tl = __shfl((int)tall, (int)lo, 64) != 0;
      Reach rg;  // (the shuffles need every lane)
      rg.mx = __shfl(rr.mx, lo, 64); rg.my = __shfl(rr.my, lo, 64); rg.ca = __shfl(rr.ca, lo, 64);
      rg.cb = __shfl(rr.cb, lo, 64); rg.L = __shfl(rr.L, lo, 64); rg.det = __shfl(rr.det, lo, 64);
      rg.ey = __shfl(rr.ey, lo, 64); rg.dya = __shfl(rr.dya, lo, 64); rg.ica = __shfl(rr.ica, lo, 64);
      rg.ok = __shfl(rr.ok, lo, 64);
      mask = tl ? bin_mask(bx, by, bshift, x0, y0, x1, y1, tq, true, rg) : bin_mask_tab<S>(bx, by, x0, y0, tq);
    }
    if (k < end && k < cap_pairs) {
      keys[k] = (uint32_t)(by * gbx + bx) | (mask << 16);
      vals[k] = gg;
    }
    __builtin_amdgcn_wave_barrier();  // (the next chunk's owner row is rewritten)
  }
}

// [start, end) of every bin in the bin-sorted keys (upstream's
// identifyTileRanges on bin ids): one thread per entry, bins with no entry
// keep the zero range written before the launch.
__global__ __launch_bounds__(256) void k_bin_bounds(const uint32_t* __restrict__ skeys, uint32_t NB,
                                                    uint2* __restrict__ bounds) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= NB) return;
  const uint32_t b = skeys[e] & 0xFFFFu;
  if (e == 0 || (skeys[e - 1] & 0xFFFFu) != b) bounds[b].x = e;
  if (e + 1 == NB || (skeys[e + 1] & 0xFFFFu) != b) bounds[b].y = e + 1;
}

// One workgroup per (bin, row of its tiles): the exact lists of the row's
// 2^s tiles, in depth order, out of the bin's sorted entries -- an entry
// belongs to tile c if bit c of its key's row mask is set; a block-wide
// stable compaction per tile (one ballot per wave, a cross-wave prefix)
// keeps the order, kExpThreads entries per step (the next step's keys and
// ids in flight).  Tile (r, c) of a bin whose entries sit at [lo, hi) writes
// at lists[2^2s lo + (r 2^s + c) (hi - lo) ...], a region as long as the
// bin's list: no count pass, no overlap.  (Measured at 1M/1080p: 256
// threads 44 us; one wave per row 73 us -- a bin's ~2000 entries then take
// ~35 dependent steps; 512 threads 55 us -- fewer workgroups in flight.)
constexpr int kExpThreads = 256;
__global__ __launch_bounds__(kExpThreads) void k_expand_bins(const uint32_t* __restrict__ skeys,
                                                             const uint32_t* __restrict__ sgid,
                                                             const uint2* __restrict__ bounds, int gx, int gy,
                                                             int bshift, int gbx, uint32_t* __restrict__ lists,
                                                             uint2* __restrict__ ranges,
                                                             uint32_t* __restrict__ tile_len,
                                                             uint32_t* __restrict__ meta) {
  constexpr int NW = kExpThreads / 64;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  if (blockIdx.x == 0 && t == 0) meta[0] = 1u;  // the lists are the sort-bin region
  const int B = 1 << bshift;
  // (an XCD-aware mapping -- the 2^s row workgroups of a bin on one XCD, so
  // that the bin comes from HBM once -- measured 31.5 vs 30.8 us: the rows'
  // re-reads already hit the last-level cache)
  const uint32_t bin = blockIdx.x >> bshift;
  const int r = (int)(blockIdx.x & (uint32_t)(B - 1));
  const int bx = (int)(bin % (uint32_t)gbx), by = (int)(bin / (uint32_t)gbx);
  const int ty = (by << bshift) + r;
  if (ty >= gy) return;  // block-uniform
  const uint2 bb = bounds[bin];
  const uint32_t lo = bb.x, hi = bb.y, len = hi - lo;
  const size_t base0 = ((size_t)lo << (2 * bshift)) + (size_t)(r << bshift) * len;
  const uint32_t shift = 16u + ((uint32_t)r << bshift), rmask = (1u << B) - 1u;
  uint32_t count[4] = {0u, 0u, 0u, 0u};
  // the step's per-wave counts of each tile as four 16-bit fields of one
  // 64-bit LDS word (<= 4 x 64 entries per field): each wave's cross-wave
  // prefix is three conditional 64-bit adds instead of 16 LDS reads and 32
  // adds; the words are double-buffered by step parity, so a step needs one
  // barrier (a wave rewrites a buffer only after the next step's barrier,
  // which every wave passes after reading it); stores through a uniform base
  // pointer with 32-bit offsets.  (Measured: 31.2 -> 28.5 us at 1M / 1080p
  // against per-wave LDS counts with two barriers per step; two entries per
  // thread per step: 35.5 us.)
  __shared__ unsigned long long s_wp[2][NW];
  uint32_t* const out0 = lists + base0;
  uint32_t key = lo + t < hi ? skeys[lo + t] : 0u, gid = lo + t < hi ? sgid[lo + t] : 0u;
  asm volatile("" ::"v"(key), "v"(gid));
  int par = 0;
  for (uint32_t e0 = lo; e0 < hi; e0 += kExpThreads, par ^= 1) {
    const uint32_t bits = (key >> shift) & rmask, my_gid = gid;
    const uint32_t e1 = e0 + kExpThreads + t;
    key = e1 < hi ? skeys[e1] : 0u;
    gid = e1 < hi ? sgid[e1] : 0u;
    uint64_t m[4];
    unsigned long long packed = 0ull;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      m[c] = wave_ballot(c < B && ((bits >> c) & 1u));
      packed |= (unsigned long long)__popcll(m[c]) << (16 * c);
    }
    if (lane == 0) s_wp[par][w] = packed;
    __syncthreads();
    unsigned long long off = 0ull, tot = 0ull;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      const unsigned long long v = s_wp[par][k];
      off += k < w ? v : 0ull;
      tot += v;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c >= B) break;
      if ((bits >> c) & 1u)
        out0[(uint32_t)c * len + count[c] + (uint32_t)((off >> (16 * c)) & 0xFFFFull) + lanes_below(m[c])] = my_gid;
      count[c] += (uint32_t)((tot >> (16 * c)) & 0xFFFFull);
    }
    asm volatile("" ::"v"(key), "v"(gid));
  }
  if (t < B) {
    const int tx = (bx << bshift) + t;
    if (tx < gx) {
      const uint32_t tile = (uint32_t)ty * (uint32_t)gx + (uint32_t)tx;
      const size_t b0 = base0 + (size_t)t * len;
      uint32_t c = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) c = k == t ? count[k] : c;
      ranges[tile] = make_uint2((uint32_t)b0, (uint32_t)b0 + c);
      tile_len[tile] = c;
    }
  }
}

// ---- per-bin depth sort (the default with sort bins) ---------------------------
// With the Gaussians duplicated in INDEX order (no global depth sort), the
// stable bin sort leaves every bin's entries in index order, one entry per
// Gaussian.  Sorting each bin stably by depth key then yields exactly the
// order a stable global depth sort leaves inside the bin: depth bits, ties by
// Gaussian index -- upstream's (tile | depth) key order with cub's stable tie
// order.  One 512-thread workgroup per bin: the bin's depth
// keys minus their minimum (R bits) are LSD-radix sorted in LDS, ceil(R / 9)
// stable passes of <= 9-bit digits, each entry's position in the bin riding
// along; the (key, Gaussian) pairs are then gathered in that order into the
// spare key / payload buffers.  A bin of more than kBdsCap entries runs the
// same passes chunk by chunk through global scratch (the sort-bin list
// region, free until k_expand_bins writes it).
// (512 threads, up to 10 entries per lane in steps of one: 1024 threads with
// 1, 2, 4, 7 entries per lane measured 42-46 vs 33 us at 1M / 1080p)
constexpr int kBdsThreads = 512, kBdsWaves = kBdsThreads / 64, kBdsItems = 10;
constexpr int kBdsCap = kBdsThreads * kBdsItems;  // entries sorted in LDS
constexpr int kBdsMaxBits = 9, kBdsDigits = 1 << kBdsMaxBits;
static_assert(kBdsDigits <= kBdsThreads, "threads t < kBdsDigits own digit t");
__device__ __forceinline__ bool bds_owns_digit() { return (int)threadIdx.x < kBdsDigits; }

// Peer groups (the wave's lanes holding the same digit) from per-(wave,
// digit) 64-bit lane masks in LDS: one ds_or_b64 + one read per entry group
// instead of one ballot and a 64-bit select per digit bit.  A wave's LDS
// instructions complete in order, so every lane's OR lands before any lane's
// read, and every read before the clear behind it.
// The lane-mask table shares LDS with the staging buffer (a pass ranks with
// the table, then scatters into the buffer; the table is zeroed again before
// the next pass) -- 61 instead of 93 KB per 512-thread workgroup, two
// workgroups per CU: the 1M frame's 510 bins in one round.  (Peer groups by
// ballots: 73 vs 45.5 us at 1M, round 3.)
struct BdsLds {
  union {
    uint2 buf[kBdsCap];                                // (depth key, position in the bin)
    unsigned long long match[kBdsWaves][kBdsDigits];  // lane masks per digit (zero between uses)
  };
  uint32_t wcnt[kBdsWaves][kBdsDigits];   // per wave digit counts, then their prefix over waves
  uint32_t base[kBdsDigits];              // per digit: first slot
  uint32_t tmp[kBdsWaves];
  uint32_t rng[2][kBdsWaves];
  uint32_t etot[kBdsWaves][16];           // emit: per-wave entries per tile of the bin
  uint32_t erun[16];                      // emit: entries per tile emitted so far
};

// The bin's exact per-tile lists, emitted straight from the depth-sorted bin
// (what k_expand_bins does from a global copy of it): tile k = r 2^s + c of
// the bin gets, in depth order, every entry whose key has bit 16 + k set, at
// lists[2^2s lo + k n + ...] (n = the bin's length: no count pass, no
// overlap).  One chunk: wave w's lanes hold sorted positions (w JN + j) 64 +
// lane of it in m[j] (the tile mask, 0 if none) and g[j] (the Gaussian);
// per-wave counts per tile first, their prefix over the waves, then a
// stable per-tile compaction (one ballot per (entry group, tile)).
struct BdsEmit {
  uint32_t* __restrict__ lists;
  uint2* __restrict__ ranges;
  uint32_t* __restrict__ tile_len;
  uint32_t* __restrict__ meta;
  int gx, gy, bshift, gbx;
};

template <int JN>
__device__ __forceinline__ void bds_emit_chunk(BdsLds& L, const uint32_t (&m)[JN], const uint32_t (&g)[JN],
                                               uint32_t cnt, int NT, uint32_t* __restrict__ out, uint32_t n) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t mine = 0;  // lane k < NT: this wave's entries of tile k
  static_for<0, JN>([&](auto J) {
    constexpr int j = decltype(J)::value;
    if ((uint32_t)(w * JN + j) * 64u < cnt) {  // wave-uniform
      const uint32_t mj = m[j];
#pragma unroll 1
      for (int k = 0; k < NT; ++k) {  // (k: an SGPR)
        const uint64_t b = wave_ballot((mj >> k) & 1u);
        mine += lane == k ? (uint32_t)__popcll(b) : 0u;
      }
    }
  });
  if (lane < 16) L.etot[w][lane] = mine;
  __syncthreads();
  uint32_t pre = 0;  // lane k: first slot of this wave's entries of tile k
  if (lane < NT) {
    pre = L.erun[lane];
    for (int q = 0; q < w; ++q) pre += L.etot[q][lane];
  }
  static_for<0, JN>([&](auto J) {
    constexpr int j = decltype(J)::value;
    if ((uint32_t)(w * JN + j) * 64u < cnt) {
      const uint32_t mj = m[j], gj = g[j];
#pragma unroll 1
      for (int k = 0; k < NT; ++k) {
        const bool bit = (mj >> k) & 1u;
        const uint64_t b = wave_ballot(bit);
        if (b != 0) {  // wave-uniform
          const uint32_t base = (uint32_t)__builtin_amdgcn_readlane((int)pre, k);
          if (bit) out[(size_t)k * n + base + lanes_below(b)] = gj;
          pre += lane == k ? (uint32_t)__popcll(b) : 0u;
        }
      }
    }
  });
  __syncthreads();  // every wave has read erun
  if (w == kBdsWaves - 1 && lane < NT) L.erun[lane] = pre;  // the last wave's end = the running totals
  __syncthreads();
}

// the bin's ranges / list lengths (and the lists' location flag), after its last chunk
__device__ __forceinline__ void bds_emit_ranges(const BdsLds& L, const BdsEmit& E, uint32_t bin, uint32_t lo,
                                                uint32_t n) {
  const int t = threadIdx.x;
  const int B = 1 << E.bshift;
  if (bin == 0 && t == 0) E.meta[0] = 1u;  // the lists are the sort-bin region
  if (t < B * B) {
    const int r = t >> E.bshift, c = t & (B - 1);
    const int bx = (int)(bin % (uint32_t)E.gbx), by = (int)(bin / (uint32_t)E.gbx);
    const int tx = (bx << E.bshift) + c, ty = (by << E.bshift) + r;
    if (tx < E.gx && ty < E.gy) {
      const uint32_t tile = (uint32_t)ty * (uint32_t)E.gx + (uint32_t)tx;
      const uint32_t b0 = (lo << (2 * E.bshift)) + (uint32_t)t * n;
      const uint32_t c_t = n ? L.erun[t] : 0u;
      E.ranges[tile] = make_uint2(b0, b0 + c_t);
      E.tile_len[tile] = c_t;
    }
  }
}

__device__ __forceinline__ uint32_t bds_excl_scan(uint32_t v, uint32_t* s_tmp, uint32_t* total) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t inc = wave_incl_scan(v);
  if (lane == 63) s_tmp[w] = inc;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kBdsWaves; ++i) {
    const uint32_t x = s_tmp[i];
    base += i < w ? x : 0u;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return base + inc - v;
}

// wave w owns the cn entries' slots [w pw, w pw + pw) (pw a multiple of 64,
// so all eight waves share the work), walked 64 at a time: ranks follow slot
// order (stable).  pk[j] packs the entry's position in the bin (bits 0-12),
// its digit (13-21) and its rank among the wave's entries of that digit
// (22-31, < 14 x 64); bds_rank fills bits 13-31.
constexpr int kBdsPosBits = 13, kBdsRankShift = kBdsPosBits + kBdsMaxBits;
static_assert(kBdsCap <= (1 << kBdsPosBits) && kBdsItems * 64 <= (1 << (32 - kBdsRankShift)), "pk packing");
__device__ __forceinline__ uint32_t bds_digit(uint32_t pk) { return (pk >> kBdsPosBits) & (kBdsDigits - 1); }
template <int JN>
__device__ __forceinline__ void bds_rank(BdsLds& L, uint32_t cn, uint32_t mn, int shift, int bits,
                                         const uint32_t (&k)[JN], uint32_t (&pk)[JN]) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t mask = (1u << bits) - 1u;
#pragma unroll
  for (int j = 0; j < JN; ++j) {
    const uint32_t le = (uint32_t)(w * JN + j) * 64u + (uint32_t)lane;
    const bool valid = le < cn;
    const uint32_t d = ((k[j] - mn) >> shift) & mask;
    (void)bits;
    if (valid) atomicOr(&L.match[w][d], 1ull << lane);
    const uint64_t peers = valid ? L.match[w][d] : 0ull;
    if (valid) L.match[w][d] = 0ull;
    const int leader = __ffsll((unsigned long long)peers) - 1;
    uint32_t old = 0;
    if (valid && lane == leader) old = atomicAdd(&L.wcnt[w][d], (uint32_t)__popcll(peers));
    old = (uint32_t)__shfl((int)old, leader & 63, 64);
    const uint32_t rk = old + lanes_below(peers);
    pk[j] = (pk[j] & ((1u << kBdsPosBits) - 1u)) | (d << kBdsPosBits) | (rk << kBdsRankShift);
    __builtin_amdgcn_sched_barrier(0);  // one entry group at a time: few live registers
  }
}
__device__ __forceinline__ uint32_t bds_slot(const BdsLds& L, uint32_t pk) {
  const int w = threadIdx.x >> 6;
  const uint32_t d = bds_digit(pk);
  return L.base[d] + L.wcnt[w][d] + (pk >> kBdsRankShift);
}

// thread t (digit t): the waves' counts -> their exclusive prefix in place;
// returns the digit's total
__device__ __forceinline__ uint32_t bds_wave_prefix(BdsLds& L) {
  const int t = threadIdx.x;
  uint32_t run = 0;
  if (!bds_owns_digit()) return 0u;
#pragma unroll
  for (int q = 0; q < kBdsWaves; ++q) {
    const uint32_t x = L.wcnt[q][t];
    L.wcnt[q][t] = run;
    run += x;
  }
  return run;
}

// Scratch written by other waves of this workgroup in the previous pass: the
// workgroup barrier orders it (same CU, so the vector L1 is coherent for
// them; an agent-scope fence would write back and invalidate the whole L2).
__device__ __forceinline__ uint2 bds_load_scratch(const uint2* p) { return *p; }

// the bin's key range over the workgroup -> (min key, R = bits of the span)
__device__ __forceinline__ uint32_t bds_range(BdsLds& L, uint32_t mn, uint32_t mx, int& R) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    mn = min(mn, (uint32_t)__shfl_xor((int)mn, off, 64));
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, off, 64));
  }
  if (lane == 0) {
    L.rng[0][w] = mn;
    L.rng[1][w] = mx;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kBdsWaves; ++q) {
    mn = min(mn, L.rng[0][q]);
    mx = max(mx, L.rng[1][q]);
  }
  const uint32_t span = mx - mn;
  R = span ? 32 - __clz((int)span) : 0;
  return mn;
}
__device__ __forceinline__ void bds_plan(int R, int& passes, int& pbits) {
  passes = (R + kBdsMaxBits - 1) / kBdsMaxBits;
  pbits = passes ? (R + passes - 1) / passes : 0;
}

// a bin of n <= 64 JN x kBdsWaves entries: wave w owns slots [w JN 64,
// (w + 1) JN 64), JN entries per lane in registers, every pass ranked in LDS
template <int JN>
__device__ __forceinline__ void bds_small(BdsLds& L, const uint32_t* __restrict__ skeys,
                                          const uint32_t* __restrict__ sgid, const uint32_t* __restrict__ sdep,
                                          const uint32_t* __restrict__ gdep, uint32_t lo, uint32_t n,
                                          uint32_t* __restrict__ okeys, uint32_t* __restrict__ ogid, bool E,
                                          const BdsEmit& EM) {
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  constexpr uint32_t kPosMask = (1u << kBdsPosBits) - 1u;
  uint32_t k[JN], pk[JN];
  uint32_t mn = 0xFFFFFFFFu, mx = 0u;
  // (loads of clamped positions, all issued before any is used: a load under
  // `le < n` is waited for at its join, one round trip per j)
  if (gdep) {  // (uniform) the Gaussians' depth keys through the bin's ids: two round trips
#pragma unroll
    for (int j = 0; j < JN; ++j) k[j] = sgid[lo + min((uint32_t)(w * JN + j) * 64u + (uint32_t)lane, n - 1u)];
#pragma unroll
    for (int j = 0; j < JN; ++j) k[j] = gdep[k[j]];
  } else {
#pragma unroll
    for (int j = 0; j < JN; ++j) k[j] = sdep[lo + min((uint32_t)(w * JN + j) * 64u + (uint32_t)lane, n - 1u)];
  }
#pragma unroll
  for (int j = 0; j < JN; ++j) {
    const uint32_t le = (uint32_t)(w * JN + j) * 64u + (uint32_t)lane;
    pk[j] = le;
    k[j] = le < n ? k[j] : 0u;
    if (le < n) {
      mn = min(mn, k[j]);
      mx = max(mx, k[j]);
    }
  }
  int R, npass, pbits;
  mn = bds_range(L, mn, mx, R);
  bds_plan(R, npass, pbits);
  for (int p = 0; p < npass; ++p) {
    const int shift = p * pbits, bits = min(pbits, R - shift);
    bds_rank<JN>(L, n, mn, shift, bits, k, pk);
    __syncthreads();
    uint32_t all;
    const uint32_t ex = bds_excl_scan(bds_wave_prefix(L), L.tmp, &all);
    if (bds_owns_digit()) L.base[t] = ex;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      const uint32_t le = (uint32_t)(w * JN + j) * 64u + (uint32_t)lane;
      if (le < n) L.buf[bds_slot(L, pk[j])] = make_uint2(k[j], pk[j] & kPosMask);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      const uint32_t le = (uint32_t)(w * JN + j) * 64u + (uint32_t)lane;
      if (le < n) {
        const uint2 kv = L.buf[le];
        k[j] = kv.x;
        pk[j] = kv.y;
      }
    }
#pragma unroll
    for (int q = 0; q < kBdsWaves; ++q)
      if (bds_owns_digit()) L.wcnt[q][t] = 0u;
    if (p + 1 < npass) {  // the next pass ranks with the table the buffer overwrote
      __syncthreads();
      for (int i = t; i < kBdsWaves * kBdsDigits; i += kBdsThreads) (&L.match[0][0])[i] = 0ull;
    }
    __syncthreads();
  }
  if (E) {  // the per-tile lists straight from the sorted bin
    uint32_t m[JN], g[JN];
    const uint32_t tmask = (1u << (1 << (2 * EM.bshift))) - 1u;
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      const uint32_t le = (uint32_t)(w * JN + j) * 64u + (uint32_t)lane;
      const uint32_t q = le < n ? pk[j] & kPosMask : 0u;  // (unconditional loads, as above)
      m[j] = skeys[lo + q];
      g[j] = sgid[lo + q];
    }
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      const uint32_t le = (uint32_t)(w * JN + j) * 64u + (uint32_t)lane;
      m[j] = le < n ? (m[j] >> 16) & tmask : 0u;
      g[j] = le < n ? g[j] : 0u;
    }
    if (t < 16) L.erun[t] = 0u;
    __syncthreads();
    bds_emit_chunk<JN>(L, m, g, n, 1 << (2 * EM.bshift), EM.lists + ((size_t)lo << (2 * EM.bshift)), n);
    return;
  }
  // every gather load issued before the first store (unconditional, clamped)
  uint32_t ok[JN], og[JN];
#pragma unroll
  for (int j = 0; j < JN; ++j) {
    const uint32_t le = (uint32_t)(w * JN + j) * 64u + (uint32_t)lane;
    const uint32_t q = le < n ? pk[j] & kPosMask : 0u;
    pk[j] = q;
    ok[j] = okeys ? skeys[lo + q] : 0u;  // (uniform; null: the stable argsort of k_argsort_small)
    og[j] = sgid ? sgid[lo + q] : q;
  }
#pragma unroll
  for (int j = 0; j < JN; ++j) {
    const uint32_t le = (uint32_t)(w * JN + j) * 64u + (uint32_t)lane;
    if (le < n) {
      if (okeys) okeys[lo + le] = ok[j];
      ogid[lo + le] = og[j];
    }
  }
}

// the emit of a bin beyond the LDS tile: chunks of JN x kBdsThreads sorted
// positions, their bin positions from the final pass's scratch (fin; null:
// already in order), running per-tile counts across the chunks
template <int JN>
__device__ __forceinline__ void bds_emit_big(BdsLds& L, const uint32_t* __restrict__ skeys,
                                             const uint32_t* __restrict__ sgid, const uint2* fin, uint32_t lo,
                                             uint32_t n, const BdsEmit& E) {
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const uint32_t tmask = (1u << (1 << (2 * E.bshift))) - 1u;
  constexpr uint32_t kChunk = JN * kBdsThreads;
  if (t < 16) L.erun[t] = 0u;
  __syncthreads();
  uint32_t* out = E.lists + ((size_t)lo << (2 * E.bshift));
  for (uint32_t c0 = 0; c0 < n; c0 += kChunk) {
    const uint32_t cn = min(kChunk, n - c0);
    uint32_t m[JN], g[JN];
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      const uint32_t le = (uint32_t)(w * JN + j) * 64u + (uint32_t)lane;
      m[j] = 0u;
      g[j] = 0u;
      if (le < cn) {
        const uint32_t q = fin ? bds_load_scratch(fin + c0 + le).y : c0 + le;
        m[j] = (skeys[lo + q] >> 16) & tmask;
        g[j] = sgid[lo + q];
      }
    }
    bds_emit_chunk<JN>(L, m, g, cn, 1 << (2 * E.bshift), out, n);
  }
}

// a bin beyond the LDS tile: each pass counts its digits over the whole bin,
// then ranks kBdsCap-entry chunks in order with running digit bases, the
// (key, position) pairs ping-ponging through global scratch
__device__ __forceinline__ void bds_big(BdsLds& L, const uint32_t* __restrict__ skeys, const uint32_t* __restrict__ sgid,
                                     const uint32_t* __restrict__ gdep, uint32_t lo, uint32_t n, uint32_t NL,
                                     uint32_t* __restrict__ okeys, uint32_t* __restrict__ ogid, uint2* scratch,
                                     bool E, const BdsEmit& EM) {
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  uint32_t mn = 0xFFFFFFFFu, mx = 0u;
  auto dep = [&](uint32_t e) { return gdep[sgid[lo + e]]; };
  for (uint32_t e = (uint32_t)t; e < n; e += kBdsThreads) {
    const uint32_t x = dep(e);
    mn = min(mn, x);
    mx = max(mx, x);
  }
  int R, passes, pbits;
  mn = bds_range(L, mn, mx, R);
  bds_plan(R, passes, pbits);
  constexpr int JN = 7;  // (chunks of half the LDS tile: fewer registers)
  if (passes == 0) {
    if (E) {
      bds_emit_big<JN>(L, skeys, sgid, nullptr, lo, n, EM);
      return;
    }
    for (uint32_t e = (uint32_t)t; e < n; e += kBdsThreads) {
      okeys[lo + e] = skeys[lo + e];
      ogid[lo + e] = sgid[lo + e];
    }
    return;
  }
  constexpr uint32_t kChunk = JN * kBdsThreads;
  uint2* bufA = scratch + lo;
  uint2* bufB = scratch + NL + lo;
  for (int p = 0; p < passes; ++p) {
    const int shift = p * pbits, bits = min(pbits, R - shift);
    const uint32_t mask = (1u << bits) - 1u;
    const uint2* src = (p & 1) ? bufA : bufB;  // pass p - 1's output
    uint2* dst = (p & 1) ? bufB : bufA;
    auto load = [&](uint32_t e) -> uint2 {
      return p == 0 ? make_uint2(dep(e), e) : bds_load_scratch(src + e);
    };
    if (bds_owns_digit()) L.base[t] = 0u;
    __syncthreads();
    for (uint32_t e = (uint32_t)t; e < n; e += kBdsThreads) atomicAdd(&L.base[((load(e).x - mn) >> shift) & mask], 1u);
    __syncthreads();
    {
      uint32_t all;
      const uint32_t c = bds_owns_digit() ? L.base[t] : 0u;
      const uint32_t ex = bds_excl_scan(c, L.tmp, &all);
      if (bds_owns_digit()) L.base[t] = ex;
    }
    __syncthreads();
    for (uint32_t c0 = 0; c0 < n; c0 += kChunk) {
      const uint32_t cn = min(kChunk, n - c0);
      uint32_t k[JN], pk[JN], pos[JN];  // (positions beyond the 13 bits of pk)
#pragma unroll
      for (int j = 0; j < JN; ++j) {
        const uint32_t le = (uint32_t)(w * JN + j) * 64u + (uint32_t)lane;
        k[j] = 0u;
        pos[j] = 0u;
        pk[j] = 0u;
        if (le < cn) {
          const uint2 kv = load(c0 + le);
          k[j] = kv.x;
          pos[j] = kv.y;
        }
      }
      bds_rank<JN>(L, cn, mn, shift, bits, k, pk);
      __syncthreads();
      const uint32_t tot = bds_wave_prefix(L);
      __syncthreads();
#pragma unroll
      for (int j = 0; j < JN; ++j) {
        const uint32_t le = (uint32_t)(w * JN + j) * 64u + (uint32_t)lane;
        if (le < cn) dst[bds_slot(L, pk[j])] = make_uint2(k[j], pos[j]);
      }
      __syncthreads();
      if (bds_owns_digit()) L.base[t] += tot;
#pragma unroll
      for (int q = 0; q < kBdsWaves; ++q)
        if (bds_owns_digit()) L.wcnt[q][t] = 0u;
      __syncthreads();
    }
    __syncthreads();
  }
  const uint2* fin = ((passes - 1) & 1) ? bufB : bufA;
  if (E) {
    bds_emit_big<JN>(L, skeys, sgid, fin, lo, n, EM);
    return;
  }
  for (uint32_t e = (uint32_t)t; e < n; e += kBdsThreads) {
    const uint32_t q = bds_load_scratch(fin + e).y;
    okeys[lo + e] = skeys[lo + q];
    ogid[lo + e] = sgid[lo + q];
  }
}

__global__ __launch_bounds__(kBdsThreads) void k_bin_depth_sort(
    const uint32_t* __restrict__ skeys, const uint32_t* __restrict__ sgid, const uint2* __restrict__ bounds,
    const uint32_t* __restrict__ gdep, uint32_t NL,
    uint32_t* __restrict__ okeys, uint32_t* __restrict__ ogid, uint2* scratch, BdsEmit emit) {
  __shared__ BdsLds L;
  const int t = threadIdx.x;
  const uint32_t bin = blockIdx.x;
  const uint2 bb = bounds[bin];
  const uint32_t lo = bb.x, n = bb.y - bb.x;
  // (a flag, not a pointer to the by-value argument: that would put it in scratch)
  const bool E = emit.lists != nullptr;
  if (n == 0) {  // block-uniform
    if (E) bds_emit_ranges(L, emit, bin, lo, 0u);
    return;
  }
#pragma unroll
  for (int q = 0; q < kBdsWaves; ++q)
    if (bds_owns_digit()) L.wcnt[q][t] = 0u;  // (published by bds_range's barrier)
  for (int i = t; i < kBdsWaves * kBdsDigits; i += kBdsThreads) (&L.match[0][0])[i] = 0ull;
  if (n <= 1u * kBdsThreads)
    bds_small<1>(L, skeys, sgid, nullptr, gdep, lo, n, okeys, ogid, E, emit);
  else if (n <= 2u * kBdsThreads)
    bds_small<2>(L, skeys, sgid, nullptr, gdep, lo, n, okeys, ogid, E, emit);
  // (every step of JN: a bin's time is its busiest wave's chain of JN entry
  // groups per pass, and a coarser JN leaves the last waves idle -- 4.7k
  // entries at JN = 7 keep 11 of 16 waves busy, at JN = 5 all 15 it needs)
  else if (n <= 3u * kBdsThreads)
    bds_small<3>(L, skeys, sgid, nullptr, gdep, lo, n, okeys, ogid, E, emit);
  else if (n <= 4u * kBdsThreads)
    bds_small<4>(L, skeys, sgid, nullptr, gdep, lo, n, okeys, ogid, E, emit);
  else if (n <= 5u * kBdsThreads)
    bds_small<5>(L, skeys, sgid, nullptr, gdep, lo, n, okeys, ogid, E, emit);
  else if (n <= 6u * kBdsThreads)
    bds_small<6>(L, skeys, sgid, nullptr, gdep, lo, n, okeys, ogid, E, emit);
  else if (n <= 7u * kBdsThreads)
    bds_small<7>(L, skeys, sgid, nullptr, gdep, lo, n, okeys, ogid, E, emit);
  else if (kBdsItems > 8 && n <= 8u * kBdsThreads)
    bds_small<(kBdsItems > 8 ? 8 : 7)>(L, skeys, sgid, nullptr, gdep, lo, n, okeys, ogid, E, emit);
  else if (kBdsItems > 9 && n <= 9u * kBdsThreads)
    bds_small<(kBdsItems > 9 ? 9 : 7)>(L, skeys, sgid, nullptr, gdep, lo, n, okeys, ogid, E, emit);
  else if (kBdsItems > 7 && n <= (uint32_t)kBdsCap)
    bds_small<kBdsItems>(L, skeys, sgid, nullptr, gdep, lo, n, okeys, ogid, E, emit);
  else
    bds_big(L, skeys, sgid, gdep, lo, n, NL, okeys, ogid, scratch, E, emit);
  if (E) bds_emit_ranges(L, emit, bin, lo, n);
}

// ---- tile ranges and the tiles' launch order ---------------------------------
// The render kernels take tile order[xcd_remap(blockIdx)]: blocks b with the
// same b % 8 run on one XCD (round-robin dispatch), and xcd_remap hands each
// XCD a contiguous chunk of tiles (a band of the image: splat records shared
// by neighbouring tiles stay in that XCD's L2).  Inside a chunk the tiles are
// ordered heaviest first (longest-processing-time list scheduling): with ~2
// waves per SIMD slot over the kernel, launch order decides the makespan
// (bench scene, backward: 68 % -> 91 % of the ideal in a list-scheduling
// simulation).  Order only changes scheduling, never a result.
constexpr int kOrderBuckets = 1024;

__device__ __forceinline__ void tile_chunk(uint32_t x, uint32_t nt, uint32_t& c0, uint32_t& c1) {
  const uint32_t q = nt / 8, r = nt % 8;
  c0 = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  c1 = c0 + (x < r ? q + 1 : q);
}

// Counting sort of the chunk's tiles by descending work bucket (one
// 1024-thread workgroup per chunk; positions inside a bucket come from LDS
// atomics, so ties may land in any order).
// work of a tile: work[tile], or with quads the max of work[4 tile .. 4 tile + 3]
__device__ __forceinline__ uint32_t tile_work(const uint32_t* __restrict__ work, bool quads, uint32_t tile) {
  if (!quads) return work[tile];
  const uint4 q = reinterpret_cast<const uint4*>(work)[tile];
  return max(max(q.x, q.y), max(q.z, q.w));
}

__device__ __forceinline__ void order_chunk(uint32_t c0, uint32_t c1, const uint32_t* __restrict__ work, bool quads,
                                            uint32_t* __restrict__ order, uint32_t* s_cnt) {
  const int t = threadIdx.x;
  s_cnt[t] = 0;
  __syncthreads();
  auto bucket = [&](uint32_t tile) {
    return (uint32_t)(kOrderBuckets - 1) - min((uint32_t)(kOrderBuckets - 1), tile_work(work, quads, tile));
  };
  for (uint32_t tile = c0 + t; tile < c1; tile += 1024) atomicAdd(&s_cnt[bucket(tile)], 1u);
  __syncthreads();
  // exclusive scan of the 1024 bucket counts (one per thread)
  __shared__ uint32_t s_w[16];
  const uint32_t v = s_cnt[t];
  uint32_t inc = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t o = __shfl_up(inc, off, 64);
    if ((t & 63) >= off) inc += o;
  }
  if ((t & 63) == 63) s_w[t >> 6] = inc;
  __syncthreads();
  uint32_t base = 0;
  for (int i = 0; i < (t >> 6); ++i) base += s_w[i];
  __syncthreads();
  s_cnt[t] = base + inc - v;
  __syncthreads();
  for (uint32_t tile = c0 + t; tile < c1; tile += 1024) order[c0 + atomicAdd(&s_cnt[bucket(tile)], 1u)] = tile;
}

// ranges[tile] = [first, end) of the tile's run in the sorted pair keys
// (binary search); len[tile] = its list length.
__global__ __launch_bounds__(256) void k_ranges(const uint32_t* __restrict__ keys, uint32_t N, int ntiles,
                                                uint2* __restrict__ ranges, uint32_t* __restrict__ len,
                                                uint32_t* __restrict__ meta) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t == 0) meta[0] = 0u;  // the lists are point_g
  if (t >= ntiles) return;
  auto lower = [&](uint32_t v) {
    uint32_t lo = 0, hi = N;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (keys[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
  };
  const uint2 r = make_uint2(lower((uint32_t)t), lower((uint32_t)t + 1));
  ranges[t] = r;
  len[t] = r.y - r.x;
}

// The backward's launch order by each tile's deepest contributor (its
// back-to-front walk length), written by the forward.
// One workgroup per XCD chunk, or (global) one for all tiles: then the
// render kernel takes order[blockIdx] and round-robin dispatch deals every
// 8th tile of the sorted list to each XCD.
__global__ __launch_bounds__(1024) void k_tile_order(const uint32_t* __restrict__ work, bool quads, bool global,
                                                     uint32_t ntiles, uint32_t* __restrict__ order) {
  __shared__ uint32_t s_cnt[kOrderBuckets];
  uint32_t c0 = 0, c1 = ntiles;
  if (!global) tile_chunk(blockIdx.x, ntiles, c0, c1);
  order_chunk(c0, c1, work, quads, order, s_cnt);
}

// Splat records arrive 64 at a time through LDS; wave 0 loads the next
// batch's records into registers while the current batch is blended (ids two
// ahead).
constexpr int kFwdBatch = 64;

// Entry-pair blend: the batch's entries that (one 8x8-quadrant wave's)
// survive the wave's culling are first compacted into the wave's own LDS area
// with two consecutive survivors interleaved per field (sQ: {x1, x2, y1, y2},
// {A.z1, A.z2, A.w1, A.w2}, {B.x1, B.x2, o1, o2}), so that one ds_read_b128
// hands two entries' operands to packed-FP32 math: the power, exp2 argument
// and opacity product of BOTH entries cost one v_pk_* instruction each (the
// forward's own operation sequence per lane, so alpha is bitwise that of
// the backward's recomputation).  Only the
// transmittance recurrence, the compares and the colour accumulation stay
// per entry.  n_touched increments are staged per compact slot.
// wave 0 streams the next batch's records into a second LDS buffer with
// global_load_lds instead of holding them in registers (every wave of the
// kernel would allocate those VGPRs)
struct FwdPairRec {   // two consecutive survivors (one LDS address per pair)
  float4 q[3];       // {x, x', y, y'}, {A.z, A.z', A.w, A.w'}, {B.x, B.x', o, o'}
  float4 c[2];       // colour (c0, c1, c2, depth) of each
  uint32_t n[2];     // contributor numbers
  uint32_t pad[2];
};
struct FwdPairLds {
  FwdPairRec p[kFwdBatch / 2];
  uint32_t touch[kFwdBatch];  // n_touched increment per compact slot
};

template <bool kTouch>
__device__ __forceinline__ void fwd_blend_one(float a, float pw, const float4& C, uint32_t cn, uint32_t* touch_slot,
                                              float& T, v2f& c01, v2f& c2d, uint32_t& last, uint64_t& dm,
                                              uint64_t valid) {
  const float test_T = fmaf(-T, a, T);  // T (1 - alpha)
  const uint64_t live = wave_ballot(pw <= 0.0f) & wave_ballot(a >= kMinAlpha) & ~dm & valid;
  const uint64_t low = wave_ballot(test_T < kMinT);
  const uint64_t blend = live & ~low;
  const bool bl = __builtin_amdgcn_inverse_ballot_w64(blend);
  const float wgt = bl ? a * T : 0.f;
  c01 += wgt * v2f{C.x, C.y};
  c2d += wgt * v2f{C.z, C.w};
  uint32_t tot = 0;
  if (kTouch) tot = (uint32_t)__popcll(blend & wave_ballot(test_T > 0.5f));
  T = bl ? test_T : T;
  last = bl ? cn : last;
  dm |= live & low;
  if (kTouch) *touch_slot = tot;
}

template <bool kTouch>
__device__ __forceinline__ void fwd_blend_pairs(int n, const FwdPairLds& L, uint32_t* touch, v2f pxy, float& T,
                                                v2f& c01, v2f& c2d, uint32_t& last, uint64_t& dm) {
  for (int i = 0; i < n && dm != ~0ull; i += 2) {
    const FwdPairRec& R = L.p[i >> 1];
    const float4 q0 = R.q[0], q1 = R.q[1], q2 = R.q[2];
    const float4 C1 = R.c[0], C2 = R.c[1];
    const uint2 cn = *reinterpret_cast<const uint2*>(&R.n[0]);
    const v2f DX = v2f{q0.x, q0.y} - v2f{pxy.x, pxy.x}, DY = v2f{q0.z, q0.w} - v2f{pxy.y, pxy.y};
    // splat_power per lane: fma(dx, fma(B.x, dy, A.z dx), (A.w dy) dy)
    const v2f tz = v2f{q1.x, q1.y} * DX, tw = v2f{q1.z, q1.w} * DY;
    const v2f PW = pfma(DX, pfma(v2f{q2.x, q2.y}, DY, tz), tw * DY);
    const v2f ag = v2f{q2.z, q2.w} * v2f{__builtin_amdgcn_exp2f(PW.x), __builtin_amdgcn_exp2f(PW.y)};
    const float a1 = fminf(kMaxAlpha, ag.x), a2 = fminf(kMaxAlpha, ag.y);
    fwd_blend_one<kTouch>(a1, PW.x, C1, cn.x, touch + i, T, c01, c2d, last, dm, ~0ull);
    // (an odd survivor count leaves the last pair's second half unused)
    fwd_blend_one<kTouch>(a2, PW.y, C2, cn.y, touch + i + 1, T, c01, c2d, last, dm, i + 1 < n ? ~0ull : 0ull);
  }
}

// cull the staged batch against the wave's pixel box, compact the survivors
// into L, blend them front to back in pairs, flush n_touched
// after(): called once the survivors are compacted (the LDS-DMA of the next
// batch is queued there, behind every LDS write of this batch)
template <class F>
__device__ __forceinline__ void fwd_blend_batch_pairs(int cnt, uint32_t cbase, const float4* sA, const float4* sB,
                                                      const float4* sC, const uint32_t* sG, FwdPairLds& L, int wx0,
                                                      int wx1, int wy0, int wy1, v2f pxy, int lane,
                                                      int32_t* __restrict__ n_touched, float& T, v2f& c01, v2f& c2d,
                                                      uint32_t& last, uint64_t& dm, uint32_t* fl_gid,
                                                      uint32_t* fl_tv, const float4* pre, uint32_t pre_gid, F after) {
  // (pre: this lane's records, read by the caller before it queued an LDS DMA)
  const float4 A = pre ? pre[0] : sA[lane], B = pre ? pre[1] : sB[lane];
  const bool mine = lane < cnt && ellipse_hits(A, B, wx0, wx1, wy0, wy1);
  const uint64_t todo = wave_ballot(mine);
  const int n = __popcll(todo);
  const uint32_t k = lanes_below(todo);
  // (uniform) a batch whose wave has no pixel left with T > 0.5 runs the entry
  // loop without the n_touched bookkeeping: T only falls, so none of its
  // entries can touch a pixel (one compare, two moves, one LDS store fewer)
  const bool touch = (wave_ballot(T > 0.5f) & ~dm) != 0;
  if (mine) {
    FwdPairRec& R = L.p[k >> 1];
    float* q = &R.q[0].x + (k & 1);
    q[0] = A.x; q[2] = A.y; q[4] = A.z; q[6] = A.w; q[8] = B.x; q[10] = B.y;
    R.c[k & 1] = pre ? pre[2] : sC[lane];
    R.n[k & 1] = cbase + (uint32_t)lane;
  }
  if (touch) L.touch[lane] = 0;
  if (lane == 63 && (n & 1)) {  // the unused half of an odd last pair: finite operands
    FwdPairRec& R = L.p[n >> 1];
    float* q = &R.q[0].x + 1;
    q[0] = 0.f; q[2] = 0.f; q[4] = 0.f; q[6] = 0.f; q[8] = 0.f; q[10] = 0.f;
    R.c[1] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // (a wave's own LDS accesses complete in order; the wave barrier -- no
  // instruction -- keeps the compiler from moving the cross-lane reads below
  // above these writes)
  __builtin_amdgcn_wave_barrier();
  after();
  if (touch) {
    fwd_blend_pairs<true>(n, L, L.touch, pxy, T, c01, c2d, last, dm);
    const uint32_t tv = mine ? L.touch[k] : 0u;
    if (fl_tv) {  // the caller issues the atomic later
      *fl_gid = pre_gid;
      *fl_tv = tv;
    } else if (tv != 0) {
      atomicAdd(&n_touched[sG[lane]], (int)tv);
    }
  } else {
    fwd_blend_pairs<false>(n, L, L.touch, pxy, T, c01, c2d, last, dm);
  }
  __builtin_amdgcn_wave_barrier();  // (the next batch's compaction writes stay behind these reads)
}

// One 16x16 tile per workgroup of 4 waves; wave w owns the 8x8 quadrant w,
// one pixel per lane.  Every per-pixel predicate (done, live, low, blend) is
// an explicit SGPR lane mask combined by scalar ops: the per-entry update is
// ~22 VALU instructions (power 6, exp2, alpha 2, four compares, T update,
// weight, two packed accumulates, three selects).  Also writes each
// quadrant's deepest contributor (tile_m4), the backward's per-tile work.
__global__ __launch_bounds__(256) void k_render_fwd1(
    const uint2* __restrict__ ranges, const uint32_t* __restrict__ order, const uint32_t* __restrict__ point_g,
    const float4* __restrict__ splat, int W, int H, int gx, int ntiles, const float* __restrict__ bg,
    float* __restrict__ out_color, float* __restrict__ out_depth, float* __restrict__ out_opac,
    float* __restrict__ final_T, uint32_t* __restrict__ n_contrib, int32_t* __restrict__ n_touched,
    uint32_t* __restrict__ tile_m4) {
  // two batch buffers as separate objects, so that the compiler can tell the
  // LDS-DMA into one from the reads of the other (no vmcnt wait before them)
  __shared__ float4 sA_0[kFwdBatch], sB_0[kFwdBatch], sC_0[kFwdBatch];
  __shared__ float4 sA_1[kFwdBatch], sB_1[kFwdBatch], sC_1[kFwdBatch];
  __shared__ uint32_t sG_0[kFwdBatch], sG_1[kFwdBatch];
  __shared__ uint32_t sDone[2][4];  // per batch parity: wave w has no pixel left
  __shared__ FwdPairLds sPair[4];  // per wave: the batch's surviving entries, compacted
  const uint32_t slot = xcd_remap(blockIdx.x, (uint32_t)ntiles);
  const uint32_t tile = order ? order[slot] : slot;  // null: xcd_remap's order as it is
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int tx0 = (int)(tile % gx) * kTile, ty0 = (int)(tile / gx) * kTile;
  int ox, oy;
  tile_pixel<1>(w, lane, 0, ox, oy);
  const int px = tx0 + ox, py = ty0 + oy;
  const v2f pxy{(float)px, (float)py};
  // per-pixel predicates live in SGPR lane masks (a ballot of a compound
  // predicate would be materialised through VGPRs): dm = finished pixels
  uint64_t dm = wave_ballot(!(px < W && py < H));
  const uint2 range = ranges[tile];
  int wx0, wx1, wy0, wy1;
  wave_box<1>(w, tx0, ty0, wx0, wx1, wy0, wy1);
  float T = 1.f;
  v2f c01{0.f, 0.f}, c2d{0.f, 0.f};  // (colour 0, colour 1), (colour 2, depth)
  uint32_t last = 0;

  // prefetch pipeline (wave 0): batch b+1's records stream straight into the
  // other LDS buffer (global_load_lds_dwordx4, no VGPRs held), ids of b+2 in
  // registers.  ONE barrier per batch, which waits for LDS only: wave 0's
  // vmcnt wait before it finds every load a batch old, and the n_touched
  // atomics of a batch are issued right after the next batch's barrier, so
  // no wave ever waits for an atomic.  Loads past the list re-read its last
  // entry (valid; culled by lane < cnt), so they need no branch.
  const uint32_t last_i = range.y > range.x ? range.y - 1 : range.x;
  auto fetch = [&](uint32_t g, float4* dA, float4* dB, float4* dC) {
    const float4* src = splat + 3 * (size_t)g;
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dA, 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(src + 1), (__attribute__((address_space(3))) void*)dB, 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(src + 2), (__attribute__((address_space(3))) void*)dC, 16, 0, 0);
  };
  uint32_t gcur = 0, gnext = 0;
  if (w == 0 && range.x < range.y) {
    gcur = point_g[min(range.x + t, last_i)];
    fetch(gcur, sA_0, sB_0, sC_0);
    if (range.x + kFwdBatch < range.y) gnext = point_g[min(range.x + kFwdBatch + t, last_i)];
  }
  uint32_t fl_gid = 0, fl_tv = 0;  // this lane's n_touched increment of the previous batch
  // one batch: read buffer (cA..cG), DMA target (nA..nC) as restrict
  // parameters, so that the compiler's LDS-DMA wait tracking sees that the
  // reads cannot alias the DMA in flight
  auto body = [&](uint32_t b0, uint32_t* __restrict__ done, float4* __restrict__ cA, float4* __restrict__ cB,
                  float4* __restrict__ cC, uint32_t* __restrict__ cG, float4* __restrict__ nA_,
                  float4* __restrict__ nB_, float4* __restrict__ nC_) -> bool {
    if (w == 0) {
      cG[t] = gcur;
      __builtin_amdgcn_s_waitcnt(0);  // this batch's records have landed
    }
    if (lane == 0) done[w] = dm == ~0ull ? 1u : 0u;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // (every wave is done with the other buffer)
    const uint4 dn = *reinterpret_cast<const uint4*>(done);
    // this lane's entry, read before the DMA is queued: the compiler would
    // otherwise wait for the DMA before reading the other buffer
    const float4 pre[3] = {cA[lane], cB[lane], cC[lane]};
    const uint32_t gme = cG[lane];
    // wave 0 queues the next batch's DMA after this batch's LDS writes (the
    // compiler orders LDS writes behind a DMA in flight), its id loads, then
    // the previous batch's n_touched atomics (a wait the compiler places for
    // the loads then never covers an atomic)
    bool queued = false;
    auto queue_next = [&]() {
      if (queued) return;
      queued = true;
      if (w == 0 && b0 + kFwdBatch < range.y) {
        gcur = gnext;
        fetch(gcur, nA_, nB_, nC_);
        if (b0 + 2 * kFwdBatch < range.y) gnext = point_g[min(b0 + 2 * kFwdBatch + t, last_i)];
      }
      if (fl_tv != 0) atomicAdd(&n_touched[fl_gid], (int)fl_tv);
      fl_tv = 0;
    };
    if (dn.x & dn.y & dn.z & dn.w) return false;
    if (dm != ~0ull) {
      const int cnt = (int)min((uint32_t)kFwdBatch, range.y - b0);
      fwd_blend_batch_pairs(cnt, b0 - range.x + 1, cA, cB, cC, cG, sPair[w], wx0, wx1, wy0, wy1, pxy, lane, n_touched,
                            T, c01, c2d, last, dm, &fl_gid, &fl_tv, pre, gme, queue_next);
    }
    queue_next();  // (a finished wave: keeps the barriers and the pipeline)
    return true;
  };
  auto step = [&](auto par, uint32_t b0) -> bool {
    if constexpr (decltype(par)::value == 0)
      return body(b0, sDone[0], sA_0, sB_0, sC_0, sG_0, sA_1, sB_1, sC_1);
    else
      return body(b0, sDone[1], sA_1, sB_1, sC_1, sG_1, sA_0, sB_0, sC_0);
  };
  for (uint32_t b0 = range.x; b0 < range.y; b0 += 2 * kFwdBatch) {
    if (!step(std::integral_constant<int, 0>{}, b0)) break;
    if (b0 + kFwdBatch >= range.y || !step(std::integral_constant<int, 1>{}, b0 + kFwdBatch)) break;
  }
  if (fl_tv != 0) atomicAdd(&n_touched[fl_gid], (int)fl_tv);
  {  // this quadrant's deepest contributor: tile_m4[4 tile + w] (no barrier)
    uint32_t mx = last;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off, 64));
    if (lane == 0) tile_m4[4 * tile + w] = mx;
  }
  if (!(px < W && py < H)) return;
  const size_t HW = (size_t)H * W;
  const size_t pid = (size_t)py * W + px;
  final_T[pid] = T;
  n_contrib[pid] = last;
  out_color[pid] = c01.x + T * bg[0];
  out_color[HW + pid] = c01.y + T * bg[1];
  out_color[2 * HW + pid] = c2d.x + T * bg[2];
  out_depth[pid] = c2d.y;
  out_opac[pid] = 1.f - T;
}

// k_render_fwd1 with the quadrant waves decoupled (the default;
// WGSR_FWD_DEC=0 keeps k_render_fwd1): every wave prefetches its own batch
// records into registers one batch ahead (lane j entry j) instead of wave 0
// streaming them into shared LDS behind a barrier per batch, and stops as
// soon as its own 64 pixels are done -- no wave waits for its tile's
// slowest quadrant.  Same blend per pixel in the same order, n_touched as
// integer atomics: bit-identical outputs.
#ifndef WGSR_FWD_DEC
#define WGSR_FWD_DEC 1
#endif
// diagnostic build: per quadrant wave of k_render_fwd_dec -- [0] waves, [1]
// batches, [2] entries in them, [3] survivors of the culling, [4] pair
// iterations (survivor pairs), [5] batches with the n_touched bookkeeping,
// [6] waves that stopped with every pixel done (wgsr_debug_fwd_stats)
#ifndef WGSR_FWD_STATS
#define WGSR_FWD_STATS 0
#endif
#if WGSR_FWD_STATS
__device__ unsigned long long g_fwd_stats[8];
#endif
__global__ __launch_bounds__(256) void k_render_fwd_dec(
    const uint2* __restrict__ ranges, const uint32_t* __restrict__ order, const uint32_t* __restrict__ point_g,
    const float4* __restrict__ splat, int W, int H, int gx, int ntiles, const float* __restrict__ bg,
    float* __restrict__ out_color, float* __restrict__ out_depth, float* __restrict__ out_opac,
    float* __restrict__ final_T, uint32_t* __restrict__ n_contrib, int32_t* __restrict__ n_touched,
    uint32_t* __restrict__ tile_m4) {
  __shared__ FwdPairLds sPair[4];  // per wave: the batch's surviving entries, compacted
  const uint32_t slot = xcd_remap(blockIdx.x, (uint32_t)ntiles);
  const uint32_t tile = order ? order[slot] : slot;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int tx0 = (int)(tile % gx) * kTile, ty0 = (int)(tile / gx) * kTile;
  int ox, oy;
  tile_pixel<1>(w, lane, 0, ox, oy);
  const int px = tx0 + ox, py = ty0 + oy;
  const v2f pxy{(float)px, (float)py};
  uint64_t dm = wave_ballot(!(px < W && py < H));
  const uint2 range = ranges[tile];
  int wx0, wx1, wy0, wy1;
  wave_box<1>(w, tx0, ty0, wx0, wx1, wy0, wy1);
  float T = 1.f;
  v2f c01{0.f, 0.f}, c2d{0.f, 0.f};
  uint32_t last = 0;
  (void)t;
  const uint32_t last_i = range.y > range.x ? range.y - 1 : range.x;
  uint32_t gcur = 0, gnext = 0;
  float4 nA = make_float4(0, 0, 0, 0), nB = nA, nC = nA;
  if (range.x < range.y) {
    gcur = point_g[min(range.x + lane, last_i)];
    nA = splat[3 * (size_t)gcur];
    nB = splat[3 * (size_t)gcur + 1];
    nC = splat[3 * (size_t)gcur + 2];
    if (range.x + kFwdBatch < range.y) gnext = point_g[min(range.x + kFwdBatch + lane, last_i)];
  }
  uint32_t fl_gid = 0, fl_tv = 0;  // this lane's n_touched increment of the previous batch
#if WGSR_FWD_STATS
  uint32_t st_b = 0, st_e = 0, st_s = 0, st_p = 0, st_t = 0;
#endif
  for (uint32_t b0 = range.x; b0 < range.y && dm != ~0ull; b0 += kFwdBatch) {  // (wave-uniform)
    const float4 pre[3] = {nA, nB, nC};
    const uint32_t gme = gcur;
    if (b0 + kFwdBatch < range.y) {  // the next batch's records, the one after's ids
      gcur = gnext;
      nA = splat[3 * (size_t)gcur];
      nB = splat[3 * (size_t)gcur + 1];
      nC = splat[3 * (size_t)gcur + 2];
      if (b0 + 2 * kFwdBatch < range.y) gnext = point_g[min(b0 + 2 * kFwdBatch + lane, last_i)];
    }
    const int cnt = (int)min((uint32_t)kFwdBatch, range.y - b0);
    // cull against the wave's pixel box, compact the survivors in pairs, blend
    // (fwd_blend_batch_pairs on register-held records)
    FwdPairLds& L = sPair[w];
    const bool mine = lane < cnt && ellipse_hits(pre[0], pre[1], wx0, wx1, wy0, wy1);
    const uint64_t todo = wave_ballot(mine);
    const int n = __popcll(todo);
    const uint32_t k = lanes_below(todo);
    const bool touch = (wave_ballot(T > 0.5f) & ~dm) != 0;  // (uniform)
    if (mine) {
      FwdPairRec& R = L.p[k >> 1];
      float* q = &R.q[0].x + (k & 1);
      q[0] = pre[0].x; q[2] = pre[0].y; q[4] = pre[0].z; q[6] = pre[0].w; q[8] = pre[1].x; q[10] = pre[1].y;
      R.c[k & 1] = pre[2];
      R.n[k & 1] = b0 - range.x + 1 + (uint32_t)lane;
    }
    if (touch) L.touch[lane] = 0;
    if (lane == 63 && (n & 1)) {  // the unused half of an odd last pair: finite operands
      FwdPairRec& R = L.p[n >> 1];
      float* q = &R.q[0].x + 1;
      q[0] = 0.f; q[2] = 0.f; q[4] = 0.f; q[6] = 0.f; q[8] = 0.f; q[10] = 0.f;
      R.c[1] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
#if WGSR_FWD_STATS
    ++st_b;
    st_e += (uint32_t)cnt;
    st_s += (uint32_t)n;
    st_p += (uint32_t)((n + 1) / 2);
    st_t += touch ? 1u : 0u;
#endif
    // cross-lane LDS traffic of one wave: ordered by the hardware, and kept in
    // program order by the (instruction-free) wave barriers here and below
    __builtin_amdgcn_wave_barrier();
    if (fl_tv != 0) atomicAdd(&n_touched[fl_gid], (int)fl_tv);  // the previous batch's
    fl_tv = 0;
    if (touch) {
      fwd_blend_pairs<true>(n, L, L.touch, pxy, T, c01, c2d, last, dm);
      fl_gid = gme;
      fl_tv = mine ? L.touch[k] : 0u;
    } else {
      fwd_blend_pairs<false>(n, L, L.touch, pxy, T, c01, c2d, last, dm);
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (fl_tv != 0) atomicAdd(&n_touched[fl_gid], (int)fl_tv);
#if WGSR_FWD_STATS
  if (lane == 0) {
    atomicAdd(&g_fwd_stats[0], 1ull);
    atomicAdd(&g_fwd_stats[1], (unsigned long long)st_b);
    atomicAdd(&g_fwd_stats[2], (unsigned long long)st_e);
    atomicAdd(&g_fwd_stats[3], (unsigned long long)st_s);
    atomicAdd(&g_fwd_stats[4], (unsigned long long)st_p);
    atomicAdd(&g_fwd_stats[5], (unsigned long long)st_t);
    atomicAdd(&g_fwd_stats[6], dm == ~0ull ? 1ull : 0ull);
  }
#endif
  {  // this quadrant's deepest contributor: tile_m4[4 tile + w]
    uint32_t mx = last;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off, 64));
    if (lane == 0) tile_m4[4 * tile + w] = mx;
  }
  if (!(px < W && py < H)) return;
  const size_t HW = (size_t)H * W;
  const size_t pid = (size_t)py * W + px;
  final_T[pid] = T;
  n_contrib[pid] = last;
  out_color[pid] = c01.x + T * bg[0];
  out_color[HW + pid] = c01.y + T * bg[1];
  out_color[2 * HW + pid] = c2d.x + T * bg[2];
  out_depth[pid] = c2d.y;
  out_opac[pid] = 1.f - T;
}



__global__ __launch_bounds__(256) void k_mark_visible(int P, const float* __restrict__ means,
                                                      const float* __restrict__ viewm, uint8_t* __restrict__ present) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  const f3 p = mk3(means[3 * i], means[3 * i + 1], means[3 * i + 2]);
  const f3 pv = xform43(viewm, p);
  present[i] = pv.z > kNearZ ? 1 : 0;
}

}  // namespace

// Capacity-mode forward: the counter block's partial pair counts (upstream's
// rect pairs, exact pairs, bin pairs: kRectPairLanes u64 each) -> counts[0..2]
// (saturating u32), the bin-pair count clamped to the buffers (counts[4], what
// the sort reads as its key count) and the overflow flag (counts[3] and the
// image buffer's meta[1], which makes the render backward a no-op).

__global__ __launch_bounds__(64) void k_cap_counts(const unsigned long long* __restrict__ partial,
                                                   uint64_t cap_rect, uint64_t cap_bin, uint32_t* __restrict__ counts,
                                                   uint32_t* __restrict__ meta) {
  const int t = threadIdx.x;
  unsigned long long r = partial[t], e = partial[kRectPairLanes + t], b = partial[2 * kRectPairLanes + t];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    r += __shfl_xor(r, off, 64);
    e += __shfl_xor(e, off, 64);
    b += __shfl_xor(b, off, 64);
  }
  if (t == 0) {
    const uint32_t ovf = (r > cap_rect || b > cap_bin) ? 1u : 0u;
    counts[0] = (uint32_t)min(r, 0xFFFFFFFFull);
    counts[1] = (uint32_t)min(e, 0xFFFFFFFFull);
    counts[2] = (uint32_t)min(b, 0xFFFFFFFFull);
    counts[3] = ovf;
    counts[4] = (uint32_t)min(b, (unsigned long long)cap_bin);
    meta[1] = ovf;
  }
}
static_assert(kRectPairLanes == 64, "k_cap_counts: one lane per partial");

hipError_t launch_cap_counts(const unsigned long long* partial, uint64_t cap_rect, uint64_t cap_bin, uint32_t* counts,
                             uint32_t* meta, hipStream_t s) {
  hipLaunchKernelGGL(k_cap_counts, dim3(1), dim3(64), 0, s, partial, cap_rect, cap_bin, counts, meta);
  return hipGetLastError();
}

hipError_t launch_preprocess(const wgsr_raster_args& a, void* geom, int32_t* radii, int32_t* n_touched,
                             uint32_t* err_flag, unsigned long long* rect_pairs, int bshift, const ZeroJob& zero,
                             hipStream_t s, uint32_t* meta) {
  unsigned long long* list_pairs = rect_pairs + kRectPairLanes;
  unsigned long long* bin_pairs = rect_pairs + 2 * kRectPairLanes;
  uint32_t* drange = reinterpret_cast<uint32_t*>(rect_pairs + 3 * kRectPairLanes);  // kDepthRangeOffset
  if (a.P == 0) return hipSuccess;
  const GeomLayout L(a.P);
  const int gx = (a.W + kTile - 1) / kTile, gy = (a.H + kTile - 1) / kTile;
  const bool sh_on = a.shs && !a.colors;
  const bool ch4 = sh_on && (a.M * 3) % 4 == 0 && (reinterpret_cast<uintptr_t>(a.shs) & 15) == 0;
  const int nf = 3 * (a.D + 1) * (a.D + 1);
  const int kch = ch4 ? 4 : 1;
  const size_t lds2 = sh_on ? sizeof(float) * 64 * (size_t)(((nf + kch - 1) / kch) * kch) : 0;
  using PreKernel = decltype(&k_preprocess2<1, -1>);
  static constexpr PreKernel kPre[2][4] = {{k_preprocess2<1, 0>, k_preprocess2<1, 1>, k_preprocess2<1, 2>,
                                            k_preprocess2<1, 3>},
                                           {k_preprocess2<4, 0>, k_preprocess2<4, 1>, k_preprocess2<4, 2>,
                                            k_preprocess2<4, 3>}};
  const PreKernel kern = sh_on ? kPre[ch4 ? 1 : 0][std::min(std::max(a.D, 0), 3)] : k_preprocess2<1, -1>;
  hipLaunchKernelGGL(kern, dim3((a.P + kPreWave - 1) / kPreWave), dim3(kPreWave),
                     lds2, s, a.P, a.D, a.M, a.means3D, a.scales, a.rotations, a.opacities, a.shs, a.colors,
                     a.cov3D_precomp, a.scale_modifier, a.viewmatrix, a.projmatrix, a.campos, a.W, a.H, a.tan_fovx,
                     a.tan_fovy, gx, gy, a.prefiltered, at<float4>(geom, L.splat), at<ListRec>(geom, L.lrec),
                     at<uint32_t>(geom, L.clamped), at<uint32_t>(geom, L.dkey), radii, n_touched, err_flag, rect_pairs,
                     list_pairs, bin_pairs, bshift, at<uint32_t>(geom, L.tb), at<uint8_t>(geom, L.gflag), drange, zero,
                     meta);
  return hipGetLastError();
}

hipError_t launch_duplicate_bins(const wgsr_raster_args& a, void* geom, const uint32_t* depth_order, int bshift,
                                 uint8_t* pflag, uint32_t* keys, uint32_t* vals, bool bsup, const ZeroJob& zero,
                                 uint32_t* meta, hipStream_t s, uint32_t cap_slots, uint32_t cap_pairs) {
  if (a.P == 0) return hipSuccess;
  const GeomLayout L(a.P);
  const Bins B((a.W + kTile - 1) / kTile, (a.H + kTile - 1) / kTile, bshift);
  if (bshift < 1 || bshift > kMaxBinShift) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bshift == 1 ? k_duplicate_bins<1> : k_duplicate_bins<2>,
                     dim3((a.P + kDupScanThreads - 1) / kDupScanThreads), dim3(kDupScanThreads), 0,
                     s, (uint32_t)a.P, B.bx, at<ListRec>(geom, L.lrec), depth_order, at<uint2>(geom, L.bsum),
                     bsup ? at<uint2>(geom, L.bsup) : nullptr,
                     at<float4>(geom, L.splat),
                     at<uint32_t>(geom, L.slot_start), pflag, keys, vals, zero, meta, cap_slots, cap_pairs);
  return hipGetLastError();
}

hipError_t launch_expand_bins(const wgsr_raster_args& a, const uint32_t* sorted_keys, const uint32_t* sorted_g,
                              uint32_t NB, int bshift, uint2* bounds, bool bounds_done, uint32_t* lists, uint2* ranges,
                              uint32_t* tile_len, uint32_t* meta, hipStream_t s) {
  const int gx = (a.W + kTile - 1) / kTile, gy = (a.H + kTile - 1) / kTile;
  const Bins B(gx, gy, bshift);
  if (!bounds_done) {  // (a one-pass sort already wrote them)
    hipError_t e = hipMemsetAsync(bounds, 0, sizeof(uint2) * (size_t)B.n, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_bin_bounds, dim3((NB + 255) / 256), dim3(256), 0, s, sorted_keys, NB, bounds);
  }
  hipLaunchKernelGGL(k_expand_bins, dim3((uint32_t)B.n << bshift), dim3(kExpThreads), 0, s, sorted_keys, sorted_g, bounds, gx,
                     gy, bshift, B.bx, lists, ranges, tile_len, meta);
  return hipGetLastError();
}

namespace {
// Stable argsort of n <= kBdsCap 32-bit keys in one workgroup: the per-bin
// depth sort's LDS passes on a single "bin" whose payload is the position
// (ties keep index order).  perm[i] = the index of the i-th smallest key.
__global__ __launch_bounds__(kBdsThreads) void k_argsort_small(const uint32_t* __restrict__ keys, uint32_t n,
                                                              uint32_t* __restrict__ perm) {
  __shared__ BdsLds L;
  const int t = threadIdx.x;
  const BdsEmit none{};
#pragma unroll
  for (int q = 0; q < kBdsWaves; ++q)
    if (bds_owns_digit()) L.wcnt[q][t] = 0u;
  for (int i = t; i < kBdsWaves * kBdsDigits; i += kBdsThreads) (&L.match[0][0])[i] = 0ull;
  if (kBdsThreads >= 1024 && n <= 1u * kBdsThreads)
    bds_small<1>(L, nullptr, nullptr, keys, nullptr, 0u, n, nullptr, perm, false, none);
  else if (n <= 2u * kBdsThreads)
    bds_small<2>(L, nullptr, nullptr, keys, nullptr, 0u, n, nullptr, perm, false, none);
  else if (n <= 4u * kBdsThreads)
    bds_small<4>(L, nullptr, nullptr, keys, nullptr, 0u, n, nullptr, perm, false, none);
  else
    bds_small<kBdsItems>(L, nullptr, nullptr, keys, nullptr, 0u, n, nullptr, perm, false, none);
}
}  // namespace

uint32_t argsort_small_max() { return (uint32_t)kBdsCap; }
hipError_t launch_argsort_small(const uint32_t* keys, uint32_t n, uint32_t* perm, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (n > (uint32_t)kBdsCap) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_argsort_small, dim3(1), dim3(kBdsThreads), 0, s, keys, n, perm);
  return hipGetLastError();
}

hipError_t launch_bin_depth_sort(const wgsr_raster_args& a, const uint32_t* sorted_keys, const uint32_t* sorted_g,
                                 uint32_t NB, int bshift, uint2* bounds, bool bounds_done, const uint32_t* gdepth,
                                 uint32_t* okeys, uint32_t* ogid, void* scratch, hipStream_t s, uint32_t* lists,
                                 uint2* ranges, uint32_t* tile_len, uint32_t* meta) {
  const int gx = (a.W + kTile - 1) / kTile, gy = (a.H + kTile - 1) / kTile;
  const Bins B(gx, gy, bshift);
  if (!bounds_done) {  // (a one-pass sort already wrote them)
    hipError_t e = hipMemsetAsync(bounds, 0, sizeof(uint2) * (size_t)B.n, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_bin_bounds, dim3((NB + 255) / 256), dim3(256), 0, s, sorted_keys, NB, bounds);
  }
  // lists != null: the per-tile lists and ranges are emitted here (no
  // k_expand_bins); else the sorted bins go to okeys / ogid
  const BdsEmit emit{lists, ranges, tile_len, meta, gx, gy, bshift, B.bx};
  hipLaunchKernelGGL(k_bin_depth_sort, dim3((uint32_t)B.n), dim3(kBdsThreads), 0, s, sorted_keys, sorted_g, bounds,
                     gdepth, NB, okeys, ogid, static_cast<uint2*>(scratch), emit);
  return hipGetLastError();
}

hipError_t launch_duplicate(const wgsr_raster_args& a, const void* geom, const uint32_t* sorted_g, uint32_t P,
                            uint32_t* keys, uint32_t* slot_g, uint8_t* pflag, hipStream_t s) {
  if (P == 0) return hipSuccess;
  const GeomLayout L(P);
  const int gx = (a.W + kTile - 1) / kTile;
  hipLaunchKernelGGL(k_duplicate, dim3((P + 255) / 256), dim3(256), 0, s, P, gx, at<uint32_t>(geom, L.offs),
                     sorted_g, at<ListRec>(geom, L.lrec), at<float4>(geom, L.splat),
                     keys, slot_g, pflag);
  return hipGetLastError();
}

hipError_t launch_ranges(const uint32_t* sorted_keys, uint32_t N, int ntiles, uint2* ranges, uint32_t* len,
                         uint32_t* meta, hipStream_t s) {
  hipLaunchKernelGGL(k_ranges, dim3((ntiles + 255) / 256), dim3(256), 0, s, sorted_keys, N, ntiles, ranges, len, meta);
  return hipGetLastError();
}

hipError_t launch_tile_order(const uint32_t* work_quads, int ntiles, uint32_t* order, hipStream_t s) {
  // per-XCD chunks (one global LPT list measured 2 % slower)
  hipLaunchKernelGGL(k_tile_order, dim3(8), dim3(1024), 0, s, work_quads, true, false, (uint32_t)ntiles, order);
  return hipGetLastError();
}

hipError_t launch_render_fwd(const wgsr_raster_args& a, const uint2* ranges, const uint32_t* point_g, const void* geom, float* out_color, float* out_depth,
                             float* out_opacity, float* final_T, uint32_t* n_contrib, int32_t* n_touched,
                             uint32_t* tile_m, hipStream_t s) {
  const GeomLayout L(a.P);
  const int gx = (a.W + kTile - 1) / kTile, gy = (a.H + kTile - 1) / kTile;
  const int nt = gx * gy;
  const char* dec = getenv("WGSR_FWD_DEC");  // (read per launch: tests compare the two)
  auto kern = (dec ? atoi(dec) != 0 : WGSR_FWD_DEC != 0) ? k_render_fwd_dec : k_render_fwd1;
  hipLaunchKernelGGL(kern, dim3(nt), dim3(256), 0, s, ranges, nullptr, point_g,
                     at<float4>(geom, L.splat), a.W, a.H, gx, nt, a.bg, out_color, out_depth, out_opacity, final_T,
                     n_contrib, n_touched, tile_m);
  return hipGetLastError();
}

// Consistency check of a forward's tile lists (wgsr_check_tile_lists): one
// wave per tile.  bad[0] += tiles whose [start, end) leaves the list region
// or disagrees with tile_len; bad[1] += listed ids >= P; bad[2] += pixels
// whose last contributor lies beyond their tile's list.  The entries of a
// tile with a bad range are not read.
__global__ __launch_bounds__(64) void k_check_tile_lists(const uint2* __restrict__ ranges,
                                                         const uint32_t* __restrict__ tile_len,
                                                         const uint32_t* __restrict__ meta,
                                                         const uint32_t* __restrict__ lists_exact,
                                                         const uint32_t* __restrict__ lists_bins, uint64_t n_exact,
                                                         uint64_t n_bins, uint32_t P, int W, int H, int gx,
                                                         const uint32_t* __restrict__ n_contrib,
                                                         uint32_t* __restrict__ bad) {
  const uint32_t tile = blockIdx.x;
  const int lane = threadIdx.x;
  const bool bins = meta[0] != 0u;
  const uint32_t* __restrict__ lists = bins ? lists_bins : lists_exact;
  const uint64_t region = bins ? n_bins : n_exact;
  const uint2 r = ranges[tile];
  const bool ok = r.x <= r.y && (uint64_t)r.y <= region && tile_len[tile] == r.y - r.x;
  if (!ok) {
    if (lane == 0) atomicAdd(&bad[0], 1u);
    return;
  }
  uint32_t nb = 0;
  for (uint32_t e = r.x + (uint32_t)lane; e < r.y; e += 64) nb += lists[e] >= P ? 1u : 0u;
  const int tx0 = (int)(tile % (uint32_t)gx) * kTile, ty0 = (int)(tile / (uint32_t)gx) * kTile;
  uint32_t np = 0;
  for (int q = lane; q < kTile * kTile; q += 64) {
    const int px = tx0 + (q % kTile), py = ty0 + (q / kTile);
    if (px < W && py < H) np += n_contrib[(size_t)py * W + px] > r.y - r.x ? 1u : 0u;
  }
  if (nb) atomicAdd(&bad[1], nb);
  if (np) atomicAdd(&bad[2], np);
}

// p[0..n) = 0 by a kernel: the capacity-mode forward zeroes its buffers with
// kernel nodes, not memset nodes.  A hipMemsetAsync captured into a HIP graph
// (a memset node) was measured NOT to have zeroed the counter block before
// k_preprocess accumulated into it on some replays -- the two-rank
// data-parallel loop on one GPU: a replayed forward of an unchanged map and
// camera reported N_rect >= 2^32 while the eager forward of the same state
// gave 8561, deterministically, and the kernel zeroing below fixed it.  Garbage
// counts make the bin sort take `cap` keys of which only the written ones are
// valid, so the per-bin sort then gathers depth keys through unwritten
// Gaussian ids: the out-of-bounds reads behind round 5's SIGABRT in the
// overflow-recovery test are consistent with it.
__global__ __launch_bounds__(256) void k_zero_u32(uint32_t* __restrict__ p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = 0u;
}

hipError_t launch_zero_u32(uint32_t* p, size_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const size_t blocks = std::min<size_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(k_zero_u32, dim3((uint32_t)blocks), dim3(256), 0, s, p, n);
  return hipGetLastError();
}

hipError_t launch_check_tile_lists(const wgsr_raster_args& a, int bshift, uint64_t num_rendered, const void* binning,
                                   const void* image, uint32_t* bad, hipStream_t s) {
  const int gx = (a.W + kTile - 1) / kTile, gy = (a.H + kTile - 1) / kTile;
  const ImageLayout IL(a.W, a.H);
  const BinLayout BL((size_t)num_rendered);
  hipLaunchKernelGGL(k_check_tile_lists, dim3((uint32_t)(gx * gy)), dim3(64), 0, s, at<uint2>(image, IL.ranges),
                     at<uint32_t>(image, IL.tile_len), at<uint32_t>(image, IL.meta), at<uint32_t>(binning, BL.point_g),
                     at<uint32_t>(binning, BL.total), num_rendered, num_rendered << (2 * bshift), (uint32_t)a.P, a.W,
                     a.H, gx, at<uint32_t>(image, IL.n_contrib), bad);
  return hipGetLastError();
}

hipError_t launch_mark_visible(int P, const float* means3D, const float* view, const float* proj, uint8_t* present,
                               hipStream_t s) {
  (void)proj;
  if (P == 0) return hipSuccess;
  hipLaunchKernelGGL(k_mark_visible, dim3((P + 255) / 256), dim3(256), 0, s, P, means3D, view, present);
  return hipGetLastError();
}

}  // namespace wgsr

#if WGSR_FWD_STATS
// diagnostic build only: read and clear the forward's per-wave census
extern "C" int wgsr_debug_fwd_stats(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(wgsr::g_fwd_stats), sizeof(unsigned long long) * 8) != hipSuccess)
    return 1;
  unsigned long long z[8] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(wgsr::g_fwd_stats), z, sizeof(z)) != hipSuccess;
}
#endif
