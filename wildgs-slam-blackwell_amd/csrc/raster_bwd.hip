// Backward rasteriser stages for gfx950.
//
//   render_bwd  one wave64 per tile (4 pixels per lane) walks the tile's list
//               back to front (upstream BACKWARD::renderCUDA math).  Instead of one
//               float atomic per (pixel, Gaussian, quantity) -- scattered
//               single-lane atomics run ~17x under the chip's atomic rate on
//               MI355X -- each lane sums its four pixels in registers, one
//               packed wave reduction covers the whole tile, and the tile
//               writes ONE 48-byte partial record per (Gaussian, tile) pair
//               that actually received gradient (plus a 1-byte slot flag),
//               into that pair's duplicate slot.  No atomics, deterministic.
//   gauss_bwd   one lane per Gaussian: sums the flagged records of its
//               contiguous slot range (fixed order -> bitwise reproducible), then
//               runs cov2D -> cov3D -> (scale, rotation), SH, projection,
//               depth and pose (w-pose dL/dtau) backward in registers and
//               writes every output of _C.rasterize_gaussians_backward once.
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "wgsr_common.h"
#include "wgsr_internal.h"

namespace wgsr {

namespace {

constexpr int kBatch = 64;  // entries staged per LDS batch in the backward
// diagnostic build: histogram of (quadrants reached, quadrants evaluated in
// phase 2) per entry over the quad backward (wgsr_debug_bwd_stats)
#ifndef WGSR_BWD_STATS
#define WGSR_BWD_STATS 0
#endif
#if WGSR_BWD_STATS
__device__ unsigned long long g_bwd_stats[64];
#endif
// diagnostic build: per-workgroup phase clocks of k_gauss_bwd_compact summed
// over workgroups (s_memtime; wgsr_debug_gbc_times)
#ifndef WGSR_GBC_TIMES
#define WGSR_GBC_TIMES 0
#endif
#if WGSR_GBC_TIMES
__device__ unsigned long long g_gbc_times[16];
#define GBC_MARK(k)                                                                    \
  do {                                                                                 \
    if (t == 0) {                                                                      \
      const unsigned long long now = __builtin_amdgcn_s_memtime();                    \
      atomicAdd(&g_gbc_times[k], now - gbc_t0);                                         \
    }                                                                                  \
  } while (0)
#else
#define GBC_MARK(k) do {} while (0)
#endif
// diagnostic build: each k_render_bwd_quad workgroup's start / end
// (s_memrealtime, 100 MHz) and hardware id (wgsr_debug_bwd_wgtime)
#ifndef WGSR_BWD_WGTIME
#define WGSR_BWD_WGTIME 0
#endif
#if WGSR_BWD_WGTIME
constexpr int kWgtMax = 32768;
__device__ unsigned long long g_bwd_wgt[3 * kWgtMax];
#endif
// below this many tiles the backward runs k_render_bwd_seg (four waves per
// tile) instead of k_render_bwd_quad (one); WGSR_BWD_SPLIT_BELOW overrides
constexpr int kBwdSplitBelowTiles = 3072;

constexpr float SH_C0 = 0.28209479177387814f;
constexpr float SH_C1 = 0.4886025119029199f;
__constant__ float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
__constant__ float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f,  -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

// The render backward sums, over a tile's pixels, u = G dL/dalpha (dx, dy),
// its moments u_x dx, u_x dy, u_y dy and G dL/dalpha; the entry's own
// constants come out of those sums here, once per (Gaussian, tile) record:
//   g0 = o (2 A.z Su_x + B.x Su_y), g1 = o (2 A.w Su_y + B.x Su_x)  -- log2(e) x dL/d(mean2D pixel)
//   g2, g3, g4 = o x moments                                         -- dL/dconic / (-1/2)
//   g5 = S G dL/dalpha                                               -- dL/dopacity
// (A.z, A.w, B.x: the log2(e)-scaled conic of the splat record, o = B.y.)
// (no contraction: every kernel that writes records rounds them alike)
__device__ __forceinline__ void record_sums(const float4& A, const float4& B, float (&g)[10]) {
#pragma clang fp contract(off)
  const float o = B.y, ux = g[0], uy = g[1];
  g[0] = o * (2.f * A.z * ux + B.x * uy);
  g[1] = o * (2.f * A.w * uy + B.x * ux);
  g[2] *= o;
  g[3] *= o;
  g[4] *= o;
}

// ONE wave per 16x16 tile; lane l owns pixel (l & 7,
// l >> 3) of each of the four 8x8 quadrants.  Lane j tests entry j's ellipse
// against each quadrant (four ballots), so per entry the wave evaluates only
// the quadrants the splat can reach (wave-uniform branches) -- the culling of
// the 4-wave layout -- but sums all of them with ONE wave reduction and writes
// the record without a cross-wave combine.
// Measured (round 5, 1M/1080p, rocprof): reducing two hit entries' sums
// together with wave_sum20 (42 instead of 2 x 23 VALU) costs 10 more VGPRs
// held across the walk -- 326 us with 5 spilled VGPRs at 4 waves/SIMD, 350 us
// at 3 waves/SIMD, vs 311 us for one wave_sum10 per entry (3 waves/SIMD with
// this code: 313 us).
// kBg = false: a black background (the mapper's default), whose term
// -T_final (bg . dL/dpixel) / (1 - alpha) of dL/dalpha is zero -- one packed
// multiply and a register move fewer per evaluation
template <bool kBg>
__device__ __forceinline__ void render_bwd_quad_tile(
    const uint32_t tile, const uint2* __restrict__ ranges, const uint32_t* __restrict__ point_g,
    const float4* __restrict__ splat, const ListRec* __restrict__ lrec, const uint32_t* __restrict__ slot_start, int W,
    int H, int gx, float bg0, float bg1, float bg2, const float* __restrict__ final_Ts,
    const uint32_t* __restrict__ n_contrib, const float* __restrict__ dL_dpix, const float* __restrict__ dL_ddep,
    float4* __restrict__ partial, uint8_t* __restrict__ pflag, uint8_t* __restrict__ gflag, float4* sA, float4* sB,
    float4* sC, uint32_t* sG, float (*sP)[11], uint32_t* sHit) {
  constexpr int Q = 4;
  const int lane = threadIdx.x;
  const int tx0 = (int)(tile % gx) * kTile, ty0 = (int)(tile / gx) * kTile;
  const size_t HW = (size_t)H * W;
  const uint2 range = ranges[tile];
#if WGSR_BWD_STATS
  uint32_t* const sStat = sHit;  // [0, 16) reach masks, [16, 32) phase-2 masks, [32, 40) pixels per hit
  sStat[lane] = 0;                // entry (log2 bins), [40, 48) lanes per phase-2 evaluation, [48] phase-2
                                  // lanes, [49] phase-1 evaluations without a phase 2, [50] phase-1
                                  // evaluations in batches live at every pixel of the quadrant
  __syncthreads();
#endif

  // per-quadrant pixel state; pairs are packed for v_pk_* math.  Pixel
  // positions are not kept per quadrant: quadrant p's pixel is this lane's
  // quadrant-0 pixel p0 + 8 (p & 1, p >> 1), so (dx, dy) for quadrant p is
  // (mean - p0) minus an immediate (fewer live VGPRs: no spills)
  const v2f p0{(float)(tx0 + (lane & 7)), (float)(ty0 + (lane >> 3))};
  v2f dp01[Q], dp2d[Q];
  // upstream's accum_rec (colour, depth) dotted with this pixel's dL/d(colour,
  // depth), held negated as a pair (-accd = na.x + na.y, na.y stays 0): the
  // pair rides in the packed dot product, c.dp - accd = sum of
  // fma(c2d, dp2d, fma(c01, dp01, na)) -- one instruction fewer per evaluation
  v2f na[Q];
  float T[Q], tb[Q];
  uint32_t last[Q], mq[Q];
#if WGSR_BWD_STATS
  uint32_t minq[Q];  // every pixel of quadrant p takes entries below minq[p]
#endif
  uint32_t m = 0;
  // every quadrant's pixel loads first (one round trip; pixels outside the
  // image read pixel 0 and are zeroed after), then the sums
  bool inside[Q];
#pragma unroll
  for (int p = 0; p < Q; ++p) {
    const int px = tx0 + (p & 1) * 8 + (lane & 7), py = ty0 + (p >> 1) * 8 + (lane >> 3);
    inside[p] = px < W && py < H;
    const size_t pid = inside[p] ? (size_t)py * W + px : 0;
    T[p] = final_Ts[pid];
    last[p] = n_contrib[pid];
    dp01[p] = v2f{dL_dpix[pid], dL_dpix[HW + pid]};
    dp2d[p] = v2f{dL_dpix[2 * HW + pid], dL_ddep[pid]};
  }
#pragma unroll
  for (int p = 0; p < Q; ++p) {
    T[p] = inside[p] ? T[p] : 0.f;
    last[p] = inside[p] ? last[p] : 0u;
    dp01[p] = inside[p] ? dp01[p] : v2f{0.f, 0.f};
    dp2d[p] = inside[p] ? dp2d[p] : v2f{0.f, 0.f};
    const float Tf = T[p], d0 = dp01[p].x, d1 = dp01[p].y, d2 = dp2d[p].x;
    tb[p] = kBg ? -Tf * (bg0 * d0 + bg1 * d1 + bg2 * d2) : 0.f;  // background: dL/dalpha += tb / (1 - alpha)
    na[p] = v2f{0.f, 0.f};
    // quadrant p takes gradient from list indices < mq[p] only
    uint32_t x = last[p];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, off, 64));
    mq[p] = (uint32_t)__builtin_amdgcn_readfirstlane((int)x);  // wave-uniform: an SGPR
    m = max(m, mq[p]);
#if WGSR_BWD_STATS
    uint32_t y = last[p];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) y = min(y, (uint32_t)__shfl_xor((int)y, off, 64));
    minq[p] = (uint32_t)__builtin_amdgcn_readfirstlane((int)y);
#endif
  }
  // entries behind every pixel's last contributor get no record: their slot
  // flags stay 0 (zeroed before the launch), and so does every entry no pixel
  // of the tile receives gradient from -- typically > 90 % of all pairs
  const uint32_t end = range.x + m;
  // this lane's store slot in an entry's row (an LDS-space pointer: 32-bit address math)
  using lds_f = __attribute__((address_space(3))) float;
  const uint32_t sPm = (uint32_t)(size_t)((lds_f*)(&sP[0][0]) + sum10_slot(lane));  // (LDS byte address)

  // prefetch pipeline (back to front): records of the next batch in
  // registers, ids one batch further.  A batch's partial records are written
  // at the top of the NEXT batch, from the sums left in sP, with each hit
  // entry's slot_start / ListRec loaded one batch early: the stores then sit
  // in the memory queue behind loads that are waited for only a batch later,
  // and no dependent load stands between the walk and the stores.
  uint32_t gcur = 0, gnext = 0;
  float4 nA = make_float4(0, 0, 0, 0), nB = nA, nC = nA;
  if (end >= range.x + 1 + lane) {
    gcur = point_g[end - 1 - lane];
    nA = splat[3 * (size_t)gcur];
    nB = splat[3 * (size_t)gcur + 1];
    nC = splat[3 * (size_t)gcur + 2];
  }
  if (end >= range.x + 1 + kBatch + lane) gnext = point_g[end - 1 - kBatch - lane];
  uint64_t hit_prev = 0;             // entries of the previous batch that left sums in sP
  uint32_t gid_prev = 0, ss_prev = 0;
  uint2 rw_prev = make_uint2(0u, 0u);
  uint4 tab_prev = make_uint4(0u, 0u, 0u, 0u);
  auto write_records = [&]() {
    if ((hit_prev >> lane) & 1) {
      // duplicate slot of (Gaussian, this tile): its first slot plus the
      // tile's index in the Gaussian's exact tile list (k_duplicate)
      const float4 A = sA[lane], B = sB[lane];
      const size_t k = ss_prev + pair_local(A, B, lr_rect(make_uint4(rw_prev.x, rw_prev.y, 0u, 0u)), tab_prev,
                                            (int)(tile % gx), (int)(tile / gx));
      float sv[10];
#pragma unroll
      for (int q = 0; q < 10; ++q) sv[q] = sP[lane][q];
      record_sums(A, B, sv);
      partial[3 * k] = make_float4(sv[0], sv[1], sv[2], sv[3]);
      partial[3 * k + 1] = make_float4(sv[4], sv[5], sv[6], sv[7]);
      partial[3 * k + 2] = make_float4(sv[8], sv[9], 0.f, 0.f);
      pflag[k] = 1;
      gflag[gid_prev] = 1;  // same value from every tile: a benign race
    }
  };

  for (uint32_t b_end = end; b_end > range.x; b_end = (b_end - range.x > (uint32_t)kBatch) ? b_end - kBatch : range.x) {
    const int cnt = (int)min((uint32_t)kBatch, b_end - range.x);
    // (one wave per workgroup: LDS accesses of the wave stay in order, and
    // the barriers compile to wave barriers)
    // the previous batch's records and sums, before this batch overwrites them
    float4 pA = make_float4(0, 0, 0, 0), pB = pA;
    float psv[10];
    const bool phit = (hit_prev >> lane) & 1;
    if (phit) {
      pA = sA[lane];
      pB = sB[lane];
#pragma unroll
      for (int q = 0; q < 10; ++q) psv[q] = sP[lane][q];
    }
    __syncthreads();
    sA[lane] = nA;
    sB[lane] = nB;
    sC[lane] = nC;
    __syncthreads();
    if (phit) {
      const size_t k = ss_prev + pair_local(pA, pB, lr_rect(make_uint4(rw_prev.x, rw_prev.y, 0u, 0u)), tab_prev,
                                            (int)(tile % gx), (int)(tile / gx));
      record_sums(pA, pB, psv);
      partial[3 * k] = make_float4(psv[0], psv[1], psv[2], psv[3]);
      partial[3 * k + 1] = make_float4(psv[4], psv[5], psv[6], psv[7]);
      partial[3 * k + 2] = make_float4(psv[8], psv[9], 0.f, 0.f);
      pflag[k] = 1;
      gflag[gid_prev] = 1;  // same value from every tile: a benign race
    }
    // this batch's entry of this lane: its slot data, for the write one batch on
    // (every lane loads: lanes past the batch hold id 0 or an earlier id, a
    // valid row, and a conditional load would cost register copies that wait
    // for it)
    gid_prev = gcur;
    ss_prev = slot_start[gcur];
    rw_prev = *reinterpret_cast<const uint2*>(&lrec[gcur].w);
    tab_prev = lrec[gcur].tab;
    gcur = gnext;
    if (b_end >= range.x + 1 + kBatch + lane) {
      nA = splat[3 * (size_t)gcur];
      nB = splat[3 * (size_t)gcur + 1];
      nC = splat[3 * (size_t)gcur + 2];
    }
    if (b_end >= range.x + 1 + 2 * kBatch + lane) gnext = point_g[b_end - 1 - 2 * kBatch - lane];

    const uint32_t cfirst = b_end - range.x - 1;  // tile-list index of entry j = cfirst - j
    // lane j tests entry j against each quadrant (reach ellipse and the
    // quadrant's last contributor); quadrant p's survivors are bits of qb[p]
    uint64_t qb[Q];
    {
      const uint32_t myidx = cfirst - (uint32_t)lane;
      const float4 a = sA[lane], b = sB[lane];
#pragma unroll
      for (int p = 0; p < Q; ++p) {
        const int x0 = tx0 + (p & 1) * 8, y0 = ty0 + (p >> 1) * 8;
        qb[p] = wave_ballot(lane < cnt && myidx < mq[p] && ellipse_hits(a, b, x0, x0 + 7, y0, y0 + 7));
      }
    }
    uint64_t todo = qb[0] | qb[1] | qb[2] | qb[3];
    uint64_t hitm = 0;  // entries that left a partial (wave-uniform: SGPRs, not an LDS array)
    while (todo) {
      const int j = __builtin_ctzll(todo);
      todo &= todo - 1;
      const uint32_t cidx = cfirst - j;
      const float4 A = sA[j];
      const float4 B = sB[j];
      const float4 Cc = sC[j];
      const v2f mxy{A.x, A.y}, cd{A.z, A.w}, c01{Cc.x, Cc.y}, c2d{Cc.z, Cc.w};
      const v2f d0 = mxy - p0;  // (dx, dy) for quadrant 0
      const float cxy = B.x, op = B.y;
      // pixel sums of u = G dL/dalpha (dx, dy) and of its moments; the
      // entry's constants (opacity, conic) multiply the sums afterwards
      // (record_sums)
      // (zero pairs: one 64-bit move each per entry)
      v2f g01{0.f, 0.f}, g23{0.f, 0.f}, g67{0.f, 0.f}, g89{0.f, 0.f};
      float g4 = 0.f, g5 = 0.f;  // (scalars: one FMA + one add, no pair to build)
      bool hit = false;
#if WGSR_BWD_STATS
      uint32_t st_reach = 0, st_p2 = 0, st_pix = 0;
#endif
#pragma unroll
      for (int p = 0; p < Q; ++p) {
        if (!((qb[p] >> j) & 1)) continue;  // wave-uniform: the splat cannot reach quadrant p
#if WGSR_BWD_STATS
        st_reach |= 1u << p;
#endif
        // phase 1: does entry j reach this lane's pixel of quadrant p?
        const v2f d = d0 - v2f{8.f * (p & 1), 8.f * (p >> 1)};  // (dx, dy) = mean - pixel
        const float power = splat_power(cd, cxy, d);  // log2(e) x upstream's power
        const float G = __builtin_amdgcn_exp2f(power);
        const float av = fminf(kMaxAlpha, op * G);
        const bool v = cidx < last[p] && power <= 0.0f && av >= kMinAlpha;
#if WGSR_BWD_STATS
        const uint32_t nv = (uint32_t)__builtin_popcountll(wave_ballot(v));
        if (lane == 0 && nv == 0) atomicAdd(&sStat[49], 1u);
        if (lane == 0 && cfirst < minq[p]) atomicAdd(&sStat[50], 1u);  // the batch is live at every pixel
#endif
        if (!wave_any(v)) continue;
#if WGSR_BWD_STATS
        st_p2 |= 1u << p;
        st_pix += nv;
        if (lane == 0) {
          atomicAdd(&sStat[40 + min(7u, 31u - (uint32_t)__builtin_clz(nv))], 1u);
          atomicAdd(&sStat[48], nv);
        }
#endif
        // phase 2 on the lanes whose pixel the entry reaches (exec mask): the
        // others keep T, the accumulated colour and their sums as they are.
        // Constant factors of the mean2D (0.5 W, 0.5 H) and conic (-0.5)
        // gradients are applied once per Gaussian in k_gauss_bwd.
        // colour / depth behind this contributor: upstream's accum_rec enters
        // dL/dalpha only through its dot product with dL/d(colour, depth),
        // which follows the same recurrence (accd += alpha (c.dp - accd))
        hit = true;
        if (v) {
          const float alpha = av;
          const float rinv = __builtin_amdgcn_rcpf(1.f - alpha);  // alpha <= 0.99
          const float Tn = T[p] * rinv;
          T[p] = Tn;
          const float dch = alpha * Tn;
          const v2f cp = pfma(c2d, dp2d[p], pfma(c01, dp01[p], na[p]));
          const float sd = cp.x + cp.y;
          const float dLda = kBg ? sd * Tn + tb[p] * rinv : sd * Tn;
          na[p].x = fmaf(-alpha, sd, na[p].x);
          const float gl = G * dLda;   // dL/dG / opacity
          const v2f u = gl * d;        // (G dx, G dy) dL/dG / opacity
          g01 += u;
          g23 += u.x * d;  // (G dx dx, G dx dy) dL/dG / opacity
          g4 = fmaf(u.y, d.y, g4);
          g5 += gl;
          g67 += dch * dp01[p];
          g89 += dch * dp2d[p];
        }
      }
#if WGSR_BWD_STATS
      if (lane == 0) {
        atomicAdd(&sStat[st_reach], 1u);
        atomicAdd(&sStat[16 + st_p2], 1u);
        if (st_pix) atomicAdd(&sStat[32 + min(7u, 31u - (uint32_t)__builtin_clz(st_pix))], 1u);
      }
#endif
      if (!hit) continue;  // no pixel of the tile: no partial
      const float gv[10] = {g01.x, g01.y, g23.x, g23.y, g4, g5, g67.x, g67.y, g89.x, g89.y};
      // (the entry's row offset on the scalar unit: one VALU add per entry)
      uint32_t joff;
      asm("s_mul_i32 %0, %1, 44" : "=s"(joff) : "s"(j));  // (else a 64-bit VALU multiply-add)
      wave_sum10_store_m(gv, (lds_f*)(size_t)(sPm + joff));
      hitm |= 1ull << j;
    }
    hit_prev = hitm & (cnt >= 64 ? ~0ull : ((1ull << cnt) - 1ull));
  }
  write_records();  // the last batch's
#if WGSR_BWD_STATS
  __syncthreads();
  atomicAdd(&g_bwd_stats[lane], (unsigned long long)sStat[lane]);
#endif
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_render_bwd_quad(
    const uint2* __restrict__ ranges, const uint32_t* __restrict__ order, bool global_order,
    const uint32_t* __restrict__ meta, const uint32_t* __restrict__ lists_exact,
    const uint32_t* __restrict__ lists_bins, const float4* __restrict__ splat,
    const ListRec* __restrict__ lrec, const uint32_t* __restrict__ slot_start, int W, int H, int gx, int ntiles,
    const float* __restrict__ bg, const float* __restrict__ final_Ts, const uint32_t* __restrict__ n_contrib,
    const float* __restrict__ dL_dpix, const float* __restrict__ dL_ddep, float4* __restrict__ partial,
    uint8_t* __restrict__ pflag, uint8_t* __restrict__ gflag, const ZeroJob zero) {
  __shared__ float4 sA[kBatch], sB[kBatch], sC[kBatch];
  __shared__ uint32_t sG[kBatch];
  __shared__ float sP[kBatch][11];
  __shared__ uint32_t sHit[kBatch];
  // a capacity-mode forward that overflowed its buffers (ImageLayout::meta[1])
  // leaves no gradient: the zero fill only, no record, no flag (the
  // per-Gaussian backward then finds nothing to sum); the caller's optimizer
  // steps skip on the same flag
  if (meta[1]) {
    zero_share(zero, blockIdx.x, gridDim.x, threadIdx.x, 64);
    return;
  }
#if WGSR_BWD_WGTIME
  const unsigned long long wgt0 = __builtin_amdgcn_s_memrealtime();
#endif
  // where the forward left the tile lists (ImageLayout::meta)
  const uint32_t* __restrict__ point_g = meta[0] ? lists_bins : lists_exact;
  const uint32_t tile = order[global_order ? blockIdx.x : xcd_remap(blockIdx.x, (uint32_t)ntiles)];
  const float bg0 = bg[0], bg1 = bg[1], bg2 = bg[2];
  if (bg0 == 0.f && bg1 == 0.f && bg2 == 0.f)  // (uniform)
    render_bwd_quad_tile<false>(tile, ranges, point_g, splat, lrec, slot_start, W, H, gx, bg0, bg1, bg2, final_Ts,
                                n_contrib, dL_dpix, dL_ddep, partial, pflag, gflag, sA, sB, sC, sG, sP, sHit);
  else
    render_bwd_quad_tile<true>(tile, ranges, point_g, splat, lrec, slot_start, W, H, gx, bg0, bg1, bg2, final_Ts,
                               n_contrib, dL_dpix, dL_ddep, partial, pflag, gflag, sA, sB, sC, sG, sP, sHit);
  // this tile's share of the per-Gaussian outputs' zero fill (HBM is idle
  // here; measured at 1M/1080p: render_bwd +2 % with the fill after the walk,
  // +4.5 % before it, while k_gauss_bwd drops from 86 to 49 us)
  zero_share(zero, blockIdx.x, gridDim.x, threadIdx.x, 64);
#if WGSR_BWD_WGTIME
  const unsigned long long wgt1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x < (unsigned)kWgtMax) {
    g_bwd_wgt[3 * blockIdx.x] = wgt0;
    g_bwd_wgt[3 * blockIdx.x + 1] = wgt1;
    // HW_ID (wave, SIMD, CU, SH, SE), XCC_ID and the tile
    g_bwd_wgt[3 * blockIdx.x + 2] = (unsigned long long)__builtin_amdgcn_s_getreg((4 << 0) | (31 << 11)) |
                                    ((unsigned long long)(__builtin_amdgcn_s_getreg((20 << 0) | (15 << 11)) & 15) << 32) |
                                    ((unsigned long long)tile << 40);
  }
#endif
}

// Entry pairs in the four-wave backward (k_render_bwd_seg): a wave owns one
// 8x8 quadrant, so the batch's entries that reach it are
// compacted (two consecutive survivors interleaved per field, as the
// forward's FwdPairRec) and walked in pairs: both entries' power, alpha,
// 1 / (1 - alpha), colour dot products and gradient terms in packed-FP32
// math, only the T / accumulated-colour recurrence per entry, and the two
// entries' 10 sums reduced together (wave_sum20: two independent chains in
// flight, 42 instead of 46 VALU).  A pixel an entry does not reach runs it
// with alpha = 0 and G = 0 (pass-through, zero sums).  The background enters
// as the accumulated colour's starting value: upstream's dL/dalpha term
// -T_final / (1 - alpha) (bg . dL/dpix) equals -T (prod of (1 - alpha) behind
// the entry) (bg . dL/dpix), which is what the accum_rec recurrence adds when
// it starts from bg instead of 0 -- one code path for every background.
struct BwdPairRec {
  float4 q[3];   // {x, x', y, y'}, {A.z, A.z', A.w, A.w'}, {B.x, B.x', o, o'}
  float4 c[2];   // {c0, c0', c1, c1'}, {c2, c2', depth, depth'}
  uint32_t j[2]; // batch slots
  uint32_t pad[2];
};

// (A, B, C: this lane's entry of the batch -- lane j holds entry j)
__device__ __forceinline__ uint64_t split_batch_pairs(uint64_t todo, uint32_t cfirst, const float4 A, const float4 B,
                                                      const float4 C, BwdPairRec* R, float (*sPw)[11], v2f p0,
                                                      uint32_t last, const v2f& dp01, const v2f& dp2d, float& T,
                                                      float& accd, int lane) {
  const int n = __popcll(todo);
  const uint32_t k = lanes_below(todo);
  if ((todo >> lane) & 1) {
    BwdPairRec& r = R[k >> 1];
    float* q = &r.q[0].x + (k & 1);
    q[0] = A.x; q[2] = A.y; q[4] = A.z; q[6] = A.w; q[8] = B.x; q[10] = B.y;
    float* c = &r.c[0].x + (k & 1);
    c[0] = C.x; c[2] = C.y; c[4] = C.z; c[6] = C.w;
    r.j[k & 1] = (uint32_t)lane;
  }
  if (lane == 63 && (n & 1)) {  // the unused half of an odd last pair: finite operands
    BwdPairRec& r = R[n >> 1];
    float* q = &r.q[0].x + 1;
    q[0] = 0.f; q[2] = 0.f; q[4] = 0.f; q[6] = 0.f; q[8] = 0.f; q[10] = 0.f;
    float* c = &r.c[0].x + 1;
    c[0] = 0.f; c[2] = 0.f; c[4] = 0.f; c[6] = 0.f;
    r.j[1] = 0u;
  }
  // (the wave's own LDS accesses complete in order; the instruction-free wave
  // barrier keeps the compiler from hoisting the cross-lane reads below)
  __builtin_amdgcn_wave_barrier();
  // per-lane targets of the two-entry sums (constants of the lane)
  const int yv = sum20_y_value(lane), zv = sum20_z_value(lane);
  const int yk = yv >> 1, ye = yv & 1, zk = zv >> 1, ze = zv & 1;
  const v2f px{p0.x, p0.x}, py{p0.y, p0.y};
  uint64_t hits = 0;
  for (int i = 0; i < n; i += 2) {
    const BwdPairRec& r = R[i >> 1];
    const float4 q0 = r.q[0], q1 = r.q[1], q2 = r.q[2], c0 = r.c[0], c1 = r.c[1];
    const uint2 jj = *reinterpret_cast<const uint2*>(&r.j[0]);
    const v2f DX = v2f{q0.x, q0.y} - px, DY = v2f{q0.z, q0.w} - py;
    // splat_power per lane: fma(dx, fma(B.x, dy, A.z dx), (A.w dy) dy)
    const v2f tz = v2f{q1.x, q1.y} * DX, tw = v2f{q1.z, q1.w} * DY;
    const v2f PW = pfma(DX, pfma(v2f{q2.x, q2.y}, DY, tz), tw * DY);
    const v2f G = v2f{__builtin_amdgcn_exp2f(PW.x), __builtin_amdgcn_exp2f(PW.y)};
    const v2f ag = v2f{q2.z, q2.w} * G;
    const v2f av{fminf(kMaxAlpha, ag.x), fminf(kMaxAlpha, ag.y)};
    const uint32_t ci1 = cfirst - jj.x, ci2 = cfirst - jj.y;
    const uint64_t m1 = wave_ballot(ci1 < last) & wave_ballot(PW.x <= 0.0f) & wave_ballot(av.x >= kMinAlpha);
    const uint64_t m2 = (i + 1 < n) ? (wave_ballot(ci2 < last) & wave_ballot(PW.y <= 0.0f) &
                                       wave_ballot(av.y >= kMinAlpha))
                                    : 0ull;
    if ((m1 | m2) == 0) continue;
    const bool v1 = __builtin_amdgcn_inverse_ballot_w64(m1), v2 = __builtin_amdgcn_inverse_ballot_w64(m2);
    const v2f a{v1 ? av.x : 0.f, v2 ? av.y : 0.f};
    const v2f Ge{v1 ? G.x : 0.f, v2 ? G.y : 0.f};
    const v2f om = v2f{1.f, 1.f} - a;
    const float r1 = __builtin_amdgcn_rcpf(om.x), r2 = __builtin_amdgcn_rcpf(om.y);  // alpha <= 0.99
    const float Tn1 = T * r1, Tn2 = Tn1 * r2;
    T = Tn2;
    const v2f Tn{Tn1, Tn2};
    const v2f dch = a * Tn;
    // c . dL/d(colour, depth) of both entries
    const v2f cp = pfma(v2f{c1.z, c1.w}, v2f{dp2d.y, dp2d.y},
                        pfma(v2f{c1.x, c1.y}, v2f{dp2d.x, dp2d.x},
                             pfma(v2f{c0.z, c0.w}, v2f{dp01.y, dp01.y}, v2f{c0.x, c0.y} * v2f{dp01.x, dp01.x})));
    const float sd1 = cp.x - accd;
    accd = fmaf(a.x, sd1, accd);
    const float sd2 = cp.y - accd;
    accd = fmaf(a.y, sd2, accd);
    const v2f gl = Ge * (v2f{sd1, sd2} * Tn);  // dL/dG / opacity of each entry
    v2f S[10];
    S[0] = gl * DX;
    S[1] = gl * DY;
    S[2] = S[0] * DX;
    S[3] = S[0] * DY;
    S[4] = S[1] * DY;
    S[5] = gl;
    S[6] = dch * v2f{dp01.x, dp01.x};
    S[7] = dch * v2f{dp01.y, dp01.y};
    S[8] = dch * v2f{dp2d.x, dp2d.x};
    S[9] = dch * v2f{dp2d.y, dp2d.y};
    if (m1 && m2) {
      float Y, Z;
      wave_sum20(S, Y, Z);
      float* const rowy = &sPw[ye ? jj.y : jj.x][0];
      float* const rowz = &sPw[ze ? jj.y : jj.x][0];
      if (__builtin_amdgcn_inverse_ballot_w64(kSum20StoreY)) rowy[yk] = Y;
      if (__builtin_amdgcn_inverse_ballot_w64(kSum20StoreZ)) rowz[zk] = Z;
      hits |= (1ull << jj.x) | (1ull << jj.y);
    } else if (m1) {
      float gv[10];
#pragma unroll
      for (int q = 0; q < 10; ++q) gv[q] = S[q].x;
      wave_sum10_store(gv, &sPw[jj.x][0]);
      hits |= 1ull << jj.x;
    } else {
      float gv[10];
#pragma unroll
      for (int q = 0; q < 10; ++q) gv[q] = S[q].y;
      wave_sum10_store(gv, &sPw[jj.y][0]);
      hits |= 1ull << jj.y;
    }
  }
  __builtin_amdgcn_wave_barrier();  // (the next batch's compaction writes stay behind these reads)
  return hits;
}

// Small images (few tiles: TUM's 512x384 has 768) leave most SIMDs without a
// wave under k_render_bwd_quad, and each tile's serial walk sets the time.
// Below kBwdSplitBelowTiles tiles a tile gets FOUR waves, one per 8x8
// quadrant, with the quadrant waves decoupled: every wave fetches the batch
// records itself (lane j entry j, one batch ahead in registers), culls and
// evaluates only its quadrant (entry pairs, split_batch_pairs), and leaves its
// per-entry quadrant sums in a segment table of kSegBatches batches; the four
// waves meet only once per segment, where the workgroup adds each entry's (up
// to four) quadrant sums in quadrant order and writes its record (that
// entry's slot data loaded at the segment's start).  A quadrant wave with
// less work never waits for the slowest one at a batch.  Same per-pixel
// arithmetic as the one-wave kernel; only the order of the final
// cross-quadrant sum differs.  (The batch-synchronous four-wave form, wave 0
// staging every batch for all four behind two barriers, measured 71.5-71.8
// vs 69.8-70.4 us at TUM scale and was removed in round 5.)
constexpr int kSegBatches = 3, kSegCap = kSegBatches * kBatch;
__global__ __launch_bounds__(256) void k_render_bwd_seg(
    const uint2* __restrict__ ranges, const uint32_t* __restrict__ order, bool global_order,
    const uint32_t* __restrict__ meta, const uint32_t* __restrict__ lists_exact,
    const uint32_t* __restrict__ lists_bins, const float4* __restrict__ splat,
    const ListRec* __restrict__ lrec, const uint32_t* __restrict__ slot_start, int W,
    int H, int gx, int ntiles, const float* __restrict__ bg, const float* __restrict__ final_Ts,
    const uint32_t* __restrict__ n_contrib, const float* __restrict__ dL_dpix, const float* __restrict__ dL_ddep,
    float4* __restrict__ partial, uint8_t* __restrict__ pflag, uint8_t* __restrict__ gflag, const ZeroJob zero) {
  __shared__ float sS[4][kSegCap][11];              // per quadrant: the segment's entry sums
  __shared__ uint64_t sHit[4][kSegBatches];         // per quadrant and batch: the entries it summed
  __shared__ BwdPairRec sPairs[4][kBatch / 2];      // per wave: the batch's compacted survivors
  __shared__ uint32_t sEnd[4];
  if (meta[1]) {  // overflowed capacity-mode forward (see k_render_bwd_quad)
    zero_share(zero, blockIdx.x, gridDim.x, threadIdx.x, 256);
    return;
  }
  const uint32_t* __restrict__ point_g = meta[0] ? lists_bins : lists_exact;
  const uint32_t tile = order[global_order ? blockIdx.x : xcd_remap(blockIdx.x, (uint32_t)ntiles)];
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int tx = (int)(tile % gx), ty = (int)(tile / gx);
  const int qx0 = tx * kTile + (w & 1) * 8, qy0 = ty * kTile + (w >> 1) * 8;  // this wave's quadrant
  const size_t HW = (size_t)H * W;
  const uint2 range = ranges[tile];
  const float bg0 = bg[0], bg1 = bg[1], bg2 = bg[2];

  const int px = qx0 + (lane & 7), py = qy0 + (lane >> 3);
  const v2f p0{(float)px, (float)py};
  const bool inside = px < W && py < H;
  const size_t pid = (size_t)py * W + px;
  const float Tf = inside ? final_Ts[pid] : 0.f;
  const uint32_t last = inside ? n_contrib[pid] : 0u;
  const float d0 = inside ? dL_dpix[pid] : 0.f, d1 = inside ? dL_dpix[HW + pid] : 0.f;
  const float d2 = inside ? dL_dpix[2 * HW + pid] : 0.f, dd = inside ? dL_ddep[pid] : 0.f;
  const v2f dp01{d0, d1}, dp2d{d2, dd};
  float accd = bg0 * d0 + bg1 * d1 + bg2 * d2;  // the background as the colour behind the last contributor
  float T = Tf;
  uint32_t x = last;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, off, 64));
  const uint32_t mq = (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
  if (lane == 0) sEnd[w] = mq;
  __syncthreads();
  const uint32_t end = range.x + max(max(sEnd[0], sEnd[1]), max(sEnd[2], sEnd[3]));

  // this wave's batch records, one batch ahead (lanes past the list hold
  // entry 0's: valid rows, culled by lane < cnt)
  uint32_t gnext = 0;
  float4 nA = make_float4(0, 0, 0, 0), nB = nA, nC = nA;
  if (end > range.x) {
    const uint32_t g0 = point_g[end >= range.x + 1 + lane ? end - 1 - lane : range.x];
    nA = splat[3 * (size_t)g0];
    nB = splat[3 * (size_t)g0 + 1];
    nC = splat[3 * (size_t)g0 + 2];
    gnext = point_g[end >= range.x + 1 + kBatch + lane ? end - 1 - kBatch - lane : range.x];
  }
  for (uint32_t s_end = end; s_end > range.x;) {  // segments, back to front (block-uniform)
    const uint32_t s_beg = s_end - range.x > (uint32_t)kSegCap ? s_end - kSegCap : range.x;
    const uint32_t scnt = s_end - s_beg;
    // the record writer's slot data of segment entry t (list index s_end - 1 - t),
    // in flight during the walk
    uint32_t rg = 0, rss = 0;
    float4 rA = make_float4(0, 0, 0, 0), rB = rA;
    uint2 rrw = make_uint2(0u, 0u);
    uint4 rtab = make_uint4(0u, 0u, 0u, 0u);
    if ((uint32_t)t < scnt) {
      rg = point_g[s_end - 1 - t];
      rA = splat[3 * (size_t)rg];
      rB = splat[3 * (size_t)rg + 1];
      rss = slot_start[rg];
      rrw = *reinterpret_cast<const uint2*>(&lrec[rg].w);
      rtab = lrec[rg].tab;
    }
    int bi = 0;
    for (uint32_t b_end = s_end; b_end > s_beg; b_end = b_end - s_beg > (uint32_t)kBatch ? b_end - kBatch : s_beg, ++bi) {
      const int cnt = (int)min((uint32_t)kBatch, b_end - s_beg);
      const float4 A = nA, B = nB, C = nC;
      // next batch (possibly the next segment's first)
      const uint32_t nb_end = b_end - range.x > (uint32_t)kBatch ? b_end - kBatch : range.x;
      if (nb_end > range.x) {
        const uint32_t g = gnext;
        nA = splat[3 * (size_t)g];
        nB = splat[3 * (size_t)g + 1];
        nC = splat[3 * (size_t)g + 2];
        gnext = point_g[nb_end >= range.x + 1 + kBatch + lane ? nb_end - 1 - kBatch - lane : range.x];
      }
      const uint32_t cfirst = b_end - range.x - 1;  // tile-list index of entry j = cfirst - j
      const uint64_t todo = wave_ballot(lane < cnt && cfirst - (uint32_t)lane < mq &&
                                        ellipse_hits(A, B, qx0, qx0 + 7, qy0, qy0 + 7));
      const uint64_t hits = split_batch_pairs(todo, cfirst, A, B, C, sPairs[w], &sS[w][bi * kBatch], p0, last, dp01,
                                              dp2d, T, accd, lane);
      if (lane == 0) sHit[w][bi] = hits;
    }
    __syncthreads();
    // entry t of the segment: its quadrant sums in quadrant order, its record
    if ((uint32_t)t < scnt) {
      const int b = t >> 6;
      const uint64_t bit = 1ull << (t & 63);
      const uint64_t h0 = sHit[0][b], h1 = sHit[1][b], h2 = sHit[2][b], h3 = sHit[3][b];
      if ((h0 | h1 | h2 | h3) & bit) {
        float sv[10];
#pragma unroll
        for (int k = 0; k < 10; ++k) sv[k] = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint64_t hq = q == 0 ? h0 : (q == 1 ? h1 : (q == 2 ? h2 : h3));
          if (hq & bit)
#pragma unroll
            for (int k = 0; k < 10; ++k) sv[k] += sS[q][t][k];
        }
        record_sums(rA, rB, sv);
        const size_t k = rss + pair_local(rA, rB, lr_rect(make_uint4(rrw.x, rrw.y, 0u, 0u)), rtab, tx, ty);
        partial[3 * k] = make_float4(sv[0], sv[1], sv[2], sv[3]);
        partial[3 * k + 1] = make_float4(sv[4], sv[5], sv[6], sv[7]);
        partial[3 * k + 2] = make_float4(sv[8], sv[9], 0.f, 0.f);
        pflag[k] = 1;
        gflag[rg] = 1;
      }
    }
    __syncthreads();  // (the table is rewritten by the next segment)
    s_end = s_beg;
  }
  zero_share(zero, blockIdx.x, gridDim.x, threadIdx.x, 256);
}

__device__ __forceinline__ f3 ldc(const float* sh, int k) { return mk3(sh[3 * k], sh[3 * k + 1], sh[3 * k + 2]); }

// upstream computeColorFromSH backward; returns dL/dmean and writes dL/dsh
// for all M stored coefficients (zeros past K).  `sh` and `dsh` may be the
// same row (the LDS-staged coefficients): every read precedes the writes.
// kAcc: dsh is a caller register array of 48 floats that receives += (the
// multi-view backward); otherwise dsh is written, zeros past K.
template <bool kAcc = false>
__device__ __forceinline__ f3 sh_backward(int deg, int M, const float* sh, f3 pos, f3 campos, uint32_t cbits, f3 dRGB, float* dsh) {
  const f3 dir_orig = sub3(pos, campos);
  const float len = sqrtf(dot3(dir_orig, dir_orig));
  const f3 dir = mk3(dir_orig.x / len, dir_orig.y / len, dir_orig.z / len);
  dRGB.x *= (cbits & 1u) ? 0.f : 1.f;
  dRGB.y *= (cbits & 2u) ? 0.f : 1.f;
  dRGB.z *= (cbits & 4u) ? 0.f : 1.f;
  f3 dx = mk3(0.f, 0.f, 0.f), dy = dx, dz = dx;
  const float x = dir.x, y = dir.y, z = dir.z;
  const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
  if (deg > 0) {
    dx = scl3(-SH_C1, ldc(sh, 3));
    dy = scl3(-SH_C1, ldc(sh, 1));
    dz = scl3(SH_C1, ldc(sh, 2));
    if (deg > 1) {
      dx = add3(dx, add3(add3(scl3(SH_C2[0] * y, ldc(sh, 4)), scl3(SH_C2[2] * 2.f * -x, ldc(sh, 6))),
                         add3(scl3(SH_C2[3] * z, ldc(sh, 7)), scl3(SH_C2[4] * 2.f * x, ldc(sh, 8)))));
      dy = add3(dy, add3(add3(scl3(SH_C2[0] * x, ldc(sh, 4)), scl3(SH_C2[1] * z, ldc(sh, 5))),
                         add3(scl3(SH_C2[2] * 2.f * -y, ldc(sh, 6)), scl3(SH_C2[4] * 2.f * -y, ldc(sh, 8)))));
      dz = add3(dz, add3(add3(scl3(SH_C2[1] * y, ldc(sh, 5)), scl3(SH_C2[2] * 2.f * 2.f * z, ldc(sh, 6))),
                         scl3(SH_C2[3] * x, ldc(sh, 7))));
      if (deg > 2) {
        dx = add3(dx, scl3(SH_C3[0] * 3.f * 2.f * xy, ldc(sh, 9)));
        dx = add3(dx, scl3(SH_C3[1] * yz, ldc(sh, 10)));
        dx = add3(dx, scl3(SH_C3[2] * -2.f * xy, ldc(sh, 11)));
        dx = add3(dx, scl3(SH_C3[3] * -3.f * 2.f * xz, ldc(sh, 12)));
        dx = add3(dx, scl3(SH_C3[4] * (-3.f * xx + 4.f * zz - yy), ldc(sh, 13)));
        dx = add3(dx, scl3(SH_C3[5] * 2.f * xz, ldc(sh, 14)));
        dx = add3(dx, scl3(SH_C3[6] * 3.f * (xx - yy), ldc(sh, 15)));
        dy = add3(dy, scl3(SH_C3[0] * 3.f * (xx - yy), ldc(sh, 9)));
        dy = add3(dy, scl3(SH_C3[1] * xz, ldc(sh, 10)));
        dy = add3(dy, scl3(SH_C3[2] * (-3.f * yy + 4.f * zz - xx), ldc(sh, 11)));
        dy = add3(dy, scl3(SH_C3[3] * -3.f * 2.f * yz, ldc(sh, 12)));
        dy = add3(dy, scl3(SH_C3[4] * -2.f * xy, ldc(sh, 13)));
        dy = add3(dy, scl3(SH_C3[5] * -2.f * yz, ldc(sh, 14)));
        dy = add3(dy, scl3(SH_C3[6] * -3.f * 2.f * xy, ldc(sh, 15)));
        dz = add3(dz, scl3(SH_C3[1] * xy, ldc(sh, 10)));
        dz = add3(dz, scl3(SH_C3[2] * 4.f * 2.f * yz, ldc(sh, 11)));
        dz = add3(dz, scl3(SH_C3[3] * 3.f * (2.f * zz - xx - yy), ldc(sh, 12)));
        dz = add3(dz, scl3(SH_C3[4] * 4.f * 2.f * xz, ldc(sh, 13)));
        dz = add3(dz, scl3(SH_C3[5] * (xx - yy), ldc(sh, 14)));
      }
    }
  }
  auto put = [&](int k, float wgt) {
    if (kAcc) {
      dsh[3 * k] += wgt * dRGB.x;
      dsh[3 * k + 1] += wgt * dRGB.y;
      dsh[3 * k + 2] += wgt * dRGB.z;
    } else {
      dsh[3 * k] = wgt * dRGB.x;
      dsh[3 * k + 1] = wgt * dRGB.y;
      dsh[3 * k + 2] = wgt * dRGB.z;
    }
  };
  put(0, SH_C0);
  if (deg > 0) {
    put(1, -SH_C1 * y);
    put(2, SH_C1 * z);
    put(3, -SH_C1 * x);
    if (deg > 1) {
      put(4, SH_C2[0] * xy);
      put(5, SH_C2[1] * yz);
      put(6, SH_C2[2] * (2.f * zz - xx - yy));
      put(7, SH_C2[3] * xz);
      put(8, SH_C2[4] * (xx - yy));
      if (deg > 2) {
        put(9, SH_C3[0] * y * (3.f * xx - yy));
        put(10, SH_C3[1] * xy * z);
        put(11, SH_C3[2] * y * (4.f * zz - xx - yy));
        put(12, SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy));
        put(13, SH_C3[4] * x * (4.f * zz - xx - yy));
        put(14, SH_C3[5] * z * (xx - yy));
        put(15, SH_C3[6] * x * (xx - 3.f * yy));
      }
    }
  }
  if (!kAcc)
    for (int k = 3 * (deg + 1) * (deg + 1); k < 3 * M; ++k) dsh[k] = 0.f;
  const f3 dL_ddir = mk3(dot3(dx, dRGB), dot3(dy, dRGB), dot3(dz, dRGB));
  const f3 v = dir_orig;
  const float sum2 = dot3(v, v);
  const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
  return mk3(((sum2 - v.x * v.x) * dL_ddir.x - v.y * v.x * dL_ddir.y - v.z * v.x * dL_ddir.z) * invsum32,
             (-v.x * v.y * dL_ddir.x + (sum2 - v.y * v.y) * dL_ddir.y - v.z * v.y * dL_ddir.z) * invsum32,
             (-v.x * v.z * dL_ddir.x - v.y * v.z * dL_ddir.y + (sum2 - v.z * v.z) * dL_ddir.z) * invsum32);
}

// Sum Gaussian i's flagged per-tile partial records in fixed slot order.
// Flags are read 32 slots per chunk (8 independent word loads) and packed to a
// bit mask; records are then fetched four at a time with independent loads, so
// a Gaussian with many hit tiles costs few round trips, not one per record.
__device__ __forceinline__ void sum_partials(uint32_t s0, uint32_t s1, const uint8_t* __restrict__ pflag,
                                             const float4* __restrict__ partial, float g[10]) {
#pragma unroll
  for (int q = 0; q < 10; ++q) g[q] = 0.f;
  const uint32_t* fw = reinterpret_cast<const uint32_t*>(pflag);
  for (uint32_t base = s0 & ~3u; base < s1; base += 32) {
    uint32_t m = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      uint32_t x = (base + 4 * w < s1) ? fw[(base >> 2) + w] : 0u;
      x &= 0x01010101u;  // flags are 0 / 1 bytes
      m |= ((x | (x >> 7) | (x >> 14) | (x >> 21)) & 0xFu) << (4 * w);
    }
    if (base < s0) m &= ~0u << (s0 - base);
    if (s1 - base < 32) m &= (1u << (s1 - base)) - 1u;
    while (m) {
      uint32_t kk[4];
      bool v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[u] = m != 0;
        kk[u] = base + (v[u] ? (uint32_t)__builtin_ctz(m) : 0u);
        m &= m - 1u;
      }
      float4 r[4][3];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int h = 0; h < 3; ++h) r[u][h] = v[u] ? partial[3 * (size_t)kk[u] + h] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (!v[u]) continue;
        g[0] += r[u][0].x; g[1] += r[u][0].y; g[2] += r[u][0].z; g[3] += r[u][0].w;
        g[4] += r[u][1].x; g[5] += r[u][1].y; g[6] += r[u][1].z; g[7] += r[u][1].w;
        g[8] += r[u][2].x; g[9] += r[u][2].y;
      }
    }
  }
}

// factors the render kernel leaves out of its per-pixel terms
__device__ __forceinline__ void scale_partial_sums(float g[10], int W, int H) {
  g[0] *= 0.5f * W * (1.f / kL2E);  // d(pixel x) / d(NDC x); power2 is log2(e) x power
  g[1] *= 0.5f * H * (1.f / kL2E);
  g[2] *= -0.5f;     // dG/dconic
  g[3] *= -0.5f;
  g[4] *= -0.5f;
}

// Camera-side backward of one Gaussian in one view (upstream
// computeCov2DCUDA + the projection / depth terms of preprocessCUDA backward,
// plus the w-pose gradient): from its screen-space partial sums g[10] to
// dL/dmean3D (without the SH term), dL/dcov3D and the pose gradient (rho,
// theta).  pa, pb, pe: projmatrix_raw[0], [5], [11].
struct CamBwd {
  f3 dm;
  float ocov[6];
  f3 rho, theta;
};

__device__ __forceinline__ void cam_backward(const Cam& c, float pa, float pb, float pe, f3 mean, const float cv[6],
                                             const float g[10], CamBwd& o) {
  const float dcx = g[2], dcy = g[3], dcw = g[4], ddepth = g[9];
  // ---- cov2D backward (upstream computeCov2DCUDA)
  const f3 t = xform43(c.view, mean);
  float S[3][3];
  sym3(cv, S);
  float T[2][3];
  f3 tc;
  float xm, ym;
  ewa_T(c, t, T, tc, xm, ym);
  float a, b, cc;
  cov2d(T, S, a, b, cc);
  const float denom = a * cc - b * b;
  float dL_da = 0.f, dL_db = 0.f, dL_dc = 0.f;
  const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
  float* ocov = o.ocov;
#pragma unroll
  for (int k = 0; k < 6; ++k) ocov[k] = 0.f;
  if (denom2inv != 0) {
    dL_da = denom2inv * (-cc * cc * dcx + 2 * b * cc * dcy + (denom - a * cc) * dcw);
    dL_dc = denom2inv * (-a * a * dcw + 2 * a * b * dcy + (denom - a * cc) * dcx);
    dL_db = denom2inv * 2 * (b * cc * dcx - (denom + 2 * b * b) * dcy + a * b * dcw);
    ocov[0] = T[0][0] * T[0][0] * dL_da + T[0][0] * T[1][0] * dL_db + T[1][0] * T[1][0] * dL_dc;
    ocov[3] = T[0][1] * T[0][1] * dL_da + T[0][1] * T[1][1] * dL_db + T[1][1] * T[1][1] * dL_dc;
    ocov[5] = T[0][2] * T[0][2] * dL_da + T[0][2] * T[1][2] * dL_db + T[1][2] * T[1][2] * dL_dc;
    ocov[1] = 2 * T[0][0] * T[0][1] * dL_da + (T[0][0] * T[1][1] + T[0][1] * T[1][0]) * dL_db +
              2 * T[1][0] * T[1][1] * dL_dc;
    ocov[2] = 2 * T[0][0] * T[0][2] * dL_da + (T[0][0] * T[1][2] + T[0][2] * T[1][0]) * dL_db +
              2 * T[1][0] * T[1][2] * dL_dc;
    ocov[4] = 2 * T[0][2] * T[0][1] * dL_da + (T[0][1] * T[1][2] + T[0][2] * T[1][1]) * dL_db +
              2 * T[1][1] * T[1][2] * dL_dc;
  }
  float dT[2][3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float s0 = T[0][0] * S[k][0] + T[0][1] * S[k][1] + T[0][2] * S[k][2];
    const float s1 = T[1][0] * S[k][0] + T[1][1] * S[k][1] + T[1][2] * S[k][2];
    dT[0][k] = 2 * s0 * dL_da + s1 * dL_db;
    dT[1][k] = 2 * s1 * dL_dc + s0 * dL_db;
  }
  const float dJ00 = c.Rw[0][0] * dT[0][0] + c.Rw[0][1] * dT[0][1] + c.Rw[0][2] * dT[0][2];
  const float dJ02 = c.Rw[2][0] * dT[0][0] + c.Rw[2][1] * dT[0][1] + c.Rw[2][2] * dT[0][2];
  const float dJ11 = c.Rw[1][0] * dT[1][0] + c.Rw[1][1] * dT[1][1] + c.Rw[1][2] * dT[1][2];
  const float dJ12 = c.Rw[2][0] * dT[1][0] + c.Rw[2][1] * dT[1][1] + c.Rw[2][2] * dT[1][2];
  const float tz = 1.f / tc.z, tz2 = tz * tz, tz3 = tz2 * tz;
  const f3 dL_dt = mk3(xm * -c.fx * tz2 * dJ02, ym * -c.fy * tz2 * dJ12,
                       -c.fx * tz2 * dJ00 - c.fy * tz2 * dJ11 + (2 * c.fx * tc.x) * tz3 * dJ02 +
                           (2 * c.fy * tc.y) * tz3 * dJ12);
  f3 dm = mk3(c.Rw[0][0] * dL_dt.x + c.Rw[1][0] * dL_dt.y + c.Rw[2][0] * dL_dt.z,
              c.Rw[0][1] * dL_dt.x + c.Rw[1][1] * dL_dt.y + c.Rw[2][1] * dL_dt.z,
              c.Rw[0][2] * dL_dt.x + c.Rw[1][2] * dL_dt.y + c.Rw[2][2] * dL_dt.z);
  // pose (w-pose): left perturbation of the camera point (clamped, V8) and of W
  f3 tau_rho = dL_dt;
  f3 tau_theta = cross3(tc, dL_dt);
  {
    const float J00 = c.fx / tc.z, J02 = -(c.fx * tc.x) / (tc.z * tc.z);
    const float J11 = c.fy / tc.z, J12 = -(c.fy * tc.y) / (tc.z * tc.z);
#pragma unroll
    for (int col = 0; col < 3; ++col) {
      const f3 rc = mk3(c.Rw[0][col], c.Rw[1][col], c.Rw[2][col]);
      const f3 gc = mk3(J00 * dT[0][col], J11 * dT[1][col], J02 * dT[0][col] + J12 * dT[1][col]);
      tau_theta = add3(tau_theta, cross3(rc, gc));
    }
  }
  // ---- preprocess backward: NDC means2D -> mean (through projmatrix)
  const float* pm = c.proj;
  const float4 hom = xform44(pm, mean);
  const float m_w = 1.0f / (hom.w + 0.0000001f);
  const float mul1 = (pm[0] * mean.x + pm[4] * mean.y + pm[8] * mean.z + pm[12]) * m_w * m_w;
  const float mul2 = (pm[1] * mean.x + pm[5] * mean.y + pm[9] * mean.z + pm[13]) * m_w * m_w;
  const float g2x = g[0], g2y = g[1];
  dm.x += (pm[0] * m_w - pm[3] * mul1) * g2x + (pm[1] * m_w - pm[3] * mul2) * g2y;
  dm.y += (pm[4] * m_w - pm[7] * mul1) * g2x + (pm[5] * m_w - pm[7] * mul2) * g2y;
  dm.z += (pm[8] * m_w - pm[11] * mul1) * g2x + (pm[9] * m_w - pm[11] * mul2) * g2y;
  // pose through the projection (projmatrix_raw a, b, e terms: V5) and depth
  {
    const float alpha_ = m_w, beta_ = -hom.x * m_w * m_w, gamma_ = -hom.y * m_w * m_w;
    f3 gp = add3(scl3(g2x, mk3(alpha_ * pa, 0.f, beta_ * pe)), scl3(g2y, mk3(0.f, alpha_ * pb, gamma_ * pe)));
    gp.z += ddepth;
    tau_rho = add3(tau_rho, gp);
    tau_theta = add3(tau_theta, cross3(t, gp));
  }
  dm.x += ddepth * c.view[2];
  dm.y += ddepth * c.view[6];
  dm.z += ddepth * c.view[10];
  o.dm = dm;
  o.rho = tau_rho;
  o.theta = tau_theta;
}

// Upstream computeCov3D backward: dL/dcov3D -> dL/dscale (w.r.t. the modified
// scale, V9) and dL/drotation (raw quaternion).  Linear in dL/dcov3D.
__device__ __forceinline__ void cov_to_scale_rot(float4 q, f3 sv, float scale_mod, const float ocov[6], float* o_sc,
                                                 float* o_rot) {
  float R[3][3];
  quat_rot(q, R);
  const float s3[3] = {scale_mod * sv.x, scale_mod * sv.y, scale_mod * sv.z};
  const float dS[3][3] = {{ocov[0], 0.5f * ocov[1], 0.5f * ocov[2]},
                          {0.5f * ocov[1], ocov[3], 0.5f * ocov[4]},
                          {0.5f * ocov[2], 0.5f * ocov[4], ocov[5]}};
  float Mm[3][3], dM[3][3];
#pragma unroll
  for (int r0 = 0; r0 < 3; ++r0)
#pragma unroll
    for (int c0 = 0; c0 < 3; ++c0) Mm[r0][c0] = s3[r0] * R[c0][r0];
#pragma unroll
  for (int r0 = 0; r0 < 3; ++r0)
#pragma unroll
    for (int c0 = 0; c0 < 3; ++c0)
      dM[r0][c0] = 2.f * (Mm[r0][0] * dS[0][c0] + Mm[r0][1] * dS[1][c0] + Mm[r0][2] * dS[2][c0]);
  // w.r.t. the modified scale, as upstream (V9)
#pragma unroll
  for (int k = 0; k < 3; ++k) o_sc[k] = R[0][k] * dM[k][0] + R[1][k] * dM[k][1] + R[2][k] * dM[k][2];
  float G[3][3];
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int k = 0; k < 3; ++k) G[j][k] = s3[k] * dM[k][j];
  const float rr = q.x, x = q.y, y = q.z, z = q.w;
  *reinterpret_cast<float4*>(o_rot) = make_float4(
      2 * z * (G[1][0] - G[0][1]) + 2 * y * (G[0][2] - G[2][0]) + 2 * x * (G[2][1] - G[1][2]),
      2 * y * (G[1][0] + G[0][1]) + 2 * z * (G[2][0] + G[0][2]) + 2 * rr * (G[2][1] - G[1][2]) -
          4 * x * (G[2][2] + G[1][1]),
      2 * x * (G[1][0] + G[0][1]) + 2 * rr * (G[0][2] - G[2][0]) + 2 * z * (G[2][1] + G[1][2]) -
          4 * y * (G[2][2] + G[0][0]),
      2 * rr * (G[1][0] - G[0][1]) + 2 * x * (G[2][0] + G[0][2]) + 2 * y * (G[2][1] + G[1][2]) -
          4 * z * (G[1][1] + G[0][0]));
}

// Per-Gaussian backward of a Gaussian that received gradient: from its
// screen-space sums g[10] through the camera-side backward to every output
// row (the render backward zero-filled the rows of the others).  dm_sh: the
// SH term of dL/dmean (the caller ran sh_backward first).
__device__ __forceinline__ void gauss_bwd_one(
    int i, const float g[10], const float* __restrict__ means, const float* __restrict__ scales,
    const float* __restrict__ rots, const float* __restrict__ cov_pre, f3 dm_sh, float scale_mod,
    const float* __restrict__ viewm, const float* __restrict__ projm, const float* __restrict__ praw, int W, int H,
    float tanx, float tany, float* __restrict__ o_m2d, float* __restrict__ o_col, float* __restrict__ o_opac,
    float* __restrict__ o_m3d, float* __restrict__ o_cov, float* __restrict__ o_sc, float* __restrict__ o_rot,
    float* __restrict__ o_tau) {
  const size_t i3 = 3 * (size_t)i, i6 = 6 * (size_t)i;
  const f3 mean = mk3(means[i3], means[i3 + 1], means[i3 + 2]);
  float4 q = make_float4(1.f, 0.f, 0.f, 0.f);
  f3 sv = mk3(0.f, 0.f, 0.f);
  float cv[6];
  if (cov_pre) {
#pragma unroll
    for (int k = 0; k < 6; ++k) cv[k] = cov_pre[i6 + k];
  } else {
    sv = mk3(scales[i3], scales[i3 + 1], scales[i3 + 2]);
    q = reinterpret_cast<const float4*>(rots)[i];
  }
  o_m2d[i3] = g[0]; o_m2d[i3 + 1] = g[1]; o_m2d[i3 + 2] = 0.f;
  o_opac[i] = g[5];
  o_col[i3] = g[6]; o_col[i3 + 1] = g[7]; o_col[i3 + 2] = g[8];

  Cam c;
  load_cam(c, viewm, projm, W, H, tanx, tany);
  if (!cov_pre) cov3d_from(sv, scale_mod, q, cv);
  CamBwd cb;
  cam_backward(c, praw[0], praw[5], praw[11], mean, cv, g, cb);
#pragma unroll
  for (int k = 0; k < 6; ++k) o_cov[i6 + k] = cb.ocov[k];
  const f3 dm = add3(cb.dm, dm_sh);
  const f3 tau_rho = cb.rho, tau_theta = cb.theta;
  if (!cov_pre) cov_to_scale_rot(q, sv, scale_mod, cb.ocov, &o_sc[i3], &o_rot[4 * (size_t)i]);
  o_m3d[i3] = dm.x; o_m3d[i3 + 1] = dm.y; o_m3d[i3 + 2] = dm.z;
  o_tau[i6 + 0] = tau_rho.x; o_tau[i6 + 1] = tau_rho.y; o_tau[i6 + 2] = tau_rho.z;
  o_tau[i6 + 3] = tau_theta.x; o_tau[i6 + 4] = tau_theta.y; o_tau[i6 + 5] = tau_theta.z;
}

// One wave of 64 Gaussians per workgroup (the view-sharded owner kernel below).
constexpr int kGbWave = 64;

// Per-Gaussian backward in one launch, on outputs the render backward
// zero-filled: a workgroup of 256 threads owns 256 kR Gaussians and compacts
// the ones that received gradient (gflag; ~8 % on the bench scene) into an
// LDS list; the listed Gaussians' record slots are flattened into one list
// whose flags and records every thread loads (kRecChunk slots at a time,
// coalesced, into LDS), each listed Gaussian's thread sums its own slots in
// order (deterministic), and then runs the SH and camera-side backward,
// writing only its rows.  The per-Gaussian VALU work runs on ~1/12 of the
// waves a one-lane-per-Gaussian kernel would need.  (Measured alternatives,
// removed in round 5: one lane per Gaussian over every row, 0.18 ms at
// 1M / 1080p; the two-kernel sparse path k_sum_active + k_gauss_bwd, 89 us;
// 16-lane groups per listed Gaussian with a dependent slot-range load per
// group pass, 75 us; parameters loaded ahead of the record sums, 68-70 us.)
constexpr int kGbcThreads = 256;
constexpr int kRecChunk = 512;  // flattened record slots staged in LDS at a time
// ... with 256 / 512 Gaussians per workgroup, whose smaller lists leave room
// for 768 slots at four workgroups per CU: fewer chunk round trips
#ifndef WGSR_GBC_IDX
#define WGSR_GBC_IDX 1
#endif
#ifndef WGSR_GBC_CHUNK_SMALL
#define WGSR_GBC_CHUNK_SMALL 768
#endif
template <int kR>
__global__ __launch_bounds__(kGbcThreads) void k_gauss_bwd_compact(
    int P, int D, int M, const uint8_t* __restrict__ gflag, const uint32_t* __restrict__ slot_start,
    const ListRec* __restrict__ lrec, const uint32_t* __restrict__ clamped, const float4* __restrict__ partial,
    const uint8_t* __restrict__ pflag, const float* __restrict__ means, const float* __restrict__ scales,
    const float* __restrict__ rots, const float* __restrict__ cov_pre, const float* __restrict__ shs, float scale_mod,
    const float* __restrict__ viewm, const float* __restrict__ projm, const float* __restrict__ praw,
    const float* __restrict__ campos_p, int W, int H, float tanx, float tany, const uint32_t* __restrict__ meta,
    float* __restrict__ o_m2d, float* __restrict__ o_col, float* __restrict__ o_opac, float* __restrict__ o_m3d,
    float* __restrict__ o_cov, float* __restrict__ o_sh, float* __restrict__ o_sc, float* __restrict__ o_rot,
    float* __restrict__ o_tau) {
  constexpr int NW = kGbcThreads / 64;
  constexpr int kRecChunk = kR == 4 ? wgsr::kRecChunk : WGSR_GBC_CHUNK_SMALL;
  __shared__ uint32_t s_list[(kGbcThreads * kR)];
  __shared__ uint32_t s_s0[(kGbcThreads * kR)], s_n[(kGbcThreads * kR)], s_off[(kGbcThreads * kR) + 1];
  __shared__ uint2 s_tmp4[4];
  __shared__ float s_rec[kRecChunk][10];
  __shared__ uint32_t s_wc[kR][NW];
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int i0 = blockIdx.x * (kGbcThreads * kR);
#if WGSR_GBC_TIMES
  const unsigned long long gbc_t0 = __builtin_amdgcn_s_memtime();
  if (t == 0) atomicAdd(&g_gbc_times[15], 1ull);
#endif
  // compaction of the live Gaussians (list order = index order)
  bool live[kR];
  uint64_t bal[kR];
  // (unconditional loads of clamped rows: a short-circuit load would be
  // waited for at its join, one round trip per r instead of one in all)
  uint8_t gf[kR];
#pragma unroll
  for (int r = 0; r < kR; ++r) gf[r] = gflag[min(i0 + r * kGbcThreads + t, P - 1)];
  // record slots in index order (ImageLayout::meta[2], the default sort-bin
  // forward): each row's slot range from two coalesced slot_start words,
  // loaded with the flags -- no dependent gather of the live rows' ranges
  // (the last row's end from its list length)
  const bool idx = WGSR_GBC_IDX && meta[2] != 0u;  // (uniform)
  uint32_t ss[kR], se[kR];
  if (idx) {
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const int i = min(i0 + r * kGbcThreads + t, P - 1);
      ss[r] = slot_start[i];
      se[r] = slot_start[min(i + 1, P - 1)];
    }
#pragma unroll
    for (int r = 0; r < kR; ++r)
      if (i0 + r * kGbcThreads + t == P - 1) se[r] = ss[r] + lrec[P - 1].w.w;
  }
#pragma unroll
  for (int r = 0; r < kR; ++r) live[r] = i0 + r * kGbcThreads + t < P && gf[r] != 0;
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    bal[r] = wave_ballot(live[r]);
    if (lane == 0) s_wc[r][w] = (uint32_t)__popcll(bal[r]);
  }
  __syncthreads();
  uint32_t nlive = 0;
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    uint32_t base = nlive;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      base += k < w ? s_wc[r][k] : 0u;
      nlive += s_wc[r][k];
    }
    if (live[r]) {
      const uint32_t c = base + lanes_below(bal[r]);
      s_list[c] = (uint32_t)(i0 + r * kGbcThreads + t);
      if (idx) {
        s_s0[c] = ss[r];
        s_n[c] = se[r] - ss[r];
      }
    }
  }
  if (nlive == 0) return;  // block-uniform
  __syncthreads();
  GBC_MARK(0);  // flags loaded, list built
#if WGSR_GBC_TIMES
  if (t == 0) { atomicAdd(&g_gbc_times[8], 1ull); atomicAdd(&g_gbc_times[9], (unsigned long long)nlive); }
#endif
  // record sums over the listed Gaussians' slots flattened into one list:
  // their slot ranges in one round trip, then kRecChunk slots at a time every
  // thread loads one slot's flag and record (coalesced within a range; the
  // slot's Gaussian by binary search over the range offsets) into LDS, and
  // each Gaussian's own thread sums its slots in slot order (deterministic)
  // (measured, round 5: each live row's slot range loaded by its own thread
  // during the compaction instead of this gather: the mean workgroup's clocks
  // -8 % (WGSR_GBC_TIMES) but the kernel 58.3 vs 57.8 us -- its time is the
  // slowest workgroups', the ones with the most record slots; loading every
  // row's range instead reads all of the 32-byte list records: 62 us)
  for (uint32_t c = idx ? nlive : t; c < nlive; c += kGbcThreads) {
    const uint32_t gi = s_list[c];
    s_s0[c] = slot_start[gi];
    s_n[c] = lrec[gi].w.w;
#if WGSR_GBC_TIMES
    atomicMax(&g_gbc_times[14], (unsigned long long)s_n[c]);
#endif
  }
  __syncthreads();
  GBC_MARK(1);  // slot ranges loaded
  {
    uint32_t v[kR], loc = 0;
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const uint32_t c = kR * t + r;
      v[r] = c < nlive ? s_n[c] : 0u;
      loc += v[r];
    }
    uint2 tot2;
    uint32_t ex = block_excl_scan256_2(make_uint2(loc, 0u), s_tmp4, &tot2).x;
    const uint32_t tot = tot2.x;
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const uint32_t c = kR * t + r;
      if (c < nlive) s_off[c] = ex;
      ex += v[r];
    }
    if (t == 0) s_off[nlive] = tot;
  }
  __syncthreads();
  const uint32_t total = s_off[nlive];
  GBC_MARK(2);  // scanned
#if WGSR_GBC_TIMES
  if (t == 0) atomicAdd(&g_gbc_times[10], (unsigned long long)total);
#endif
  float acc[kR][10];
#pragma unroll
  for (int r = 0; r < kR; ++r)
#pragma unroll
    for (int k = 0; k < 10; ++k) acc[r][k] = 0.f;
  // software pipeline: this thread's slots of the NEXT chunk are loaded into
  // registers while the current chunk is summed out of LDS (the loads' round
  // trip overlaps the sums and barriers instead of following them); same
  // slots, same order of the sums
  constexpr int U = kRecChunk / kGbcThreads;
  float4 ra0[U], ra1[U], ra2[U];
  bool rf[U];
  auto fetch = [&](uint32_t b) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t q = b + u * kGbcThreads + t;
      rf[u] = false;
      ra0[u] = ra1[u] = ra2[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (q < total) {
        uint32_t lo = 0, hi = nlive;  // s_off[lo] <= q < s_off[hi]
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (s_off[mid] <= q) lo = mid; else hi = mid;
        }
        const size_t sl = (size_t)s_s0[lo] + (q - s_off[lo]);
        rf[u] = pflag[sl] != 0;
        ra0[u] = partial[3 * sl];
        ra1[u] = partial[3 * sl + 1];
        ra2[u] = partial[3 * sl + 2];
      }
    }
  };
  if (total > 0) fetch(0);
  for (uint32_t base = 0; base < total; base += kRecChunk) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t q = base + u * kGbcThreads + t;
      if (q < total) {
        const bool f = rf[u];
        const float4 a0 = ra0[u], a1 = ra1[u], a2 = ra2[u];
        float* d = s_rec[q - base];
        d[0] = f ? a0.x : 0.f; d[1] = f ? a0.y : 0.f; d[2] = f ? a0.z : 0.f; d[3] = f ? a0.w : 0.f;
        d[4] = f ? a1.x : 0.f; d[5] = f ? a1.y : 0.f; d[6] = f ? a1.z : 0.f; d[7] = f ? a1.w : 0.f;
        d[8] = f ? a2.x : 0.f; d[9] = f ? a2.y : 0.f;
      }
    }
    if (base + kRecChunk < total) fetch(base + kRecChunk);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const uint32_t c = r * kGbcThreads + t;
      if (c < nlive) {
        const uint32_t qa = max(s_off[c], base), qb = min(s_off[c + 1], base + kRecChunk);
        // four slots' rows read before their adds (one LDS round trip per
        // four slots on the long ranges the slowest workgroups wait for);
        // the adds keep the slot order, so the sums are bit-identical
        uint32_t q = qa;
        for (; q + 4 <= qb; q += 4) {
          float v[4][10];
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int k = 0; k < 10; ++k) v[j][k] = s_rec[q + j - base][k];
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int k = 0; k < 10; ++k) acc[r][k] += v[j][k];
        }
        for (; q < qb; ++q)
#pragma unroll
          for (int k = 0; k < 10; ++k) acc[r][k] += s_rec[q - base][k];
      }
    }
    __syncthreads();
  }
  GBC_MARK(3);  // records summed
#if WGSR_GBC_TIMES
  if (t == 0) {
    atomicMax(&g_gbc_times[11], __builtin_amdgcn_s_memtime() - gbc_t0);   // slowest to here
    atomicMax(&g_gbc_times[12], (unsigned long long)total);               // most slots
  }
#endif
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    const uint32_t c = r * kGbcThreads + t;
    if (c >= nlive) break;
    const int i = (int)s_list[c];
    float g[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) g[k] = acc[r][k];
    scale_partial_sums(g, W, H);
    // SH backward first: its dL/dmean term goes into gauss_bwd_one's single
    // store of the row (no read-modify-write of o_m3d behind its stores)
    f3 dm_sh = mk3(0.f, 0.f, 0.f);
    if (o_sh) {
      const size_t S = 3 * (size_t)M;
      dm_sh = sh_backward(D, M, shs + (size_t)i * S, mk3(means[3 * (size_t)i], means[3 * (size_t)i + 1],
                                                        means[3 * (size_t)i + 2]),
                          mk3(campos_p[0], campos_p[1], campos_p[2]), clamped[i], mk3(g[6], g[7], g[8]),
                          o_sh + (size_t)i * S);
    }
    gauss_bwd_one(i, g, means, scales, rots, cov_pre, dm_sh, scale_mod, viewm, projm, praw, W, H, tanx, tany, o_m2d,
                  o_col, o_opac, o_m3d, o_cov, o_sc, o_rot, o_tau);
  }
#if WGSR_GBC_TIMES
  __syncthreads();
  GBC_MARK(4);  // every listed Gaussian's backward done
  if (t == 0) atomicMax(&g_gbc_times[13], __builtin_amdgcn_s_memtime() - gbc_t0);
#endif
}

// ---- view-sharded backward (wgsr/dp.py) ---------------------
// A view's backward is split at the per-Gaussian screen-space partial sums:
// k_view_records writes each Gaussian's 12-float record (the ten sums g[10]
// k_gauss_bwd would start from, its radius and SH clamp bits), so a rank can
// ship 48 bytes per Gaussian per view to the Gaussian's owner instead of
// all-reducing 59 floats of parameter gradients; the owner's
// k_gauss_bwd_views then runs the camera-side backward of every view for its
// shard and sums the views in registers.
__global__ __launch_bounds__(256) void k_view_records(int P, int P_pad, const int32_t* __restrict__ radii,
                                                      const uint32_t* __restrict__ slot_start,
                                                      const ListRec* __restrict__ lrec,
                                                      const uint32_t* __restrict__ clamped,
                                                      const uint8_t* __restrict__ pflag,
                                                      const float4* __restrict__ partial, int W, int H,
                                                      float4* __restrict__ rec) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P_pad) return;
  float g[10];
  const bool live = i < P && radii[i] > 0;
  const uint32_t s0 = live ? slot_start[i] : 0u, s1 = live ? s0 + lrec[i].w.w : 0u;
  sum_partials(s0, s1, pflag, partial, g);
  scale_partial_sums(g, W, H);
  const float r = live ? (float)radii[i] : 0.f, cb = live ? (float)clamped[i] : 0.f;
  rec[3 * (size_t)i] = make_float4(g[0], g[1], g[2], g[3]);
  rec[3 * (size_t)i + 1] = make_float4(g[4], g[5], g[6], g[7]);
  rec[3 * (size_t)i + 2] = make_float4(g[8], g[9], r, cb);
}

// Camera table row (WGSR_VIEW_CAMERA_FLOATS floats): viewmatrix[16],
// projmatrix[16], projmatrix_raw[16], campos[3], tan_fovx, tan_fovy, W, H.
__global__ __launch_bounds__(64) void k_pack_camera(const float* __restrict__ viewm, const float* __restrict__ projm,
                                                    const float* __restrict__ praw, const float* __restrict__ campos,
                                                    float tanx, float tany, int W, int H, float* __restrict__ row) {
  const int l = threadIdx.x;
  float v = 0.f;
  if (l < 16) v = viewm[l];
  else if (l < 32) v = projm[l - 16];
  else if (l < 48) v = praw[l - 32];
  else if (l < 51) v = campos[l - 48];
  else if (l == 51) v = tanx;
  else if (l == 52) v = tany;
  else if (l == 53) v = (float)W;
  else if (l == 54) v = (float)H;
  row[l] = v;
}

// Owner side: Gaussians [lo, hi), one wave per 64, the SH slab through LDS
// (as k_gauss_bwd).  For each of the nv views, the view's record (a block of
// rec_stride float4s per view, row i - lo) drives cam_backward and the SH
// backward with that view's camera; dL/dmean3D, dL/dsh, dL/dopacity and
// dL/dcov3D are summed over the views in registers, and the view-independent
// cov3D -> (scale, rotation) step runs once on the summed dL/dcov3D (it is
// linear).  Per view, the wave's pose-gradient sum goes to
// tau_blk[block][view][6] (fixed-order wave reduction: deterministic); stats
// (optional) receive the densification statistics of the reference's
// add_densification_stats summed over views: sum ||dL/dmeans2D[:2]||, the
// number of views that see the Gaussian and its largest screen radius.
__global__ __launch_bounds__(kGbWave) void k_gauss_bwd_views(
    int lo, int hi, int D, int M, const float* __restrict__ means, const float* __restrict__ scales,
    const float* __restrict__ rots, const float* __restrict__ shs, float scale_mod, int nv,
    const float* __restrict__ cams, const float4* __restrict__ rec, int64_t rec_stride, float* __restrict__ o_m3d,
    float* __restrict__ o_sh, float* __restrict__ o_opac, float* __restrict__ o_sc, float* __restrict__ o_rot,
    float* __restrict__ tau_blk, float* __restrict__ stats) {
  extern __shared__ float s_sh[];  // kGbWave x (3M + 1) floats (dynamic)
  const int lane = threadIdx.x;
  const int i0 = lo + blockIdx.x * kGbWave, i = i0 + lane;
  const int ng = min(kGbWave, hi - i0);
  const bool live = i < hi;
  const int S = 3 * M, SP = S + 1;
  const bool sh = shs != nullptr;
  const size_t i3 = 3 * (size_t)i;
  if (sh) {
    slab_to_lds(shs + (size_t)i0 * S, ng, S, s_sh, lane);
    __syncthreads();
  }
  f3 mean = mk3(0.f, 0.f, 0.f), sv = mk3(1.f, 1.f, 1.f);
  float4 q = make_float4(1.f, 0.f, 0.f, 0.f);
  if (live) {
    mean = mk3(means[i3], means[i3 + 1], means[i3 + 2]);
    sv = mk3(scales[i3], scales[i3 + 1], scales[i3 + 2]);
    q = reinterpret_cast<const float4*>(rots)[i];
  }
  float cv[6];
  cov3d_from(sv, scale_mod, q, cv);  // view independent: once per Gaussian
  float dsh[48];
#pragma unroll
  for (int k = 0; k < 48; ++k) dsh[k] = 0.f;
  f3 dm = mk3(0.f, 0.f, 0.f);
  float ocov[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float dop = 0.f, st_norm = 0.f, st_cnt = 0.f, st_rad = 0.f;
  const float4* my = rec + 3 * (size_t)(i - lo);
  for (int v = 0; v < nv; ++v) {
    float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f), r1 = r0, r2 = r0;
    if (live) {
      r0 = my[(size_t)v * rec_stride];
      r1 = my[(size_t)v * rec_stride + 1];
      r2 = my[(size_t)v * rec_stride + 2];
    }
    const bool vis = r2.z > 0.f;  // this view's radius
    f3 rho = mk3(0.f, 0.f, 0.f), theta = rho;
    if (vis) {
      const float g[10] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w, r2.x, r2.y};
      const float* t = cams + (size_t)v * WGSR_VIEW_CAMERA_FLOATS;
      Cam c;
      load_cam(c, t, t + 16, (int)t[53], (int)t[54], t[51], t[52]);
      CamBwd cb;
      cam_backward(c, t[32], t[37], t[43], mean, cv, g, cb);
      f3 dmv = cb.dm;
      if (sh)
        dmv = add3(dmv, sh_backward<true>(D, M, &s_sh[lane * SP], mean, mk3(t[48], t[49], t[50]), (uint32_t)r2.w,
                                          mk3(g[6], g[7], g[8]), dsh));
      dm = add3(dm, dmv);
#pragma unroll
      for (int k = 0; k < 6; ++k) ocov[k] += cb.ocov[k];
      dop += g[5];
      rho = cb.rho;
      theta = cb.theta;
      st_norm += sqrtf(g[0] * g[0] + g[1] * g[1]);
      st_cnt += 1.f;
      st_rad = fmaxf(st_rad, r2.z);
    }
    if (tau_blk) {
      const float tv[6] = {rho.x, rho.y, rho.z, theta.x, theta.y, theta.z};
      float* dst = tau_blk + ((size_t)blockIdx.x * nv + v) * 6;
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const float s = wave_sum(tv[k]);
        if (lane == 0) dst[k] = s;
      }
    }
  }
  if (live) {
    o_m3d[i3] = dm.x; o_m3d[i3 + 1] = dm.y; o_m3d[i3 + 2] = dm.z;
    o_opac[i] = dop;
    cov_to_scale_rot(q, sv, scale_mod, ocov, &o_sc[i3], &o_rot[4 * (size_t)i]);
    if (stats) {
      const size_t j = 3 * (size_t)(i - lo);
      stats[j] = st_norm; stats[j + 1] = st_cnt; stats[j + 2] = st_rad;
    }
  }
  if (sh) {
    // this lane's row only, then the wave moves the slab: all rows written
    // before lds_to_slab reads across lanes
#pragma unroll
    for (int k = 0; k < 48; ++k)
      if (k < S) s_sh[lane * SP + k] = dsh[k];
    __syncthreads();
    lds_to_slab(s_sh, ng, S, o_sh + (size_t)i0 * S, lane);
  }
}

}  // namespace

hipError_t launch_render_bwd(const wgsr_raster_args& a, const uint2* ranges, const uint32_t* order,
                             const uint32_t* meta, const uint32_t* lists_exact, const uint32_t* lists_bins,
                             const void* geom, const float* final_T,
                             const uint32_t* n_contrib, const float* dL_dcolor, const float* dL_ddepth,
                             float4* partial, uint8_t* pflag, const ZeroJob& zero, hipStream_t s) {
  const GeomLayout L(a.P);
  const int gx = (a.W + kTile - 1) / kTile, gy = (a.H + kTile - 1) / kTile;
  const int nt = gx * gy;
  // few tiles (small images): four waves per tile keep the SIMDs busy
  const char* env = getenv("WGSR_BWD_SPLIT_BELOW");  // read per launch: tests switch kernels
  const int split_below = env ? atoi(env) : kBwdSplitBelowTiles;
  if (nt < split_below) {
    hipLaunchKernelGGL(k_render_bwd_seg, dim3(nt), dim3(256), 0, s, ranges, order, false, meta,
                       lists_exact, lists_bins,
                       at<float4>(geom, L.splat), at<ListRec>(geom, L.lrec),
                       at<uint32_t>(geom, L.slot_start), a.W, a.H, gx, nt, a.bg, final_T, n_contrib, dL_dcolor,
                       dL_ddepth, partial, pflag, at<uint8_t>(const_cast<void*>(geom), L.gflag), zero);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_render_bwd_quad, dim3(nt), dim3(64), 0, s, ranges, order, false, meta,
                     lists_exact, lists_bins,
                     at<float4>(geom, L.splat),
                     at<ListRec>(geom, L.lrec), at<uint32_t>(geom, L.slot_start), a.W,
                     a.H, gx, nt, a.bg, final_T, n_contrib, dL_dcolor, dL_ddepth, partial, pflag,
                     at<uint8_t>(const_cast<void*>(geom), L.gflag), zero);
  return hipGetLastError();
}

hipError_t launch_gauss_bwd(const wgsr_raster_args& a, const void* geom, const float4* partial, const uint8_t* pflag,
                            const uint32_t* meta, float* dL_dmeans2D, float* dL_dcolors, float* dL_dopacity,
                            float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscales, float* dL_drot,
                            float* dL_dtau, hipStream_t s) {
  if (a.P == 0) return hipSuccess;
  const GeomLayout L(a.P);
  // (no pair listed: gflag is all zero and nothing is written)
  // the fewest Gaussians per workgroup (256, 512 or 1024) whose grid is ONE
  // resident round at four workgroups per CU (LDS-limited): the chain of
  // dependent loads per workgroup is the kernel's time, a second round
  // doubles it (measured at 1M / 1080p: 1024 per workgroup 57-58 us, 512
  // 63-64 us (two rounds), 768 68 us)
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  int nr = 1;
  while (nr < 4 && (a.P + kGbcThreads * nr - 1) / (kGbcThreads * nr) > 4 * ncu) nr *= 2;
  const int span = kGbcThreads * nr;
  hipLaunchKernelGGL(nr == 1 ? k_gauss_bwd_compact<1> : nr == 2 ? k_gauss_bwd_compact<2> : k_gauss_bwd_compact<4>,
                     dim3((a.P + span - 1) / span), dim3(kGbcThreads), 0, s, a.P,
                     a.D, a.M, at<uint8_t>(geom, L.gflag), at<uint32_t>(geom, L.slot_start),
                     at<ListRec>(geom, L.lrec), at<uint32_t>(geom, L.clamped), partial, pflag, a.means3D, a.scales,
                     a.rotations, a.cov3D_precomp, a.shs, a.scale_modifier, a.viewmatrix, a.projmatrix,
                     a.projmatrix_raw, a.campos, a.W, a.H, a.tan_fovx, a.tan_fovy, meta, dL_dmeans2D, dL_dcolors,
                     dL_dopacity, dL_dmeans3D, dL_dcov3D, a.shs ? dL_dsh : nullptr, dL_dscales, dL_drot, dL_dtau);
  return hipGetLastError();
}

hipError_t launch_view_records(const wgsr_raster_args& a, const int32_t* radii, const void* geom, const float4* partial,
                               const uint8_t* pflag, int P_pad, float* records, hipStream_t s) {
  if (P_pad == 0) return hipSuccess;
  const GeomLayout L(a.P);
  hipLaunchKernelGGL(k_view_records, dim3((P_pad + 255) / 256), dim3(256), 0, s, a.P, P_pad, radii,
                     at<uint32_t>(geom, L.slot_start), at<ListRec>(geom, L.lrec), at<uint32_t>(geom, L.clamped),
                     pflag, partial, a.W, a.H, reinterpret_cast<float4*>(records));
  return hipGetLastError();
}

hipError_t launch_pack_camera(const wgsr_raster_args& a, float* row, hipStream_t s) {
  hipLaunchKernelGGL(k_pack_camera, dim3(1), dim3(WGSR_VIEW_CAMERA_FLOATS), 0, s, a.viewmatrix, a.projmatrix,
                     a.projmatrix_raw, a.campos, a.tan_fovx, a.tan_fovy, a.W, a.H, row);
  return hipGetLastError();
}

int gauss_bwd_views_blocks(int lo, int hi) { return hi > lo ? (hi - lo + kGbWave - 1) / kGbWave : 0; }

hipError_t launch_gauss_bwd_views(const wgsr_raster_args& a, int lo, int hi, int nv, const float* cams,
                                  const float* records, int64_t rec_stride_floats, float* dL_dmeans3D, float* dL_dsh,
                                  float* dL_dopacity, float* dL_dscales, float* dL_drot, float* tau_blk, float* stats,
                                  hipStream_t s) {
  const int nb = gauss_bwd_views_blocks(lo, hi);
  if (nb == 0) return hipSuccess;
  const size_t lds = a.shs ? sizeof(float) * kGbWave * (3 * (size_t)a.M + 1) : 0;
  hipLaunchKernelGGL(k_gauss_bwd_views, dim3(nb), dim3(kGbWave), lds, s, lo, hi, a.D, a.M, a.means3D, a.scales,
                     a.rotations, a.shs, a.scale_modifier, nv, cams, reinterpret_cast<const float4*>(records),
                     rec_stride_floats / 4, dL_dmeans3D, a.shs ? dL_dsh : nullptr, dL_dopacity, dL_dscales, dL_drot,
                     tau_blk, stats);
  return hipGetLastError();
}

}  // namespace wgsr

#if WGSR_GBC_TIMES
// diagnostic build only: read and clear k_gauss_bwd_compact's phase clocks
// [0..4] cumulative s_memtime since the workgroup's start at each phase end,
// summed over workgroups with work; [8] such workgroups, [9] listed
// Gaussians, [10] record slots, [11] / [13] the slowest workgroup's clocks
// to the record sums' end / its end, [12] the most slots in one workgroup,
// [14] the largest slot range of one Gaussian, [15] workgroups launched
extern "C" int wgsr_debug_gbc_times(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(wgsr::g_gbc_times), sizeof(unsigned long long) * 16) != hipSuccess)
    return 1;
  unsigned long long z[16] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(wgsr::g_gbc_times), z, sizeof(z)) != hipSuccess;
}
#endif
#if WGSR_BWD_WGTIME
// diagnostic build only: read (and clear) the quad backward's workgroup times
extern "C" int wgsr_debug_bwd_wgtime(unsigned long long* out, int n) {
  n = n < wgsr::kWgtMax ? n : wgsr::kWgtMax;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(wgsr::g_bwd_wgt), sizeof(unsigned long long) * 3 * n) != hipSuccess)
    return 1;
  std::vector<unsigned long long> z(3 * (size_t)wgsr::kWgtMax, 0ull);
  return hipMemcpyToSymbol(HIP_SYMBOL(wgsr::g_bwd_wgt), z.data(), sizeof(unsigned long long) * z.size()) !=
         hipSuccess;
}
#endif
#if WGSR_BWD_STATS
// diagnostic build only: read and clear the quad backward's entry histogram
extern "C" int wgsr_debug_bwd_stats(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(wgsr::g_bwd_stats), sizeof(unsigned long long) * 64) != hipSuccess)
    return 1;
  unsigned long long z[64] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(wgsr::g_bwd_stats), z, sizeof(z)) != hipSuccess;
}
#endif
