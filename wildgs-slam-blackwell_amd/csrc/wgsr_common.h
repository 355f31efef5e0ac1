// Shared device helpers and buffer layouts for the gfx950 rasteriser.
//
// Everything here is CDNA4-first: 64-lane wavefronts (ballots are 64-bit),
// 256-thread workgroups (= one 16x16 pixel tile, four waves), and buffer
// regions aligned to 256 bytes so every array starts on its own cache lines.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wgsr {

constexpr int kTile = 16;             // tile edge in pixels (SURVEY A.1 BLOCK_X/Y)
constexpr int kTilePix = kTile * kTile;
constexpr int kWave = 64;
constexpr float kNearZ = 0.2f;        // near-plane cull
constexpr float kMinAlpha = 1.0f / 255.0f;
constexpr float kMaxAlpha = 0.99f;
constexpr float kMinT = 0.0001f;      // early termination
// The splat record stores the conic pre-scaled so that the render kernels get
// log2 of the Gaussian falloff directly: power2 = A.z dx^2 + A.w dy^2 + B.x dx dy
// = log2(e) * power, G = exp2(power2) (one v_exp_f32, no multiply).
constexpr float kL2E = 1.4426950408889634f;
constexpr float kConicSq = -0.5f * kL2E;  // A.z = kConicSq conic_xx, A.w = kConicSq conic_yy
constexpr float kConicXY = -kL2E;         // B.x = kConicXY conic_xy
constexpr float kUnConicSq = -2.0f / kL2E, kUnConicXY = -1.0f / kL2E;

typedef float v2f __attribute__((ext_vector_type(2)));  // packed-FP32 pair (v_pk_*)

// ---------------------------------------------------------------------------
// Wave-level primitives (wave64)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return __lane_id(); }

// number of set bits of `mask` strictly below this lane
__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// SSIM tile partials -> per-plane means and the overall mean, sums in double
// in a fixed order: threads t < 256 stride over a plane's tiles, then a
// tree over the 256 values (k_ssim_reduce; k_unc_combine runs the same
// sequence, so both give the same bits).  Every thread of the block calls it
// (blockDim >= 256); s_red: 256 doubles of LDS.  Returns the mean (all threads).
__device__ __forceinline__ float ssim_partials_mean(const float* __restrict__ partial, int64_t planes, int tiles,
                                                    double inv_plane_px, float* __restrict__ plane_mean,
                                                    double* s_red) {
  const int t = threadIdx.x;
  double total = 0.0;
  for (int64_t p = 0; p < planes; ++p) {
    double v = 0.0;
    if (t < 256)
      for (int i = t; i < tiles; i += 256) v += partial[p * tiles + i];
    if (t < 256) s_red[t] = v;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
      if (t < st) s_red[t] += s_red[t + st];
      __syncthreads();
    }
    const double ps = s_red[0];
    __syncthreads();
    total += ps;
    if (t == 0 && plane_mean) plane_mean[p] = (float)(ps * inv_plane_px);
  }
  return (float)(total * inv_plane_px / (double)planes);
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// Sum of x over each 16-lane row; lane 15 of every row ends with the row sum.
// Quad butterfly (quad_perm [1,0,3,2], [2,3,0,1]) then row_shr:4 and
// row_shr:8 with bound_ctrl (shifted-in lanes read 0): VALU-only DPP adds.
__device__ __forceinline__ float dpp_row_sum16(float x) {
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xf, 0xf, true));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xf, 0xf, true));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x114, 0xf, 0xf, true));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x118, 0xf, 0xf, true));
  return x;
}

// The same for unsigned sums / maxima (bound_ctrl zeros: the identity of both)
__device__ __forceinline__ uint32_t dpp_row_sum16_u32(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);
  return x;
}
__device__ __forceinline__ uint32_t dpp_row_max16_u32(uint32_t x) {
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xf, 0xf, true));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xf, 0xf, true));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true));
  return x;
}
// wave-uniform (SGPR) total / maximum: DPP row reductions, then the four row
// results read from lanes 15, 31, 47, 63 (no LDS round trips; all lanes active)
__device__ __forceinline__ uint32_t wave_total_u32(uint32_t x) {
  x = dpp_row_sum16_u32(x);
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 15) + (uint32_t)__builtin_amdgcn_readlane((int)x, 31) +
         (uint32_t)__builtin_amdgcn_readlane((int)x, 47) + (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}
__device__ __forceinline__ uint32_t wave_maximum_u32(uint32_t x) {
  x = dpp_row_max16_u32(x);
  return max(max((uint32_t)__builtin_amdgcn_readlane((int)x, 15), (uint32_t)__builtin_amdgcn_readlane((int)x, 31)),
             max((uint32_t)__builtin_amdgcn_readlane((int)x, 47), (uint32_t)__builtin_amdgcn_readlane((int)x, 63)));
}

__device__ __forceinline__ float2 permlane32_swap_add(float a, float b) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return make_float2(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// Wave-wide sums of 10 per-lane values, stored to dst[0..9] by 4 lanes.
// Packed butterfly for gfx950 (must be called with all 64 lanes active):
//   v_permlane32_swap pairs values (lanes 0-31 keep value 2k, 32-63 value
//   2k+1): 5 swaps + 5 adds; v_permlane16_swap pairs those by rows: 3 swaps
//   + 3 adds; then the 8- and 4-lane stages are transposed too, with
// bank-masked DPP adds (a bank = 4 lanes of a row): 3 + 2 adds instead of
// 3 x 2 row adds, then one quad butterfly on a single register, and each
// sum leaves from its own lane by ONE store (23 VALU + 1 LDS store per call
// instead of 28 + 3).  The stages' lane layouts:
//   after the 16-lane swap: row r of S0 holds value m, of S1 value 4 + m,
//   of S2 (even rows) value 8 + m, m = (r & 1) 2 + (r >> 1);
//   8-lane stage: S0's lanes 0-7 of a row += lanes 8-15, lanes 8-15 take
//   S1's lanes 0-7 + 8-15; S2's lanes 8-15 += lanes 0-7;
//   4-lane stage: S0's banks 0, 2 += banks 1, 3; bank 3 takes S2's banks 2 + 3;
//   quad butterfly: lanes 0-3 of row r end with value m, lanes 8-11 with
//   4 + m, lanes 12-15 (even rows) with 8 + m.
// value index whose sum this lane stores (-1: none)
__device__ __forceinline__ int sum10_value(int lane) {
  const int row = lane >> 4, pos = lane & 15, m = (row & 1) * 2 + (row >> 1);
  if (pos == 0) return m;
  if (pos == 8) return 4 + m;
  if (pos == 12 && !(row & 1)) return 8 + m;
  return -1;
}
// the lanes sum10_value names (a constant lane mask: no per-call compare)
constexpr uint64_t kSum10StoreLanes = (1ull << 0) | (1ull << 8) | (1ull << 12) | (1ull << 16) | (1ull << 24) |
                                      (1ull << 32) | (1ull << 40) | (1ull << 44) | (1ull << 48) | (1ull << 56);
// the lane part of a store address (callers add it once; lanes that store
// nothing get slot 0 and never write)
__device__ __forceinline__ int sum10_slot(int lane) {
  const int v = sum10_value(lane);
  return v < 0 ? 0 : v;
}
__device__ __forceinline__ void wave_sum10(const float (&v)[10], float (&S)[3]) {
  float R[5];
  uint32_t R4b = 0u;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[2 * k]), __float_as_uint(v[2 * k + 1]), false,
                                              false);
    R[k] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    if (k == 4) R4b = r[1];
  }
  {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(R[0]), __float_as_uint(R[1]), false, false);
    S[0] = __uint_as_float(r[0]) + __uint_as_float(r[1]);  // rows: v0 v2 v1 v3
    r = __builtin_amdgcn_permlane16_swap(__float_as_uint(R[2]), __float_as_uint(R[3]), false, false);
    S[1] = __uint_as_float(r[0]) + __uint_as_float(r[1]);  // rows: v4 v6 v5 v7
    // the partner register's rows only reach S[2]'s odd rows, which are never
    // stored: pass a dead register (no zero move)
    r = __builtin_amdgcn_permlane16_swap(__float_as_uint(R[4]), R4b, false, false);
    S[2] = __uint_as_float(r[0]) + __uint_as_float(r[1]);  // rows: v8 - v9 -
  }
  // bank-masked DPP adds write only the named banks; the rest of the tied
  // destination keeps its value.  Each asm opens with the 2 wait states a DPP
  // read of a just-written VGPR needs (the hazard check does not look inside
  // inline asm).
  asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_shl:8 row_mask:0xf bank_mask:0x3" : "+v"(S[0]));
  asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %1, %1 row_shr:8 row_mask:0xf bank_mask:0xc" : "+v"(S[0]) : "v"(S[1]));
  asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xc" : "+v"(S[2]));
  asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_shl:4 row_mask:0xf bank_mask:0x5" : "+v"(S[0]));
  asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %1, %1 row_shr:4 row_mask:0xf bank_mask:0xa" : "+v"(S[0]) : "v"(S[2]));
  S[0] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(S[0]), 0xB1, 0xf, 0xf, true));
  S[0] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(S[0]), 0x4E, 0xf, 0xf, true));
  asm volatile("" ::"v"(S[0]));
}
// dstm = the entry's 10 floats + sum10_slot(lane): the lane part of the
// address computed once by the caller, one address register for all stores
// (P: float* or an LDS-space float*, whose 32-bit address math per entry is
// one VALU add instead of a 64-bit multiply-add)
template <class P>
__device__ __forceinline__ void wave_sum10_store_m(const float (&v)[10], P dstm) {
  float S[3];
  wave_sum10(v, S);
  const int lane = __lane_id();
  (void)lane;
  if (__builtin_amdgcn_inverse_ballot_w64(kSum10StoreLanes)) dstm[0] = S[0];
}
__device__ __forceinline__ void wave_sum10_store(const float (&v)[10], float* dst) {
  wave_sum10_store_m(v, dst + sum10_slot(__lane_id()));
}

// Wave-wide sums of TWO entries' 10 per-lane values (pair k = (entry 0's
// value k, entry 1's value k) in one v2f), transposed through every stage
// (32- and 16-lane swaps, bank-masked 8- and 4-lane DPP adds, one quad
// butterfly on two registers): 42 VALU instead of 2 x 23.  Value index
// v = 2k + e ends in (lane-quad) positions: register Y, row r, bank b holds
// v = m + 4 (b >> 1) + 8 (b & 1); register Z, bank 3 of row r holds 16 + m;
// m = (r & 1) 2 + (r >> 1) (derived and checked by a lane-level simulation of
// these instructions; tests/test_gpu_raster.py checks the sums).
__device__ __forceinline__ void wave_sum20(const v2f (&S)[10], float& Y, float& Z) {
  float R[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(S[k].x), __float_as_uint(S[k].y), false, false);
    R[k] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  float Q[5];
#pragma unroll
  for (int m = 0; m < 5; ++m) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(R[2 * m]), __float_as_uint(R[2 * m + 1]), false, false);
    Q[m] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  // 8-lane stage: pairs (Q0, Q1), (Q2, Q3); Q4 alone (lanes 8-15 of each row)
  asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_shl:8 row_mask:0xf bank_mask:0x3" : "+v"(Q[0]));
  asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %1, %1 row_shr:8 row_mask:0xf bank_mask:0xc" : "+v"(Q[0]) : "v"(Q[1]));
  asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_shl:8 row_mask:0xf bank_mask:0x3" : "+v"(Q[2]));
  asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %1, %1 row_shr:8 row_mask:0xf bank_mask:0xc" : "+v"(Q[2]) : "v"(Q[3]));
  asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xc" : "+v"(Q[4]));
  // 4-lane stage: pair (Q0, Q2); Q4 bank 3 += bank 2
  asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_shl:4 row_mask:0xf bank_mask:0x5" : "+v"(Q[0]));
  asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %1, %1 row_shr:4 row_mask:0xf bank_mask:0xa" : "+v"(Q[0]) : "v"(Q[2]));
  asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0x8" : "+v"(Q[4]));
  Y = Q[0] + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(Q[0]), 0xB1, 0xf, 0xf, true));
  Y += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(Y), 0x4E, 0xf, 0xf, true));
  Z = Q[4] + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(Q[4]), 0xB1, 0xf, 0xf, true));
  Z += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(Z), 0x4E, 0xf, 0xf, true));
  asm volatile("" ::"v"(Y), "v"(Z));
}
// per lane: the value index wave_sum20 leaves in Y (all lanes) and in Z
// (lanes of bank 3; -1 elsewhere)
__device__ __forceinline__ int sum20_y_value(int lane) {
  const int r = lane >> 4, b = (lane >> 2) & 3, m = (r & 1) * 2 + (r >> 1);
  return m + 4 * (b >> 1) + 8 * (b & 1);
}
__device__ __forceinline__ int sum20_z_value(int lane) {
  const int r = lane >> 4, b = (lane >> 2) & 3, m = (r & 1) * 2 + (r >> 1);
  return b == 3 ? 16 + m : -1;
}
// one storing lane per quad (position 0) for Y, per row (bank 3, position 0) for Z
constexpr uint64_t kSum20StoreY = 0x1111111111111111ull;
constexpr uint64_t kSum20StoreZ = (1ull << 12) | (1ull << 28) | (1ull << 44) | (1ull << 60);

// inclusive prefix sum across the wave: four DPP row shifts (lanes shifted in
// from outside the row read 0), then row_bcast:15 into rows 1 and 3 and
// row_bcast:31 into rows 2 and 3 -- six VALU ops, no LDS round trips (the
// __shfl_up form was six ds_bpermute + twelve VALU)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}
// inclusive prefix maximum across the wave (the same DPP pattern)
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
  return v;
}

// exclusive scan of two u32 values per thread over a 256-thread block
__device__ __forceinline__ uint2 block_excl_scan256_2(uint2 v, uint2* s_tmp4, uint2* total) {
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const uint32_t ia = wave_incl_scan(v.x), ib = wave_incl_scan(v.y);
  if (lane == 63) s_tmp4[w] = make_uint2(ia, ib);
  __syncthreads();
  uint2 base = make_uint2(0u, 0u), tot = make_uint2(0u, 0u);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint2 x = s_tmp4[i];
    if (i < w) { base.x += x.x; base.y += x.y; }
    tot.x += x.x;
    tot.y += x.y;
  }
  __syncthreads();
  if (total) *total = tot;
  return make_uint2(base.x + ia - v.x, base.y + ib - v.y);
}

// Wave votes on a lane predicate that stays an SGPR lane mask (HIP's int
// __ballot / __any / __all materialise the predicate in a VGPR first).
__device__ __forceinline__ uint64_t wave_ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ bool wave_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }
__device__ __forceinline__ bool wave_all(bool p) { return __builtin_amdgcn_ballot_w64(!p) == 0; }

// Lanes (among `active`) whose low `bits` bits of d equal this lane's.
__device__ __forceinline__ uint64_t match_digit(uint32_t d, int bits, uint64_t active) {
  uint64_t peers = active;
  for (int b = 0; b < bits; ++b) {
    uint64_t on = __ballot((d >> b) & 1u);
    peers &= ((d >> b) & 1u) ? on : ~on;
  }
  return peers;
}

// Bijective XCD-aware block remap (cdna_hip_programming.md 5.5 T1): blocks
// b and b+8 run on one XCD, so give each XCD a contiguous run of work ids.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t bid, uint32_t nblocks) {
  const uint32_t q = nblocks / 8, r = nblocks % 8, xcd = bid % 8, loc = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// Tile geometry of the render kernels: PPL pixels per lane, 4 / PPL waves per
// 16x16 tile.  PPL 1: wave w owns the 8x8 quadrant (w & 1, w >> 1);
// PPL 2: wave w owns rows 8w..8w+7, lane = 1x2 pixels; PPL 4: one wave, lane =
// 2x2 quad.  Returns the pixel offset inside the tile.
template <int PPL>
__device__ __forceinline__ void tile_pixel(int w, int lane, int p, int& x, int& y) {
  const int lx = lane & 7, ly = lane >> 3;
  if constexpr (PPL == 1) {
    x = (w & 1) * 8 + lx;
    y = (w >> 1) * 8 + ly;
  } else if constexpr (PPL == 2) {
    x = 2 * lx + p;
    y = w * 8 + ly;
  } else {
    x = 2 * lx + (p & 1);
    y = 2 * ly + (p >> 1);
  }
}

// Pixel box [x0, x1] x [y0, y1] covered by wave w of a tile (tile_pixel).
template <int PPL>
__device__ __forceinline__ void wave_box(int w, int tx0, int ty0, int& x0, int& x1, int& y0, int& y1) {
  if constexpr (PPL == 1) {
    x0 = tx0 + (w & 1) * 8; y0 = ty0 + (w >> 1) * 8; x1 = x0 + 7; y1 = y0 + 7;
  } else if constexpr (PPL == 2) {
    x0 = tx0; y0 = ty0 + w * 8; x1 = x0 + 15; y1 = y0 + 7;
  } else {
    x0 = tx0; y0 = ty0; x1 = x0 + 15; y1 = y0 + 15;
  }
}

// Can a splat reach alpha >= 1/255 at any pixel centre of the rectangle
// [x0, x1] x [y0, y1]?  Record lanes: A = (mean x, mean y, conic xx, conic yy),
// B = (conic xy, opacity, lim, 0) with lim = 2 ln(255 o) (k_preprocess).
// Exact minimum of q(d) = d^T conic d over the continuous rectangle (d = mean -
// pixel, the render's convention): 0 if the mean lies inside, else the least of
// the four edge minima (q is convex; on an edge it is a 1-D parabola whose
// vertex is clamped to the edge).  The margin keeps the test conservative
// against the render's own fp32 rounding, so culling never changes a result.
// Evaluated lane-parallel (lane j tests entry j), then balloted.
__device__ __forceinline__ bool ellipse_hits(const float4& A, const float4& B, int x0, int x1, int y0, int y1) {
  const float lim = B.z;
  if (!(lim >= 0.f)) return false;
  const float ca = A.z * kUnConicSq, cb = B.x * kUnConicXY, cc = A.w * kUnConicSq;
  const float dxl = A.x - (float)x1, dxh = A.x - (float)x0;  // dx range over the rectangle
  const float dyl = A.y - (float)y1, dyh = A.y - (float)y0;
  if (dxl <= 0.f && dxh >= 0.f && dyl <= 0.f && dyh >= 0.f) return true;
  const float ica = __builtin_amdgcn_rcpf(ca), icc = __builtin_amdgcn_rcpf(cc);
  auto q = [&](float dx, float dy) { return ca * dx * dx + 2.f * cb * dx * dy + cc * dy * dy; };
  const float e0 = q(dxl, fminf(fmaxf(-cb * dxl * icc, dyl), dyh));
  const float e1 = q(dxh, fminf(fmaxf(-cb * dxh * icc, dyl), dyh));
  const float e2 = q(fminf(fmaxf(-cb * dyl * ica, dxl), dxh), dyl);
  const float e3 = q(fminf(fmaxf(-cb * dyh * ica, dxl), dxh), dyh);
  return fminf(fminf(e0, e1), fminf(e2, e3)) <= lim * 1.001f + 1e-2f;
}

template <int PPL>
__device__ __forceinline__ bool all_done(const bool (&d)[PPL]) {
  bool r = true;
#pragma unroll
  for (int p = 0; p < PPL; ++p) r = r && d[p];
  return r;
}

// ---- per-wave SH slabs: rows of S = 3M floats for 64 consecutive Gaussians
// are contiguous in HBM; they move between HBM and LDS rows padded to S + 1
// floats (a lane walking its own row is then bank-conflict free).  All loads
// of a lane are issued before its first LDS write (no load-wait-store chain);
// SH3 (S = 48) takes a fully unrolled float4 path.
template <bool kIn>
__device__ __forceinline__ void slab_move48(float* gmem, int ng, float* lds, int lane) {
  constexpr int S = 48, SP = 49, kV = 12;  // 64 rows x 48 floats = 768 float4 = 12 per lane
  const int nv4 = ng * S / 4;
  float4 v[kV];
  if (kIn) {
    const float4* src = reinterpret_cast<const float4*>(gmem);
#pragma unroll
    for (int r = 0; r < kV; ++r) {
      const int f = lane + 64 * r;
      v[r] = f < nv4 ? src[f] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
#pragma unroll
  for (int r = 0; r < kV; ++r) {
    const int f = lane + 64 * r;
    const int g = (4 * f) / S, c = 4 * f - g * S;
    float* row = lds + g * SP + c;
    if (kIn) {
      if (f < nv4) { row[0] = v[r].x; row[1] = v[r].y; row[2] = v[r].z; row[3] = v[r].w; }
    } else {
      v[r] = make_float4(row[0], row[1], row[2], row[3]);
    }
  }
  if (!kIn) {
    float4* dst = reinterpret_cast<float4*>(gmem);
#pragma unroll
    for (int r = 0; r < kV; ++r)
      if (lane + 64 * r < nv4) dst[lane + 64 * r] = v[r];
  }
}

template <bool kIn>
__device__ __forceinline__ void slab_move(float* gmem, int ng, int S, float* lds, int lane) {
  if (S == 48 && (reinterpret_cast<uintptr_t>(gmem) & 15) == 0) {
    slab_move48<kIn>(gmem, ng, lds, lane);
    return;
  }
  const int SP = S + 1, total = ng * S;
  for (int e0 = 0; e0 < total; e0 += 8 * 64) {
    float v[8];
    if (kIn) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + 64 * u + lane;
        v[u] = e < total ? gmem[e] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + 64 * u + lane;
      if (e < total) {
        const int g = e / S, c = e - g * S;
        if (kIn) lds[g * SP + c] = v[u];
        else gmem[e] = lds[g * SP + c];
      }
    }
  }
}

__device__ __forceinline__ void slab_to_lds(const float* src, int ng, int S, float* lds, int lane) {
  slab_move<true>(const_cast<float*>(src), ng, S, lds, lane);
}
__device__ __forceinline__ void lds_to_slab(const float* lds, int ng, int S, float* dst, int lane) {
  slab_move<false>(dst, ng, S, const_cast<float*>(lds), lane);
}

// ---- zero fill in the shadow of a VALU-bound kernel --------------------------
// The sparse per-Gaussian backward writes only the rows of Gaussians that
// received gradient (~8 % on the bench scene); every other row of its nine
// outputs must be zero.  The render backward is VALU-issue bound with HBM
// nearly idle, so its workgroups stream those zeros (float4 stores, a share
// each) before the per-Gaussian kernel runs.
constexpr int kZeroRegions = 9;
struct ZeroJob {
  float* p[kZeroRegions];
  uint64_t n[kZeroRegions];  // floats per region
  int count;
};

// Worker `w` of `nw` zeroes its share of every region with `nl` lanes (lane
// l): 16-byte stores over the aligned body, 4-byte stores for the unaligned
// head / tail (worker 0).  Regions must be 4-byte aligned.
__device__ __forceinline__ void zero_share(const ZeroJob& z, uint32_t w, uint32_t nw, int l, int nl) {
  for (int j = 0; j < z.count; ++j) {
    float* p = z.p[j];
    const uint64_t n = z.n[j];
    const uint64_t head = min<uint64_t>(n, ((16u - (reinterpret_cast<uintptr_t>(p) & 15u)) & 15u) >> 2);
    const uint64_t n4 = (n - head) >> 2, tail0 = head + 4 * n4;
    if (w == 0) {
      if ((uint64_t)l < head) p[l] = 0.f;
      if (tail0 + l < n) p[tail0 + l] = 0.f;
    }
    const uint64_t per = (n4 + nw - 1) / nw;
    const uint64_t b0 = min(n4, (uint64_t)w * per), b1 = min(n4, b0 + per);
    float4* q = reinterpret_cast<float4*>(p + head);
    for (uint64_t k = b0 + l; k < b1; k += nl) q[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// ---- exact tile lists -------------------------------------------------------
// A splat's reach ellipse {d : d^T conic d <= L}, L = lim * 1.001 + 0.01 (the
// render culling margin; lim = 2 ln(255 o), k_preprocess), with the invariants
// the per-row spans need.  Record lanes as in k_preprocess: A = (x, y,
// conic_xx, conic_yy), B.x = conic_xy, B.z = lim.
struct Reach {
  float mx, my, ca, cb, L, det, ey, dya, ica;
  int ok;  // 1: ellipse, 0: reaches nothing, -1: degenerate conic (keep the rect)
};

// k_preprocess (count), k_duplicate (enumerate) and k_render_bwd (slot of a
// pair) must agree bit for bit: FMA contraction is off and only single
// hardware instructions (v_sqrt_f32, v_rcp_f32) are used for sqrt / 1/x.
__device__ __forceinline__ Reach reach_of(const float4& A, const float4& B) {
#pragma clang fp contract(off)
  Reach r;
  r.mx = A.x; r.my = A.y; r.ca = A.z * kUnConicSq; r.cb = B.x * kUnConicXY;
  const float cc = A.w * kUnConicSq;
  r.L = B.z * 1.001f + 1e-2f;
  r.det = r.ca * cc - r.cb * r.cb;
  r.ok = !(B.z >= 0.f) ? 0 : (r.det > 0.f ? 1 : -1);
  const float idet = __builtin_amdgcn_rcpf(r.det);
  r.ica = __builtin_amdgcn_rcpf(r.ca);
  r.ey = __builtin_amdgcn_sqrtf(r.ca * r.L * idet);                  // |dy| extent (dy = mean y - y)
  const float dxe = __builtin_amdgcn_sqrtf(cc * r.L * idet);          // |dx| extent
  r.dya = -r.cb * __builtin_amdgcn_rcpf(cc) * dxe;                    // dy where dx = +dxe
  return r;
}

// Tile columns [xa, xa + n) of tile row ty that the reach ellipse can touch,
// clipped to the rect columns [x0, x1).  The ellipse cut by the row's band of
// pixel-centre y's is convex, so the columns it meets form one interval, found
// in closed form from the band's extreme x (+0.05 px padding for rounding).
// Pairs outside these spans cannot reach alpha >= 1/255 at any pixel of their
// tile, so they are never duplicated; upstream's getRect stays the outer bound.
__device__ __forceinline__ int row_span(const Reach& r, int ty, int x0, int x1, int& xa) {
#pragma clang fp contract(off)
  xa = x0;
  if (r.ok <= 0) return r.ok < 0 ? x1 - x0 : 0;
  const float Y0 = (float)(ty * kTile), Y1 = Y0 + (float)(kTile - 1);
  const float dlo = fmaxf(r.my - Y1, -r.ey), dhi = fminf(r.my - Y0, r.ey);
  if (dlo > dhi) return 0;
  const float ylo = fminf(fmaxf(r.dya, dlo), dhi), yhi = fminf(fmaxf(-r.dya, dlo), dhi);
  const float cL = r.ca * r.L;
  const float dmax = (-r.cb * ylo + __builtin_amdgcn_sqrtf(fmaxf(cL - r.det * ylo * ylo, 0.f))) * r.ica;
  const float dmin = (-r.cb * yhi - __builtin_amdgcn_sqrtf(fmaxf(cL - r.det * yhi * yhi, 0.f))) * r.ica;
  const float pad = 0.05f + 1e-4f * fabsf(r.mx);
  const float xlo = r.mx - dmax - pad, xhi = r.mx - dmin + pad;  // pixel x = mean x - dx
  const int a = max((int)ceilf((xlo - (float)(kTile - 1)) * (1.f / kTile)), x0);
  const int b = min((int)floorf(xhi * (1.f / kTile)) + 1, x1);
  xa = a;
  return max(b - a, 0);
}

// Per-Gaussian list record (written by k_preprocess, 32 B per Gaussian): the
// row table and w = (x0 | y0 << 16, x1 | y1 << 16, tb, tiles) -- the tile
// rectangle, the sort-bin word (exact list length | bins << 16) and the exact
// list length.  One record so the depth-order gathers of the scan and the
// duplicate fetch one 32-byte run per Gaussian, not three arrays.
struct ListRec {
  uint4 tab;
  uint4 w;
};
__device__ __forceinline__ ushort4 lr_rect(const uint4& w) {
  return make_ushort4((unsigned short)(w.x & 0xFFFFu), (unsigned short)(w.x >> 16), (unsigned short)(w.y & 0xFFFFu),
                      (unsigned short)(w.y >> 16));
}

// Row table (written by k_preprocess, 16 B per Gaussian): the spans of the
// first kRowTab rect rows as bytes, x = lengths of rows 0-3, y = rows 4-7,
// z = start columns - x0 of rows 0-3, w = rows 4-7 (rect widths are < 256
// tiles).  Rows past kRowTab are recomputed with row_span.
constexpr int kRowTab = 8;
__device__ __forceinline__ bool rowtab_ok(ushort4 rc) { return rc.z - rc.x <= 255; }
__device__ __forceinline__ uint32_t rowtab_len(const uint4& t, int k) {
  return ((k < 4 ? t.x : t.y) >> (8 * (k & 3))) & 0xFFu;
}
__device__ __forceinline__ uint32_t rowtab_x(const uint4& t, int k) {
  return ((k < 4 ? t.z : t.w) >> (8 * (k & 3))) & 0xFFu;
}

// Index of tile (tx, ty) in a splat's exact tile list (row-major over the
// rect rows from y0); the pair's duplicate slot is slot_start + this.
__device__ __forceinline__ uint32_t pair_local(const float4& A, const float4& B, ushort4 rc, const uint4& tab,
                                               int tx, int ty) {
  const int k = ty - rc.y;
  const bool use_tab = rowtab_ok(rc);
  uint32_t acc = 0;
  if (use_tab) {
    const int kt = min(k, kRowTab);
    for (int row = 0; row < kt; ++row) acc += rowtab_len(tab, row);
    if (k < kRowTab) return acc + (uint32_t)(tx - rc.x - (int)rowtab_x(tab, k));
  }
  const Reach r = reach_of(A, B);
  int xa;
  for (int row = rc.y + (use_tab ? kRowTab : 0); row < ty; ++row) acc += (uint32_t)row_span(r, row, rc.x, rc.z, xa);
  row_span(r, ty, rc.x, rc.z, xa);
  return acc + (uint32_t)(tx - xa);
}

// Two packed floats: arithmetic on these lowers to v_pk_*_f32 on gfx950.
typedef float v2f __attribute__((ext_vector_type(2)));
// packed fused multiply-add (v_pk_fma_f32): per element exactly fmaf
__device__ __forceinline__ v2f pfma(v2f a, v2f b, v2f c) { return __builtin_elementwise_fma(a, b, c); }

// log2(e) x upstream's power at (dx, dy) = mean - pixel, from the pre-scaled
// conic (cd = (A.z, A.w), cxy = B.x): A.z dx^2 + A.w dy^2 + B.x dx dy
// evaluated as dx (A.z dx + B.x dy) + A.w dy^2 -- one packed multiply and
// three scalar ops.  The forward and both backwards call this one helper, so
// the backward recomputes exactly the forward's alpha.
__device__ __forceinline__ float splat_power(v2f cd, float cxy, v2f d) {
  const v2f t = cd * d;
  return fmaf(d.x, fmaf(cxy, d.y, t.x), t.y * d.y);
}

// ---------------------------------------------------------------------------
// Small fp32 math (upstream operation order where it matters).  The geometry
// helpers below are evaluated without FMA contraction so that the per-Gaussian
// integer decisions (radius, tile rectangle) are bit-identical to the CPU
// restatement (oracle/cpu_raster.cpp, built with -ffp-contract=off).
// ---------------------------------------------------------------------------
struct f3 { float x, y, z; };
__device__ __forceinline__ f3 mk3(float x, float y, float z) { return {x, y, z}; }
__device__ __forceinline__ f3 add3(f3 a, f3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 sub3(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 scl3(float s, f3 a) { return {s * a.x, s * a.y, s * a.z}; }
__device__ __forceinline__ float dot3(f3 a, f3 b) {
#pragma clang fp contract(off)
  return a.x * b.x + a.y * b.y + a.z * b.z;
}
__device__ __forceinline__ f3 cross3(f3 a, f3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

// The caller's matrices are the row-vector (transposed) forms, read as
// column-major 4x4: m[4*c + r] = M[r][c] of the column-vector matrix.
struct Mat16 { float m[16]; };

__device__ __forceinline__ f3 xform43(const float* m, f3 p) {
#pragma clang fp contract(off)
  return {m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
          m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]};
}
__device__ __forceinline__ float4 xform44(const float* m, f3 p) {
#pragma clang fp contract(off)
  return make_float4(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                     m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14], m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]);
}
// upstream ndc2Pix evaluates in double: ((v + 1.0) * S - 1.0) * 0.5
__device__ __forceinline__ float ndc2pix(float v, int S) { return (float)(((v + 1.0) * S - 1.0) * 0.5); }

__device__ __forceinline__ void quat_rot(float4 q, float R[3][3]) {
#pragma clang fp contract(off)
  const float r = q.x, x = q.y, y = q.z, z = q.w;
  R[0][0] = 1.f - 2.f * (y * y + z * z); R[0][1] = 2.f * (x * y - r * z); R[0][2] = 2.f * (x * z + r * y);
  R[1][0] = 2.f * (x * y + r * z); R[1][1] = 1.f - 2.f * (x * x + z * z); R[1][2] = 2.f * (y * z - r * x);
  R[2][0] = 2.f * (x * z - r * y); R[2][1] = 2.f * (y * z + r * x); R[2][2] = 1.f - 2.f * (x * x + y * y);
}

// Sigma = R diag((mod s)^2) R^T, upper triangle (xx, xy, xz, yy, yz, zz)
__device__ __forceinline__ void cov3d_from(f3 s, float mod, float4 q, float c[6]) {
#pragma clang fp contract(off)
  float R[3][3];
  quat_rot(q, R);
  const float sx = mod * s.x, sy = mod * s.y, sz = mod * s.z;
  const float s2[3] = {sx * sx, sy * sy, sz * sz};
  int idx = 0;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = i; j < 3; ++j) {
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) acc += R[i][k] * s2[k] * R[j][k];
      c[idx++] = acc;
    }
}

// Camera constants every kernel needs, loaded once per thread from the
// device matrices (wave-uniform addresses -> scalar loads).
struct Cam {
  float view[16];
  float proj[16];
  float Rw[3][3];  // world->camera rotation, Rw[r][c] = view[4c + r]
  float fx, fy, tanx, tany;
  int W, H;
};

__device__ __forceinline__ void load_cam(Cam& c, const float* view, const float* proj, int W, int H,
                                         float tanx, float tany) {
#pragma unroll
  for (int i = 0; i < 16; ++i) { c.view[i] = view[i]; c.proj[i] = proj[i]; }
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int k = 0; k < 3; ++k) c.Rw[r][k] = c.view[4 * k + r];
  c.W = W; c.H = H; c.tanx = tanx; c.tany = tany;
  c.fx = W / (2.0f * tanx);
  c.fy = H / (2.0f * tany);
}

// EWA: T = J Rw (2x3) for camera-space mean t (clamped to 1.3 x the fov).
__device__ __forceinline__ void ewa_T(const Cam& c, f3 t, float T[2][3], f3& tc, float& xmul, float& ymul) {
#pragma clang fp contract(off)
  const float limx = 1.3f * c.tanx, limy = 1.3f * c.tany;
  const float txtz = t.x / t.z, tytz = t.y / t.z;
  tc = {fminf(limx, fmaxf(-limx, txtz)) * t.z, fminf(limy, fmaxf(-limy, tytz)) * t.z, t.z};
  xmul = (txtz < -limx || txtz > limx) ? 0.f : 1.f;
  ymul = (tytz < -limy || tytz > limy) ? 0.f : 1.f;
  const float J00 = c.fx / tc.z, J02 = -(c.fx * tc.x) / (tc.z * tc.z);
  const float J11 = c.fy / tc.z, J12 = -(c.fy * tc.y) / (tc.z * tc.z);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    T[0][k] = J00 * c.Rw[0][k] + J02 * c.Rw[2][k];
    T[1][k] = J11 * c.Rw[1][k] + J12 * c.Rw[2][k];
  }
}

__device__ __forceinline__ void sym3(const float c6[6], float S[3][3]) {
  S[0][0] = c6[0]; S[0][1] = c6[1]; S[0][2] = c6[2];
  S[1][0] = c6[1]; S[1][1] = c6[3]; S[1][2] = c6[4];
  S[2][0] = c6[2]; S[2][1] = c6[4]; S[2][2] = c6[5];
}

__device__ __forceinline__ void cov2d(const float T[2][3], const float S[3][3], float& a, float& b, float& c) {
#pragma clang fp contract(off)
  float ST0[3], ST1[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    ST0[i] = S[i][0] * T[0][0] + S[i][1] * T[0][1] + S[i][2] * T[0][2];
    ST1[i] = S[i][0] * T[1][0] + S[i][1] * T[1][1] + S[i][2] * T[1][2];
  }
  a = T[0][0] * ST0[0] + T[0][1] * ST0[1] + T[0][2] * ST0[2] + 0.3f;
  b = T[0][0] * ST1[0] + T[0][1] * ST1[1] + T[0][2] * ST1[2];
  c = T[1][0] * ST1[0] + T[1][1] * ST1[1] + T[1][2] * ST1[2] + 0.3f;
}

// ---------------------------------------------------------------------------
// State-buffer layouts (byte offsets inside the caller-owned uint8 buffers)
// ---------------------------------------------------------------------------
__host__ __device__ constexpr size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Radix passes: 256-thread workgroups of kSortItems keys per thread; sorts of
// up to kSmallSortN keys (the per-Gaussian depth / Morton sorts) use
// kSmallSortItems so that a 1M-key pass still spreads over ~1000 workgroups
// (4096-key tiles would leave a 1M-key pass at 245, under one per CU; 2048-key
// tiles measured faster than 1024).
#ifndef WGSR_SMALL_SORT_ITEMS
#define WGSR_SMALL_SORT_ITEMS 8
#endif
// and sorts of up to kTinySortN keys (TUM-scale frames) kTinySortItems: a
// pass over 100k keys is a single round of workgroups, whose time is one
// workgroup's latency (1024-key tiles: depth sort 52 -> 42 us at 100k)
#ifndef WGSR_TINY_SORT_ITEMS
#define WGSR_TINY_SORT_ITEMS 4
#endif
constexpr int kSortItems = 16;
constexpr int kSmallSortItems = WGSR_SMALL_SORT_ITEMS;
constexpr int kTinySortItems = WGSR_TINY_SORT_ITEMS;
constexpr size_t kSmallSortN = size_t(1) << 21;
constexpr size_t kTinySortN = size_t(1) << 18;
constexpr int kScanTile = 1024;                      // elements per scan workgroup
// elements per block of the dual (list length, bins) scan: one workgroup of
// k_duplicate_bins per block, thread <-> rank
constexpr int kPackedScanTile = 256;

__host__ __device__ inline int sort_items(size_t n) {
  return n <= kTinySortN ? kTinySortItems : (n <= kSmallSortN ? kSmallSortItems : kSortItems);
}
__host__ __device__ inline uint32_t sort_blocks(size_t n) {
  const size_t tile = 256 * (size_t)sort_items(n);
  return (uint32_t)((n + tile - 1) / tile);
}
// upstream num_rendered is accumulated in this many u64 partial sums (spread
// so that the per-wave atomics of k_preprocess do not serialise on one word)
constexpr int kRectPairLanes = 64;
// geometry counter block: u32 [0] scan total, [1] error flags, [2..3] the depth
// sort's reduced key range (launch_depth_sort),
// then u64 rect-pair partials [kRectPairLanes], u64 listed-pair partials
// [kRectPairLanes], u64 bin-pair partials [kRectPairLanes], then u32 maxima
// of the visible Gaussians' depth keys [kRectPairLanes] and of their
// complements [kRectPairLanes] (the depth sort's key range, DepthKeyPlan)
constexpr size_t kDepthRangeOffset = 16 + 3 * 8 * kRectPairLanes;
constexpr size_t kCounterBytes = kDepthRangeOffset + 2 * 4 * kRectPairLanes;

// The forward's one host wait without a copy-engine round trip: the first
// wave of the scan that follows k_preprocess sums the counter block's three
// sets of 64 u64 partials (upstream's num_rendered, the exact list pairs, the
// bin pairs) and lane 0 writes ONE aligned 16-byte record into fine-grained
// (coherent) pinned host memory: {seq << 8 | error flags | 0x80 if a count
// needs more than 32 bits, N_rect, N, N_bin}.  One store carries the sequence
// number and the counts together, so no fence orders them (a system-scope
// release would write the whole L2 back); the host polls the record.
struct PublishJob {
  const uint32_t* counter = nullptr;  // null: no publish
  uint4* host = nullptr;
  uint32_t seq = 0;
};
__device__ __forceinline__ void publish_counts(const PublishJob& pj, int lane) {
  const unsigned long long* partial = reinterpret_cast<const unsigned long long*>(pj.counter + 4);
  unsigned long long v[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    v[k] = partial[k * kRectPairLanes + lane];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v[k] += (unsigned long long)__shfl_xor((long long)v[k], off, 64);
  }
  if (lane == 0) {
    const bool big = ((v[0] | v[1] | v[2]) >> 32) != 0;
    *pj.host = make_uint4((pj.seq << 8) | (pj.counter[1] & 0x7Fu) | (big ? 0x80u : 0u), (uint32_t)v[0],
                          (uint32_t)v[1], (uint32_t)v[2]);
  }
}
static_assert(kRectPairLanes == 64, "publish_counts: one lane per partial");

// ---- depth sort over the visible key range -------------------------------------
// Depth keys are the float bits of view-space depth (> 0.2 for a visible
// Gaussian, so the bits order like the floats; culled Gaussians carry
// 0xFFFFFFFF).  The sort (sort.hip, launch_depth_sort) works on
//   key'' = key - lo_r   (visible; lo_r = the smallest visible key, low byte cleared)
//   key'' = 2^R - 1      (culled)
// with R = bits of (hi - lo_r + 1): an order-preserving map of the visible
// keys into [0, 2^R - 2] that puts the culled ones last, so a stable sort of
// key'' IS the stable sort of the keys.  Depths within [2, 8) (the bench
// scene) give R = 24: three 8-bit passes instead of four.  Pass 0 sorts the
// low byte (the raw key's low byte: lo_r has none), passes 1 and 2 split the
// remaining R - 8 bits (<= 10 each, so up to 1024 digits); R > 28 (the
// visible depths spanning more than ~32 octaves, e.g. 0.2 m .. 1e9 m) leaves
// extra_bits for one more stable pass that the host queues after it has
// read the range back with the pair counts.
constexpr int kDepthPasses = 3;
constexpr int kDepthMaxDigitBits = 10;
constexpr int kDepthMaxDigits = 1 << kDepthMaxDigitBits;
struct DepthKeyPlan {
  uint32_t lo_r, cul;
  int R;
  int shift[kDepthPasses], bits[kDepthPasses];
  int extra_shift, extra_bits;
};
__host__ __device__ inline DepthKeyPlan depth_key_plan(uint32_t hi, uint32_t lo) {
  DepthKeyPlan p;
  if (hi < lo) {  // nothing visible: every key'' is 0
    p.lo_r = 0u;
    p.cul = 0u;
    p.R = 0;
  } else {
    p.lo_r = lo & ~0xFFu;
    const uint32_t span = hi - p.lo_r + 1u;  // visible keys < 0x7F800001: no wrap
    int r = 0;
    while (r < 32 && (span >> r) != 0u) ++r;
    p.R = r;
    p.cul = r >= 32 ? 0xFFFFFFFFu : (1u << r) - 1u;
  }
  const int b0 = p.R < 8 ? p.R : 8;
  const int rest = p.R - b0;
  int b1 = (rest + 1) / 2;
  b1 = b1 > kDepthMaxDigitBits ? kDepthMaxDigitBits : b1;
  int b2 = rest - b1;
  b2 = b2 > kDepthMaxDigitBits ? kDepthMaxDigitBits : b2;
  p.shift[0] = 0;
  p.bits[0] = b0;
  p.shift[1] = b0;
  p.bits[1] = b1;
  p.shift[2] = b0 + b1;
  p.bits[2] = b2;
  p.extra_shift = b0 + b1 + b2;
  p.extra_bits = p.R - p.extra_shift;
  return p;
}
__host__ __device__ inline uint32_t depth_key_xform(const DepthKeyPlan& p, uint32_t key) {
  return key == 0xFFFFFFFFu ? p.cul : key - p.lo_r;
}

// ---- sort bins ----------------------------------------------------------------
// The (Gaussian, tile) lists are sorted as (Gaussian, BIN) pairs of 2^s x 2^s
// tiles -- ~7x fewer pairs to duplicate and radix-sort at s = 2 -- and then
// cut into the exact per-tile lists (k_expand_bins).  shift 0 = sort the
// exact (Gaussian, tile) pairs directly.
constexpr int kMaxBinShift = 2;  // the exact tile mask of a bin (2^2s bits) rides in 16 key bits
struct Bins {
  int shift, bx, by, n;  // bins per row / column, bin count
  __host__ __device__ Bins(int gx, int gy, int sh)
      : shift(sh), bx((gx + (1 << sh) - 1) >> sh), by((gy + (1 << sh) - 1) >> sh), n(bx * by) {}
  __host__ __device__ int of_tile(int tx, int ty) const { return (ty >> shift) * bx + (tx >> shift); }
};
// Onesweep radix sort scratch (sort.hip): look-back status words for up to
// kMaxSortPasses 8-bit passes, and global digit histograms + block counters.
constexpr int kMaxSortPasses = 4;
// Sized so that any sort of n' <= n keys fits (buffers sized for an upper
// bound, e.g. upstream's rectangle pair count, sort the exact count).
// Superblock mode keeps the per-block histogram [256][nb] followed by every
// pass's [256][nsup] superblock sums (nsup = ceil(nb / kSortSupBlocks)).
constexpr uint32_t kSortSupBlocks = 16;
__host__ __device__ inline size_t sort_status_bytes(size_t n) {
  const size_t tiny = n < kTinySortN ? n : kTinySortN;
  const size_t small = n < kSmallSortN ? n : kSmallSortN;
  const size_t b_tiny = (tiny + 256 * kTinySortItems - 1) / (256 * kTinySortItems);
  const size_t b_small = (small + 256 * kSmallSortItems - 1) / (256 * kSmallSortItems);
  const size_t b_large = (n + 256 * kSortItems - 1) / (256 * kSortItems);
  size_t nb = b_small > b_large ? b_small : b_large;
  nb = nb > b_tiny ? nb : b_tiny;
  const size_t nsup = (nb + kSortSupBlocks - 1) / kSortSupBlocks;
  const size_t onesweep = 256 * nb * kMaxSortPasses, sup = 256 * nb + 256 * nsup * kMaxSortPasses;
  return 4ull * (onesweep > sup ? onesweep : sup);
}
constexpr size_t kSortTotalsBytes = 4 * (kMaxSortPasses * 256 + kMaxSortPasses);
// Depth sort scratch (launch_depth_sort): per-block digit counts [nb][1024]
// followed by the three passes' superblock sums [3][nsup][1024] (zeroed by
// k_preprocess), in words.
// (sized for the smallest workgroup tile, so that any tile choice fits)
__host__ __device__ inline size_t depth_sort_blocks(size_t n) {
  return (n + 256 * (size_t)kTinySortItems - 1) / (256 * (size_t)kTinySortItems);
}
__host__ __device__ inline size_t depth_sort_sup_offset_words(size_t n) {
  return (size_t)kDepthMaxDigits * depth_sort_blocks(n);
}
__host__ __device__ inline size_t depth_sort_sup_words(size_t n) {
  const size_t nsup = (depth_sort_blocks(n) + kSortSupBlocks - 1) / kSortSupBlocks;
  return (size_t)kDepthPasses * kDepthMaxDigits * nsup;
}
__host__ __device__ inline size_t depth_sort_status_bytes(size_t n) {
  const size_t a = 4 * (depth_sort_sup_offset_words(n) + depth_sort_sup_words(n)), b = sort_status_bytes(n);
  return a > b ? a : b;
}

// Per-Gaussian state (geometry buffer).
// The dual scan's block sums are also summed per kScanSupBlocks consecutive
// blocks (atomics into a zeroed region), so k_duplicate_bins derives its
// blocks' exclusive prefix without a scan kernel in between.
constexpr uint32_t kScanSupBlocks = 16;
constexpr uint32_t kScanSupStride = 16;  // uint2 per superblock sum: one 128-byte line each (atomic spread)
__host__ __device__ inline size_t packed_scan_supers(size_t n) {
  const size_t nbs = (n + kPackedScanTile - 1) / kPackedScanTile;
  return (nbs + kScanSupBlocks - 1) / kScanSupBlocks;
}

struct GeomLayout {
  size_t splat, lrec, clamped, dkey, dkey_alt, dval, dval_alt, offs, slot_start, tb, hist,
      totals, bsum, bsup, counter, gflag, total;
  __host__ __device__ explicit GeomLayout(size_t P) {
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o = align256(o + bytes); return r; };
    splat = take(48 * P);          // float4 x3: (x, y, conic_xx, conic_yy) (conic_xy, opacity, lim, -) (r, g, b, depth)
    lrec = take(32 * P);           // ListRec: row table, tile rectangle, sort-bin word, exact list length
    clamped = take(4 * P);         // SH clamp flags (3 bits)
    dkey = take(4 * P);            // depth sort keys / sorted keys
    dkey_alt = take(4 * P);
    dval = take(4 * P);            // depth order: rank -> Gaussian id
    dval_alt = take(4 * P);
    offs = take(4 * (P + 1));      // rank -> first duplicate slot
    slot_start = take(4 * P);      // Gaussian -> first duplicate slot
    tb = take(4 * P);              // sort bins: the list records' tb words, dense (the scan's gather stays in L2)
    hist = take(depth_sort_status_bytes(P));  // radix sort scratch (depth sort; the fix-up pass)
    totals = take(kSortTotalsBytes);
    bsum = take(8 * ((P + kPackedScanTile - 1) / kPackedScanTile + 1));  // uint2 block sums of the (dual) scans
    bsup = take(8 * kScanSupStride * (packed_scan_supers(P) + 1));  // uint2 sums of kScanSupBlocks block sums
    counter = take(kCounterBytes);  // see kCounterBytes
    gflag = take(P);               // per Gaussian: some tile's backward wrote a partial record
                                   // (zeroed by k_preprocess, set by the render backward)
    total = o;
  }
};

// Per-pair state (binning buffer).
struct BinLayout {
  size_t key, key_alt, slot_g, point_g, flag, hist, totals, total;
  __host__ __device__ BinLayout(size_t N) {
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o = align256(o + bytes); return r; };
    key = take(4 * N);       // tile id per pair (sorted in place of key/key_alt)
    key_alt = take(4 * N);
    slot_g = take(4 * N);    // duplicate slot -> Gaussian id (the sort's payload)
    point_g = take(4 * N);   // sorted pair -> Gaussian id (the tile lists)
    flag = take(N);          // per duplicate slot: backward record written (zeroed by k_duplicate)
    hist = take(sort_status_bytes(N));    // radix sort look-back status
    totals = take(kSortTotalsBytes);
    total = o;
  }
};

// Per-pixel state (image buffer).
struct ImageLayout {
  size_t ranges, tile_len, tile_m, order_bwd, meta, final_T, n_contrib, total;
  __host__ __device__ ImageLayout(int W, int H) {
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o = align256(o + bytes); return r; };
    const size_t nt = (size_t)((W + kTile - 1) / kTile) * ((H + kTile - 1) / kTile);
    ranges = take(8 * nt);     // list [start, end) per tile
    tile_len = take(4 * nt);   // list length per tile (forward work)
    tile_m = take(16 * nt);    // deepest contributor per tile quadrant (backward work)
    order_bwd = take(4 * nt);  // the backward's launch order (heaviest first per XCD chunk)
    meta = take(16);           // [0]: where the forward left the tile lists (1: sort-bin region
                               // after the binning layout, 0: point_g) -- read by the backward;
                               // [1]: capacity-mode overflow (the backward leaves no gradient);
                               // [2]: the record slots follow the Gaussian index order
    final_T = take(4 * (size_t)W * H);
    n_contrib = take(4 * (size_t)W * H);
    total = o;
  }
};

template <typename T>
__host__ __device__ inline T* at(void* base, size_t off) { return reinterpret_cast<T*>(static_cast<char*>(base) + off); }
template <typename T>
__host__ __device__ inline const T* at(const void* base, size_t off) {
  return reinterpret_cast<const T*>(static_cast<const char*>(base) + off);
}

}  // namespace wgsr
