// The uncertainty MLP of WildGS-SLAM's mapping loss, gfx950 (SURVEY.md 8(f)
// row f2: src/utils/dyn_uncertainty/uncertainty_model.py:5-68, MLPNetwork with
// its defaults -- input C (384 DINO features), two hidden layers of 64 with
// ReLU and dropout 0.2 (applied unconditionally, :55), one output, softplus).
// It runs on every mapping iteration over the [H/14, W/14] feature map.
//
//   mlp_fwd     64 (or, for few rows, 16) rows per workgroup: layer 1 as a
//               rows x 64 x C tile product with X and W1 staged through LDS in
//               64-wide K slabs, bias + ReLU + dropout in registers, layer 2
//               from LDS, layer 3 + softplus; keeps the post-dropout
//               activations and the pre-softplus output for the backward.
//   mlp_bwd     64 rows x one 64-column chunk of dW1 per workgroup:
//               softplus', layer 3, the two ReLU/dropout masks (read off the
//               kept activations: a kept activation is > 0 exactly when ReLU
//               passed and dropout kept it), per-workgroup partial weight /
//               bias gradients.
//   mlp_reduce  sums the per-workgroup partials in a fixed order
//               (deterministic), one thread per parameter element.
// Dropout masks come from a counter hash of (seed, layer, row, column) -- the
// same draw in forward and backward, and reproducible from the seed
// (wgsr/mlp.py restates it for the tests).  Everything is fp32.
#include <stdlib.h>

#include "wgsr_common.h"
#include "wgsr_internal.h"

namespace wgsr {

namespace {

constexpr int kHid = 64;    // hidden width (MLPNetwork default)
constexpr int kRows = 64;   // rows per workgroup
constexpr int kLd = 65;     // padded LDS row

__device__ __forceinline__ uint32_t mix32(uint32_t x) {  // lowbias32
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// keep (1) or drop (0) for element (row, col) of dropout layer `layer`
__device__ __forceinline__ bool keep_elem(uint32_t seed, int layer, uint32_t row, int col, float p) {
  const uint32_t h = mix32(seed ^ mix32((uint32_t)layer * 0x9E3779B9U ^ mix32(row * 64U + (uint32_t)col)));
  return (float)(h >> 8) * (1.0f / 16777216.0f) >= p;
}

// acc[4][CW] += A[rows ty*4.., k] * B[cols tx*CW.., k] over k in [0, 64) (both in LDS, [.][kLd])
template <int CW>
__device__ __forceinline__ void tile_mac_cw(const float (*A)[kLd], const float (*B)[kLd], int ty, int tx,
                                            float (&acc)[4][CW]) {
#pragma unroll 8
  for (int k = 0; k < 64; ++k) {
    float a[4], b[CW];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = A[ty * 4 + i][k];
#pragma unroll
    for (int j = 0; j < CW; ++j) b[j] = B[tx * CW + j][k];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < CW; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
  }
}

// dst[r][c] = src[(r0 + r) * ld + c0 + c] for an R x 64 slab (zeros past n rows)
template <int R = 64>
__device__ __forceinline__ void load_slab(float (*dst)[kLd], const float* __restrict__ src, int r0, int n, int ld,
                                          int c0) {
  for (int e = threadIdx.x; e < R * 64; e += 256) {
    const int r = e >> 6, c = e & 63;
    dst[r][c] = (r0 + r < n) ? src[(size_t)(r0 + r) * ld + c0 + c] : 0.f;
  }
}

// R rows per workgroup (64, or 16 when there are few rows: more workgroups);
// each thread owns 4 rows x R/16 columns of every 64-wide layer output.
template <int R>
__global__ __launch_bounds__(256) void k_mlp_fwd(int N, int C, const float* __restrict__ X,
                                                 const float* __restrict__ W1, const float* __restrict__ b1,
                                                 const float* __restrict__ W2, const float* __restrict__ b2,
                                                 const float* __restrict__ W3, const float* __restrict__ b3, float p,
                                                 uint32_t seed, const uint32_t* __restrict__ seed_dev,
                                                 float* __restrict__ h1d, float* __restrict__ h2d,
                                                 float* __restrict__ o_pre, float* __restrict__ u) {
  constexpr int CW = R / 16, TXN = 64 / CW;
  if (seed_dev) seed = *seed_dev;  // (a graph-replayed forward: this step's seed from device memory)
  __shared__ float sA[R][kLd], sB[64][kLd];
  const int t = threadIdx.x, ty = t / TXN, tx = t % TXN;
  const int r0 = blockIdx.x * R;
  const float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  float acc[4][CW] = {};
  for (int k0 = 0; k0 < C; k0 += 64) {
    __syncthreads();
    load_slab<R>(sA, X, r0, N, C, k0);
    load_slab(sB, W1, 0, kHid, C, k0);
    __syncthreads();
    tile_mac_cw<CW>(sA, sB, ty, tx, acc);
  }
  __syncthreads();
  // layer 1 epilogue -> sA (the R x 64 layer-2 input), h1d
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < CW; ++j) {
      const int r = ty * 4 + i, c = tx * CW + j;
      float v = fmaxf(acc[i][j] + b1[c], 0.f);
      v = keep_elem(seed, 0, (uint32_t)(r0 + r), c, p) ? v * scale : 0.f;
      sA[r][c] = v;
      if (r0 + r < N) h1d[(size_t)(r0 + r) * kHid + c] = v;
      acc[i][j] = 0.f;
    }
  load_slab(sB, W2, 0, kHid, kHid, 0);
  __syncthreads();
  tile_mac_cw<CW>(sA, sB, ty, tx, acc);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < CW; ++j) {
      const int r = ty * 4 + i, c = tx * CW + j;
      float v = fmaxf(acc[i][j] + b2[c], 0.f);
      v = keep_elem(seed, 1, (uint32_t)(r0 + r), c, p) ? v * scale : 0.f;
      sA[r][c] = v;  // layer-3 input
      if (r0 + r < N) h2d[(size_t)(r0 + r) * kHid + c] = v;
    }
  __syncthreads();
  if (t < R && r0 + t < N) {
    float o = 0.f;
    for (int k = 0; k < kHid; ++k) o = fmaf(sA[t][k], W3[k], o);
    o += b3[0];
    o_pre[r0 + t] = o;
    u[r0 + t] = o > 20.f ? o : log1pf(expf(o));  // nn.Softplus(beta 1, threshold 20)
  }
}

// Few rows (the mapper's 27 x 36 feature map, the DINO term's ~300
// samples): 16 rows per workgroup with the whole of W1, the rows' C
// features and W2 streamed into LDS in ONE round of LDS-DMA loads
// (global_load_lds, 16 B per lane: no staging registers, every load in
// flight at once -- instead of a K-slab loop of dependent load -> barrier ->
// multiply-add steps), then layers 1 and 2 on the f32 matrix cores (one
// 16 x 16 output tile per wave, one b32 LDS read per operand and step) and
// layer 3 from LDS.  Same sums in the same k order as k_mlp_fwd: bit-identical
// outputs.  (The VALU form -- b128 LDS reads, each wave's four rows
// broadcast, 16 FMAs per five reads -- ran 18.9 us on the mapper's 1275 rows.)
constexpr int kSmallRows = 16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
__host__ __device__ inline size_t mlp_small_lds(int C) {
  return sizeof(float) * ((size_t)(kHid + kSmallRows) * C + (size_t)kHid * kHid + (size_t)kSmallRows * 68);
}
// Two row segments in one launch (wgsr_mlp_forward_seg2): rows [0, N1) are
// X's with the seed `seed`, rows [N1, N) X2's rows 0, 1, ... with `seed2` --
// the dropout draw of each segment is the one its own launch would make
// (row numbers restart at the segment), outputs stay contiguous.
struct MlpSeg2 {
  int N1;                                  // rows of the first segment (N: none after it)
  const float* X2;                         // the second segment's rows
  uint32_t seed2;
  const uint32_t* seed2_dev;
};
__device__ __forceinline__ bool seg2_keep(uint32_t seed, const MlpSeg2& sg, uint32_t seed2, int layer, uint32_t row,
                                          int col, float p) {
  const bool second = (int)row >= sg.N1;
  return keep_elem(second ? seed2 : seed, layer, second ? row - (uint32_t)sg.N1 : row, col, p);
}

template <int kC>
__global__ __launch_bounds__(256) void k_mlp_fwd_small(int N, const float* __restrict__ X,
                                                       const float* __restrict__ W1, const float* __restrict__ b1,
                                                       const float* __restrict__ W2, const float* __restrict__ b2,
                                                       const float* __restrict__ W3, const float* __restrict__ b3,
                                                       float p, uint32_t seed, const uint32_t* __restrict__ seed_dev,
                                                       float* __restrict__ h1d, float* __restrict__ h2d,
                                                       float* __restrict__ o_pre, float* __restrict__ u,
                                                       const MlpSeg2 sg) {
  constexpr int C4 = kC / 4;  // float4s per row
  extern __shared__ float4 s_mlp4[];
  float4* const sW = s_mlp4;                       // [64][C4], chunk k4 of row c at k4 ^ (c & 15)
  float4* const sX = sW + kHid * C4;               // [16][C4]
  float4* const sW2 = sX + kSmallRows * C4;        // [64][16], swizzled as sW
  float* const sH = reinterpret_cast<float*>(sW2 + kHid * 16);  // [16][68] layer inputs
  if (seed_dev) seed = *seed_dev;
  const uint32_t seed2 = sg.seed2_dev ? *sg.seed2_dev : sg.seed2;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int r0 = blockIdx.x * kSmallRows;
  const float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  {
    typedef __attribute__((address_space(3))) void* lds_ptr;
    const float4* W1v = reinterpret_cast<const float4*>(W1);
    const float4* W2v = reinterpret_cast<const float4*>(W2);
    const float4* Xv = reinterpret_cast<const float4*>(X);
    constexpr int NW1 = kHid * C4 / 256, NX = kSmallRows * C4 / 256, NW2 = kHid * 16 / 256;
    static_assert(NW1 * 256 == kHid * C4 && NX * 256 == kSmallRows * C4, "C: a multiple of 64");
#pragma unroll
    for (int q = 0; q < NW1; ++q) {  // wave w fills slots [(w NW1 + q) 64, +64)
      const int sl = (w * NW1 + q) * 64 + lane, c = sl / C4, k4 = sl - c * C4;
      __builtin_amdgcn_global_load_lds((const void*)(W1v + c * C4 + (k4 ^ (c & 15))),
                                       (lds_ptr)(sW + (w * NW1 + q) * 64), 16, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < NX; ++q) {  // rows past N re-read row N - 1 (their outputs are not stored)
      const int sl = (w * NX + q) * 64 + lane, r = sl / C4, k4 = sl - r * C4;
      const int rr = min(r0 + r, N - 1);
      const float4* src = rr < sg.N1 ? Xv + (size_t)rr * C4 : reinterpret_cast<const float4*>(sg.X2) + (size_t)(rr - sg.N1) * C4;
      __builtin_amdgcn_global_load_lds((const void*)(src + (k4 ^ (r & 15))), (lds_ptr)(sX + (w * NX + q) * 64), 16, 0,
                                       0);
    }
#pragma unroll
    for (int q = 0; q < NW2; ++q) {
      const int sl = (w * NW2 + q) * 64 + lane, c = sl >> 4, k4 = sl & 15;
      __builtin_amdgcn_global_load_lds((const void*)(W2v + c * 16 + (k4 ^ (c & 15))),
                                       (lds_ptr)(sW2 + (w * NW2 + q) * 64), 16, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);  // (this wave's DMA has landed; the barrier covers the others)
  }
  __syncthreads();
  // layer 1 on the matrix cores: wave w owns output columns 16 w .. 16 w + 15
  // of the 16 rows; v_mfma_f32_16x16x4_f32 step m sums k = 4 m + (lane >> 4)
  // (A: row lane & 15 of X, B: column 16 w + (lane & 15) of W1), and its
  // result is the k-ordered fmaf chain -- the same sums in the same order as
  // the VALU kernels (k_mlp_fwd): bit-identical.  X and W1 rows sit in LDS
  // with their float4 chunks XOR-swizzled by row & 15, so the 64 lanes' b32
  // reads of a step hit 64 distinct banks.
  const int ar = lane & 15, kh = lane >> 4, wc = 16 * w + ar;
  const float* const sXf = reinterpret_cast<const float*>(sX);
  const float* const sWf = reinterpret_cast<const float*>(sW);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
  for (int m = 0; m < C4; ++m) {
    const float a = sXf[4 * (ar * C4 + (m ^ ar)) + kh];
    const float b = sWf[4 * (wc * C4 + (m ^ (wc & 15))) + kh];
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  }
  // D: column wc, rows 4 kh + i
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 4 * kh + i;
    float v = fmaxf(acc[i] + b1[wc], 0.f);
    v = seg2_keep(seed, sg, seed2, 0, (uint32_t)(r0 + r), wc, p) ? v * scale : 0.f;
    sH[r * 68 + wc] = v;
    if (r0 + r < N) h1d[(size_t)(r0 + r) * kHid + wc] = v;
  }
  __syncthreads();
  // layer 2 likewise (sH rows of 68 floats: conflict-free without a swizzle)
  const float* const sW2f = reinterpret_cast<const float*>(sW2);
  acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const float a = sH[ar * 68 + 4 * m + kh];
    const float b = sW2f[4 * (wc * 16 + (m ^ (wc & 15))) + kh];
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 4 * kh + i;
    float v = fmaxf(acc[i] + b2[wc], 0.f);
    v = seg2_keep(seed, sg, seed2, 1, (uint32_t)(r0 + r), wc, p) ? v * scale : 0.f;
    sH[r * 68 + wc] = v;  // layer-3 input
    if (r0 + r < N) h2d[(size_t)(r0 + r) * kHid + wc] = v;
  }
  __syncthreads();
  if (t < kSmallRows && r0 + t < N) {
    float o = 0.f;
    for (int k = 0; k < kHid; ++k) o = fmaf(sH[t * 68 + k], W3[k], o);
    o += b3[0];
    o_pre[r0 + t] = o;
    u[r0 + t] = o > 20.f ? o : log1pf(expf(o));  // nn.Softplus(beta 1, threshold 20)
  }
}

// partial layout per workgroup: dW1 [64][C] | db1 [64] | dW2 [64][64] | db2 [64] | dW3 [64] | db3
__host__ __device__ inline int mlp_partial_floats(int C) { return kHid * C + kHid + kHid * kHid + kHid + kHid + 1; }

__global__ __launch_bounds__(256) void k_mlp_bwd(int N, int C, const float* __restrict__ X,
                                                 const float* __restrict__ W2, const float* __restrict__ W3, float p,
                                                 const float* __restrict__ h1d, const float* __restrict__ h2d,
                                                 const float* __restrict__ o_pre, const float* __restrict__ du,
                                                 float* __restrict__ part, float du_scale) {
  __shared__ float sH1[64][kLd], sDA2[64][kLd], sDA1[64][kLd], sT[64][kLd];
  __shared__ float sDo[kRows];
  const int t = threadIdx.x, ty = t >> 4, tx = t & 15;
  const int r0 = blockIdx.x * kRows;
  const float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  float* out = part + (size_t)blockIdx.x * mlp_partial_floats(C);
  float* gW1 = out;
  float* gb1 = gW1 + kHid * C;
  float* gW2 = gb1 + kHid;
  float* gb2 = gW2 + kHid * kHid;
  float* gW3 = gb2 + kHid;
  float* gb3 = gW3 + kHid;
  if (t < kRows) {
    float d = 0.f;
    if (r0 + t < N) {
      const float o = o_pre[r0 + t], g = du[r0 + t] * du_scale;
      const float z = expf(o);
      d = o > 20.f ? g : g * z / (z + 1.f);  // softplus backward
    }
    sDo[t] = d;
  }
  load_slab(sH1, h1d, r0, N, kHid, 0);
  load_slab(sT, h2d, r0, N, kHid, 0);
  __syncthreads();
  // layer 3: dW3[k] = sum_r do[r] h2d[r][k], db3; dA2 = do W3 through ReLU/dropout
  const bool head = blockIdx.y == 0;  // writes the non-dW1 gradients
  if (head && t < kHid) {
    float s = 0.f;
    for (int r = 0; r < kRows; ++r) s = fmaf(sDo[r], sT[r][t], s);
    gW3[t] = s;
  } else if (head && t == kHid) {
    float s = 0.f;
    for (int r = 0; r < kRows; ++r) s += sDo[r];
    gb3[0] = s;
  }
  for (int e = t; e < 64 * 64; e += 256) {
    const int r = e >> 6, c = e & 63;
    sDA2[r][c] = sT[r][c] > 0.f ? sDo[r] * W3[c] * scale : 0.f;
  }
  __syncthreads();
  // dW2[o][i] = sum_r dA2[r][o] h1d[r][i]: transpose so tile_mac's K runs over rows
  // (head chunk only; the block-uniform branch keeps every barrier matched)
  if (head) {
  for (int e = t; e < 64 * 64; e += 256) {
    const int r = e >> 6, c = e & 63;
    sT[c][r] = sDA2[r][c];  // sT[o][r]
  }
  __syncthreads();
  {
    // h1d transposed into sDA1 temporarily: sDA1[i][r]
    for (int e = t; e < 64 * 64; e += 256) {
      const int r = e >> 6, c = e & 63;
      sDA1[c][r] = sH1[r][c];
    }
    __syncthreads();
    float acc[4][4] = {};
    tile_mac_cw<4>(sT, sDA1, ty, tx, acc);  // acc[o][i]
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) gW2[(ty * 4 + i) * kHid + tx * 4 + j] = acc[i][j];
  }
  }  // head
  if (head && t < kHid) {
    float s = 0.f;
    for (int r = 0; r < kRows; ++r) s += sDA2[r][t];
    gb2[t] = s;
  }
  __syncthreads();
  // dA1[r][i] = sum_o dA2[r][o] W2[o][i] through ReLU/dropout: B = W2 transposed (sDA1[i][o])
  for (int e = t; e < 64 * 64; e += 256) {
    const int o = e >> 6, i = e & 63;
    sDA1[i][o] = W2[o * kHid + i];
  }
  __syncthreads();
  {
    float acc[4][4] = {};
    tile_mac_cw<4>(sDA2, sDA1, ty, tx, acc);  // acc[r][i]
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = ty * 4 + i, c = tx * 4 + j;
        sT[c][r] = sH1[r][c] > 0.f ? acc[i][j] * scale : 0.f;  // sT[i][r] = dA1 transposed
      }
  }
  __syncthreads();
  if (head && t < kHid) {
    float s = 0.f;
    for (int r = 0; r < kRows; ++r) s += sT[t][r];
    gb1[t] = s;
  }
  // dW1[o][c] = sum_r dA1[r][o] X[r][c], 64 columns of X at a time (sDA1[c][r] = X slab transposed)
  // this workgroup's 64-column chunk of dW1 (grid.y splits C; every chunk
  // recomputes the cheap 64 x 64 part above, chunk 0 alone writes it)
  for (int c0 = 64 * (int)blockIdx.y; c0 < 64 * (int)blockIdx.y + 64; c0 += 64) {
    __syncthreads();
    for (int e = t; e < 64 * 64; e += 256) {
      const int r = e >> 6, c = e & 63;
      sDA1[c][r] = (r0 + r < N) ? X[(size_t)(r0 + r) * C + c0 + c] : 0.f;
    }
    __syncthreads();
    float acc[4][4] = {};
    tile_mac_cw<4>(sT, sDA1, ty, tx, acc);  // acc[o][c]
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) gW1[(size_t)(ty * 4 + i) * C + c0 + tx * 4 + j] = acc[i][j];
  }
}

// k_mlp_bwd with every global load issued up front: the kept activations,
// W2 and the X slab stream into LDS by LDS-DMA (no staging registers, one
// round trip instead of three), and the three products run on the matrix
// cores (tile_mac_mfma).  Rows past N re-read row N - 1 (finite) and get a
// zero upstream gradient, so they add nothing.  Same products summed in the
// same order as k_mlp_bwd: bit-identical partials.  (Its VALU form -- one
// b128 LDS read per k, 16 FMAs per five reads -- ran 14.9 us on the mapper's
// 1275 rows.)
// (two row segments as k_mlp_fwd_small's: rows >= N1 take X2's rows and the
// upstream gradient du2 x du_scale2)
struct MlpBwdSeg2 {
  int N1;
  const float* X2;
  const float* du2;
  float du_scale2;
};

// The three 64 x 64 x 64 products of k_mlp_bwd2 on the f32 matrix cores.
// A operands: [64][kLdM] LDS rows (16 rows x 4 k of one step hit 64 distinct
// banks); B operands: [64][64] images whose element (k, c) sits at bsw(k, c),
// the float4 chunks of row k XOR-moved by 16 (k & 3) floats, so the four k of
// a step (lanes 16 apart, same column) hit distinct banks.
constexpr int kLdM = 68;
__device__ __forceinline__ int bsw(int k, int c) { return k * 64 + (c ^ ((k & 3) << 4)); }

// acc[j]: this wave's 16 x 16 tile j of sum_k A[row][k] Bt[k][col] -- rows
// 16 w + 4 (lane >> 4) + i (i: the register), columns 16 j + (lane & 15) --
// as v_mfma_f32_16x16x4_f32 steps over k = 0 .. 63 in order: the k-ordered
// fmaf chain of k_mlp_bwd's tile_mac_cw, bit for bit.
__device__ __forceinline__ void tile_mac_mfma(const float (*A)[kLdM], const float* __restrict__ Bt, int w, int lane,
                                              f32x4 (&acc)[4]) {
  const int ar = 16 * w + (lane & 15), kh = lane >> 4, bc = lane & 15;
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int m = 0; m < 16; ++m) {
    const int k = 4 * m + kh;
    const float a = A[ar][k];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, Bt[bsw(k, 16 * j + bc)], acc[j], 0, 0, 0);
  }
}
__global__ __launch_bounds__(256) void k_mlp_bwd2(int N, int C, const float* __restrict__ X,
                                                  const float* __restrict__ W2, const float* __restrict__ W3, float p,
                                                  const float* __restrict__ h1d, const float* __restrict__ h2d,
                                                  const float* __restrict__ o_pre, const float* __restrict__ du,
                                                  float* __restrict__ part, float du_scale, const MlpBwdSeg2 sg) {
  __shared__ float4 sH1v[1024], sH2v[1024], sW2v[1024], sXv[1024];  // [64][64] each (sH1, sW2, sX: bsw layout)
  __shared__ float sA[64][kLdM], sB[64][kLdM];
  __shared__ float sDo[kRows];
  const float* const sH1 = reinterpret_cast<const float*>(sH1v);
  const float* const sH2 = reinterpret_cast<const float*>(sH2v);
  const float* const sW2 = reinterpret_cast<const float*>(sW2v);
  const float* const sX = reinterpret_cast<const float*>(sXv);
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int r0 = blockIdx.x * kRows, c0 = 64 * (int)blockIdx.y;
  const float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  float o = 0.f, g = 0.f;
  if (t < kRows && r0 + t < N) {
    o = o_pre[r0 + t];
    g = r0 + t < sg.N1 ? du[r0 + t] * du_scale : sg.du2[r0 + t - sg.N1] * sg.du_scale2;
  }
  {
    typedef __attribute__((address_space(3))) void* lds_ptr;
    const int C4 = C >> 2;
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // wave w fills float4 slots [(4 w + q) 64, +64): row sl / 16, chunk sl % 16
      const int sl = (4 * w + q) * 64 + lane, row = min(r0 + (sl >> 4), N - 1), c4 = sl & 15;
      const int cs = c4 ^ (((sl >> 4) & 3) << 2);  // the bsw image's source chunk
      __builtin_amdgcn_global_load_lds((const void*)(reinterpret_cast<const float4*>(h1d) + (size_t)row * 16 + cs),
                                       (lds_ptr)(sH1v + (4 * w + q) * 64), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(reinterpret_cast<const float4*>(h2d) + (size_t)row * 16 + c4),
                                       (lds_ptr)(sH2v + (4 * w + q) * 64), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(reinterpret_cast<const float4*>(W2) + (sl >> 4) * 16 + cs),
                                       (lds_ptr)(sW2v + (4 * w + q) * 64), 16, 0, 0);
      const float4* xr = row < sg.N1 ? reinterpret_cast<const float4*>(X) + (size_t)row * C4
                                     : reinterpret_cast<const float4*>(sg.X2) + (size_t)(row - sg.N1) * C4;
      __builtin_amdgcn_global_load_lds((const void*)(xr + (c0 >> 2) + cs), (lds_ptr)(sXv + (4 * w + q) * 64), 16, 0,
                                       0);
    }
  }
  float* out = part + (size_t)blockIdx.x * mlp_partial_floats(C);
  float* gW1 = out;
  float* gb1 = gW1 + kHid * C;
  float* gW2 = gb1 + kHid;
  float* gb2 = gW2 + kHid * kHid;
  float* gW3 = gb2 + kHid;
  float* gb3 = gW3 + kHid;
  if (t < kRows) {
    float d = 0.f;
    if (r0 + t < N) {
      const float z = expf(o);
      d = o > 20.f ? g : g * z / (z + 1.f);  // softplus backward
    }
    sDo[t] = d;
  }
  __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA has landed (the barrier covers the others)
  __syncthreads();
  const bool head = blockIdx.y == 0;  // writes the non-dW1 gradients
  if (head && t < kHid) {
    float s = 0.f;
    for (int r = 0; r < kRows; ++r) s = fmaf(sDo[r], sH2[r * 64 + t], s);
    gW3[t] = s;
  } else if (head && t == kHid) {
    float s = 0.f;
    for (int r = 0; r < kRows; ++r) s += sDo[r];
    gb3[0] = s;
  }
  // dA2 = do W3 through ReLU / dropout: sA[r][o], and transposed sB[o][r]
  for (int e = t; e < 64 * 64; e += 256) {
    const int r = e >> 6, c = e & 63;
    const float v = sH2[r * 64 + c] > 0.f ? sDo[r] * W3[c] * scale : 0.f;
    sA[r][c] = v;
    sB[c][r] = v;
  }
  __syncthreads();
  const int orow = 16 * w + 4 * (lane >> 4), ocol = lane & 15;  // this lane's rows orow + i, columns 16 j + ocol
  if (head) {  // dW2[o][i] = sum_r dA2[r][o] h1[r][i]
    f32x4 acc[4];
    tile_mac_mfma(sB, sH1, w, lane, acc);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) gW2[(orow + i) * kHid + 16 * j + ocol] = acc[j][i];
  }
  if (head && t < kHid) {
    float s = 0.f;
    for (int r = 0; r < kRows; ++r) s += sA[r][t];
    gb2[t] = s;
  }
  // dA1[r][i] = sum_o dA2[r][o] W2[o][i] through ReLU / dropout, into sB as [i][r]
  f32x4 acc1[4];
  tile_mac_mfma(sA, sW2, w, lane, acc1);
  __syncthreads();  // (every wave is done reading sB as dA2 transposed)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = orow + i, c = 16 * j + ocol;
      sB[c][r] = sH1[bsw(r, c)] > 0.f ? acc1[j][i] * scale : 0.f;
    }
  __syncthreads();
  if (head && t < kHid) {
    float s = 0.f;
    for (int r = 0; r < kRows; ++r) s += sB[t][r];
    gb1[t] = s;
  }
  // this workgroup's 64-column chunk of dW1[o][c] = sum_r dA1[r][o] X[r][c]
  f32x4 acc[4];
  tile_mac_mfma(sB, sX, w, lane, acc);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) gW1[(size_t)(orow + i) * C + c0 + 16 * j + ocol] = acc[j][i];
}

// two-stage fixed-order sum over the row blocks' partials: grid.y segments of
// kSeg blocks each write a segment sum (stage 1), then stage 2 adds the
// segments in order
constexpr int kSeg = 16;
// (acc: the final sums are added to what `seg` / `grad` holds -- a second
// backward accumulating into the first one's gradient, as autograd does)
__global__ __launch_bounds__(256) void k_mlp_reduce_seg(int nblocks, int total, const float* __restrict__ part,
                                                        float* __restrict__ seg, int acc, int seglen) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  const int b0 = blockIdx.y * seglen, b1 = min(nblocks, b0 + seglen);
  float s = 0.f;
#pragma unroll 8
  for (int b = b0; b < b1; ++b) s += part[(size_t)b * total + e];  // (unrolled: the loads in flight together)
  float* d = &seg[(size_t)blockIdx.y * total + e];
  *d = acc ? *d + s : s;
}

__global__ __launch_bounds__(256) void k_mlp_reduce(int nseg, int total, const float* __restrict__ seg,
                                                    float* __restrict__ grad, int acc) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  float s = 0.f;
  for (int b = 0; b < nseg; ++b) s += seg[(size_t)b * total + e];
  grad[e] = acc ? grad[e] + s : s;
}

}  // namespace
}  // namespace wgsr

using namespace wgsr;

#define MLPCHK(name)                                                                         \
  do {                                                                                       \
    const hipError_t _e = hipGetLastError();                                                 \
    if (_e != hipSuccess) return set_error(WGSR_EHIP, "%s: %s", name, hipGetErrorString(_e)); \
  } while (0)

// Sampling keys of the DINO term's feature draw (wgsr.h wgsr_random_keys):
// 31-bit hashes of (seed, index); the ascending order of the keys is the
// random permutation.
__global__ __launch_bounds__(256) void k_random_keys(int64_t n, uint32_t seed, const uint32_t* __restrict__ seed_dev,
                                                     int32_t* __restrict__ keys) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t sd = seed_dev ? *seed_dev : seed;
  keys[i] = (int32_t)(mix32(sd ^ mix32((uint32_t)i * 0x9E3779B9U + 0x632BE5ABU)) >> 1);
}

// The first k entries of wgsr_random_perm's permutation -- the stable
// ascending order of k_random_keys' keys -- in one workgroup, without sorting
// all n: each index's 44-bit composite (key << 13 | index; unique, and
// ascending composites are the stable key order) stays in registers; one
// 2048-bucket histogram of the top 11 bits (LDS atomics, a block scan) finds
// the bucket holding the k-th smallest; the composites of the buckets below
// it are taken, the few in that bucket ranked among themselves, and the k
// taken composites placed by counting the smaller ones.
constexpr int kPpThreads = 1024, kPpItems = 8, kPpMaxN = kPpThreads * kPpItems, kPpMaxK = kPpThreads;
static_assert(kPpMaxN <= 8192, "13 index bits");
__global__ __launch_bounds__(kPpThreads) void k_perm_prefix(int n, int k, uint32_t seed,
                                                            const uint32_t* __restrict__ seed_dev,
                                                            int32_t* __restrict__ perm) {
  __shared__ uint32_t hist[2048];
  __shared__ uint32_t wsum[kPpThreads / 64];
  __shared__ uint32_t sel[2];
  __shared__ unsigned long long list[kPpMaxK];
  __shared__ unsigned long long bk[kPpMaxN];  // the k-th's bucket (a few entries for hash keys)
  __shared__ uint32_t cnt, nbk;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const uint32_t sd = seed_dev ? *seed_dev : seed;
  unsigned long long c[kPpItems];
#pragma unroll
  for (int j = 0; j < kPpItems; ++j) {
    const int i = t + kPpThreads * j;
    const uint32_t key = mix32(sd ^ mix32((uint32_t)i * 0x9E3779B9U + 0x632BE5ABU)) >> 1;  // k_random_keys
    c[j] = i < n ? ((unsigned long long)key << 13) | (unsigned long long)i : ~0ull;
  }
  hist[t] = 0u;
  hist[t + kPpThreads] = 0u;
  if (t == 0) {
    cnt = 0u;
    nbk = 0u;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kPpItems; ++j)
    if (c[j] != ~0ull) atomicAdd(&hist[(uint32_t)(c[j] >> 33)], 1u);
  __syncthreads();
  {
    const uint32_t h0 = hist[2 * t], h1 = hist[2 * t + 1], sm = h0 + h1;
    const uint32_t inc = wave_incl_scan(sm);
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t base = 0;
#pragma unroll
    for (int q = 0; q < kPpThreads / 64; ++q) base += q < w ? wsum[q] : 0u;
    const uint32_t e0 = base + inc - sm, e1 = e0 + h0, want = (uint32_t)k;
    if (e0 < want && want <= e0 + h0) {
      sel[0] = 2u * t;
      sel[1] = want - e0;
    } else if (e1 < want && want <= e1 + h1) {
      sel[0] = 2u * t + 1u;
      sel[1] = want - e1;
    }
  }
  __syncthreads();
  const uint32_t bsel = sel[0], want = sel[1];  // the bucket, and how many of it are taken
#pragma unroll
  for (int j = 0; j < kPpItems; ++j) {
    if (c[j] == ~0ull) continue;
    const uint32_t bj = (uint32_t)(c[j] >> 33);
    if (bj < bsel) list[atomicAdd(&cnt, 1u)] = c[j];
    else if (bj == bsel) bk[atomicAdd(&nbk, 1u)] = c[j];
  }
  __syncthreads();
  const uint32_t nb = nbk;
  for (uint32_t q = (uint32_t)t; q < nb; q += kPpThreads) {
    const unsigned long long v = bk[q];
    uint32_t r = 0;
    for (uint32_t u = 0; u < nb; ++u) r += bk[u] < v ? 1u : 0u;
    if (r < want) list[atomicAdd(&cnt, 1u)] = v;
  }
  __syncthreads();
  if (t < k) {  // exactly k taken
    const unsigned long long v = list[t];
    uint32_t r = 0;
    for (int q = 0; q < k; ++q) r += list[q] < v ? 1u : 0u;
    perm[r] = (int32_t)(v & 8191ull);
  }
}

extern "C" {

int64_t wgsr_random_perm_prefix_max_n(void) { return kPpMaxN; }
int64_t wgsr_random_perm_prefix_max_k(void) { return kPpMaxK; }

int wgsr_random_perm_prefix(int64_t n, int64_t k, uint32_t seed, const uint32_t* seed_dev, int32_t* perm,
                            void* stream) {
  if (n < 0 || n > kPpMaxN || k < 0 || k > n || k > kPpMaxK || (k > 0 && !perm))
    return set_error(WGSR_EINVAL, "wgsr_random_perm_prefix: 0 <= k <= min(n, %d), n <= %d", kPpMaxK, kPpMaxN);
  if (k == 0) return WGSR_OK;
  hipLaunchKernelGGL(k_perm_prefix, dim3(1), dim3(kPpThreads), 0, (hipStream_t)stream, (int)n, (int)k, seed, seed_dev,
                     perm);
  MLPCHK("wgsr_random_perm_prefix");
  return WGSR_OK;
}

size_t wgsr_mlp_scratch_bytes(int N, int C) {
  if (N <= 0 || C <= 0) return 0;
  const size_t nb = (N + kRows - 1) / kRows, nseg = (nb + kSeg - 1) / kSeg;
  return sizeof(float) * (nb + nseg) * (size_t)mlp_partial_floats(C);  // partials + segment sums
}

int wgsr_mlp_grad_floats(int C) { return C > 0 ? mlp_partial_floats(C) : 0; }

static bool mlp_small_ok(int N, int C, const float* X, const float* W1, const float* W2) {
  static const bool small_off = [] {
    const char* e = getenv("WGSR_MLP_SMALL");
    return e && atoi(e) == 0;
  }();
  return !small_off && (N + 63) / 64 < 1024 && (C == 64 || C == 128 || C == 256 || C == 384) &&
         ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W1) | reinterpret_cast<uintptr_t>(W2)) & 15) == 0;
}

static void launch_mlp_fwd_small(int N, int C, const float* X, const float* W1, const float* b1, const float* W2,
                                 const float* b2, const float* W3, const float* b3, float dropout_p, uint32_t seed,
                                 const uint32_t* seed_dev, float* h1d, float* h2d, float* o_pre, float* u,
                                 const MlpSeg2& sg, void* stream) {
  auto kern = C == 384 ? k_mlp_fwd_small<384> : C == 256 ? k_mlp_fwd_small<256>
            : C == 128 ? k_mlp_fwd_small<128> : k_mlp_fwd_small<64>;
  hipLaunchKernelGGL(kern, dim3((N + kSmallRows - 1) / kSmallRows), dim3(256), mlp_small_lds(C), (hipStream_t)stream,
                     N, X, W1, b1, W2, b2, W3, b3, dropout_p, seed, seed_dev, h1d, h2d, o_pre, u, sg);
}

static int mlp_forward_impl(int N, int C, const float* X, const float* W1, const float* b1, const float* W2,
                            const float* b2, const float* W3, const float* b3, float dropout_p, uint32_t seed,
                            const uint32_t* seed_dev, float* h1d, float* h2d, float* o_pre, float* u, void* stream) {
  if (N < 0 || C <= 0 || C % 64 != 0) return set_error(WGSR_EINVAL, "wgsr_mlp_forward: C must be a positive multiple of 64");
  if (!(dropout_p >= 0.f && dropout_p < 1.f)) return set_error(WGSR_EINVAL, "wgsr_mlp_forward: dropout_p in [0, 1)");
  if (N == 0) return WGSR_OK;
  if (!X || !W1 || !b1 || !W2 || !b2 || !W3 || !b3 || !h1d || !h2d || !o_pre || !u)
    return set_error(WGSR_EINVAL, "wgsr_mlp_forward: null pointer");
  if (mlp_small_ok(N, C, X, W1, W2)) {
    launch_mlp_fwd_small(N, C, X, W1, b1, W2, b2, W3, b3, dropout_p, seed, seed_dev, h1d, h2d, o_pre, u,
                         MlpSeg2{N, nullptr, 0u, nullptr}, stream);
  } else if ((N + 63) / 64 >= 1024)  // enough 64-row workgroups to fill the chip
    hipLaunchKernelGGL(k_mlp_fwd<64>, dim3((N + 63) / 64), dim3(256), 0, (hipStream_t)stream, N, C, X, W1, b1, W2,
                       b2, W3, b3, dropout_p, seed, seed_dev, h1d, h2d, o_pre, u);
  else
    hipLaunchKernelGGL(k_mlp_fwd<16>, dim3((N + 15) / 16), dim3(256), 0, (hipStream_t)stream, N, C, X, W1, b1, W2,
                       b2, W3, b3, dropout_p, seed, seed_dev, h1d, h2d, o_pre, u);
  MLPCHK("wgsr_mlp_forward");
  return WGSR_OK;
}

int wgsr_mlp_forward(int N, int C, const float* X, const float* W1, const float* b1, const float* W2,
                     const float* b2, const float* W3, const float* b3, float dropout_p, uint32_t seed, float* h1d,
                     float* h2d, float* o_pre, float* u, void* stream) {
  return mlp_forward_impl(N, C, X, W1, b1, W2, b2, W3, b3, dropout_p, seed, nullptr, h1d, h2d, o_pre, u, stream);
}

int wgsr_mlp_forward_dev_seed(int N, int C, const float* X, const float* W1, const float* b1, const float* W2,
                              const float* b2, const float* W3, const float* b3, float dropout_p,
                              const uint32_t* seed, float* h1d, float* h2d, float* o_pre, float* u, void* stream) {
  if (!seed) return set_error(WGSR_EINVAL, "wgsr_mlp_forward_dev_seed: null seed");
  return mlp_forward_impl(N, C, X, W1, b1, W2, b2, W3, b3, dropout_p, 0u, seed, h1d, h2d, o_pre, u, stream);
}

int64_t wgsr_random_perm_max(void) { return (int64_t)argsort_small_max(); }

int wgsr_random_perm(int64_t n, uint32_t seed, const uint32_t* seed_dev, uint32_t* keys, int32_t* perm,
                     void* stream) {
  if (n < 0 || n > (int64_t)argsort_small_max() || (n > 0 && (!keys || !perm)))
    return set_error(WGSR_EINVAL, "wgsr_random_perm: 0 <= n <= %u and buffers required", argsort_small_max());
  if (n == 0) return WGSR_OK;
  hipLaunchKernelGGL(k_random_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n, seed,
                     seed_dev, reinterpret_cast<int32_t*>(keys));
  const hipError_t e = launch_argsort_small(keys, (uint32_t)n, reinterpret_cast<uint32_t*>(perm), (hipStream_t)stream);
  if (e != hipSuccess) return set_error(WGSR_EHIP, "wgsr_random_perm: %s", hipGetErrorString(e));
  MLPCHK("wgsr_random_perm");
  return WGSR_OK;
}

int wgsr_random_keys(int64_t n, uint32_t seed, const uint32_t* seed_dev, int32_t* keys, void* stream) {
  if (n < 0 || (n > 0 && !keys)) return set_error(WGSR_EINVAL, "wgsr_random_keys: bad arguments");
  if (n == 0) return WGSR_OK;
  hipLaunchKernelGGL(k_random_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n, seed,
                     seed_dev, keys);
  MLPCHK("wgsr_random_keys");
  return WGSR_OK;
}

static int mlp_backward_impl(int N, int C, const float* X, const float* W2, const float* W3, float dropout_p,
                             const float* h1d, const float* h2d, const float* o_pre, const float* dL_du,
                             float du_scale, int accumulate, float* scratch, float* grad, void* stream,
                             const MlpBwdSeg2* seg2 = nullptr) {
  if (N < 0 || C <= 0 || C % 64 != 0) return set_error(WGSR_EINVAL, "wgsr_mlp_backward: C must be a positive multiple of 64");
  const int total = mlp_partial_floats(C);
  if (N == 0) {
    if (accumulate) return WGSR_OK;
    return hipMemsetAsync(grad, 0, sizeof(float) * total, (hipStream_t)stream) == hipSuccess
               ? WGSR_OK : set_error(WGSR_EHIP, "wgsr_mlp_backward: memset");
  }
  if (!X || !W2 || !W3 || !h1d || !h2d || !o_pre || !dL_du || !scratch || !grad)
    return set_error(WGSR_EINVAL, "wgsr_mlp_backward: null pointer");
  const int nb = (N + kRows - 1) / kRows;
  static const bool bwd1 = [] {
    const char* e = getenv("WGSR_MLP_BWD");
    return e && atoi(e) == 1;
  }();
  const bool aligned = ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W2) |
                         reinterpret_cast<uintptr_t>(h1d) | reinterpret_cast<uintptr_t>(h2d)) & 15) == 0;
  // (one workgroup per CU: the few-row grids of the mapper only)
  if (seg2 || (!bwd1 && aligned && (size_t)nb * (C / 64) <= 1024))  // (seg2: checked by the caller)
    hipLaunchKernelGGL(k_mlp_bwd2, dim3(nb, C / 64), dim3(256), 0, (hipStream_t)stream, N, C, X, W2, W3, dropout_p,
                       h1d, h2d, o_pre, dL_du, scratch, du_scale,
                       seg2 ? *seg2 : MlpBwdSeg2{N, nullptr, nullptr, 0.f});
  else
    hipLaunchKernelGGL(k_mlp_bwd, dim3(nb, C / 64), dim3(256), 0, (hipStream_t)stream, N, C, X, W2, W3, dropout_p,
                       h1d, h2d, o_pre, dL_du, scratch, du_scale);
  // (up to 64 row blocks -- the mapper's feature map plus the DINO sample --
  // are one segment: the second stage would be a copy)
  const int seglen = nb <= 64 ? nb : kSeg;
  const int nseg = (nb + seglen - 1) / seglen;
  // one segment (<= 16 row blocks: the mapper's feature maps): its sum is
  // the gradient -- the second stage would be a copy
  float* seg = nseg == 1 ? grad : scratch + (size_t)nb * total;
  hipLaunchKernelGGL(k_mlp_reduce_seg, dim3((total + 255) / 256, nseg), dim3(256), 0, (hipStream_t)stream, nb, total,
                     scratch, seg, nseg == 1 ? accumulate : 0, seglen);
  if (nseg > 1)
    hipLaunchKernelGGL(k_mlp_reduce, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream, nseg, total, seg,
                       grad, accumulate);
  MLPCHK("wgsr_mlp_backward");
  return WGSR_OK;
}

int wgsr_mlp_backward(int N, int C, const float* X, const float* W2, const float* W3, float dropout_p,
                      const float* h1d, const float* h2d, const float* o_pre, const float* dL_du, float* scratch,
                      float* grad, void* stream) {
  return mlp_backward_impl(N, C, X, W2, W3, dropout_p, h1d, h2d, o_pre, dL_du, 1.f, 0, scratch, grad, stream);
}

int wgsr_mlp_backward_acc(int N, int C, const float* X, const float* W2, const float* W3, float dropout_p,
                          const float* h1d, const float* h2d, const float* o_pre, const float* dL_du, float du_scale,
                          int accumulate, float* scratch, float* grad, void* stream) {
  return mlp_backward_impl(N, C, X, W2, W3, dropout_p, h1d, h2d, o_pre, dL_du, du_scale, accumulate, scratch, grad,
                           stream);
}

int wgsr_mlp_forward_seg2(int N1, int N2, int C, const float* X1, const float* X2, const float* W1, const float* b1,
                          const float* W2, const float* b2, const float* W3, const float* b3, float dropout_p,
                          const uint32_t* seed1, const uint32_t* seed2, float* h1d, float* h2d, float* o_pre,
                          float* u, void* stream) {
  if (N1 < 0 || N2 < 0 || C <= 0 || C % 64 != 0 || !seed1 || !seed2 || (N2 > 0 && !X2))
    return set_error(WGSR_EINVAL, "wgsr_mlp_forward_seg2: bad arguments");
  const int N = N1 + N2;
  if (N1 > 0 && N2 > 0 && mlp_small_ok(N, C, X1, W1, W2) && (reinterpret_cast<uintptr_t>(X2) & 15) == 0 &&
      (dropout_p >= 0.f && dropout_p < 1.f) && X1 && b1 && b2 && W3 && b3 && h1d && h2d && o_pre && u) {
    launch_mlp_fwd_small(N, C, X1, W1, b1, W2, b2, W3, b3, dropout_p, 0u, seed1, h1d, h2d, o_pre, u,
                         MlpSeg2{N1, X2, 0u, seed2}, stream);
    MLPCHK("wgsr_mlp_forward_seg2");
    return WGSR_OK;
  }
  // (otherwise one launch per segment, outputs at the second one's offset)
  int rc = mlp_forward_impl(N1, C, X1, W1, b1, W2, b2, W3, b3, dropout_p, 0u, seed1, h1d, h2d, o_pre, u, stream);
  if (rc != WGSR_OK || N2 == 0) return rc;
  return mlp_forward_impl(N2, C, X2, W1, b1, W2, b2, W3, b3, dropout_p, 0u, seed2, h1d + (size_t)N1 * kHid,
                          h2d + (size_t)N1 * kHid, o_pre + N1, u + N1, stream);
}

int wgsr_mlp_backward_seg2(int N1, int N2, int C, const float* X1, const float* X2, const float* W2, const float* W3,
                           float dropout_p, const float* h1d, const float* h2d, const float* o_pre, const float* du1,
                           const float* du2, float du_scale1, float du_scale2, int accumulate, float* scratch,
                           float* grad, void* stream) {
  if (N1 < 0 || N2 < 0 || C <= 0 || C % 64 != 0 || (N2 > 0 && (!X2 || !du2)))
    return set_error(WGSR_EINVAL, "wgsr_mlp_backward_seg2: bad arguments");
  const int N = N1 + N2, nb = (N + kRows - 1) / kRows;
  const bool aligned = ((reinterpret_cast<uintptr_t>(X1) | reinterpret_cast<uintptr_t>(X2) |
                         reinterpret_cast<uintptr_t>(W2) | reinterpret_cast<uintptr_t>(h1d) |
                         reinterpret_cast<uintptr_t>(h2d)) & 15) == 0;
  static const bool bwd1 = [] {
    const char* e = getenv("WGSR_MLP_BWD");
    return e && atoi(e) == 1;
  }();
  if (N1 > 0 && N2 > 0 && aligned && !bwd1 && (size_t)nb * (C / 64) <= 1024) {
    const MlpBwdSeg2 sg{N1, X2, du2, du_scale2};
    return mlp_backward_impl(N, C, X1, W2, W3, dropout_p, h1d, h2d, o_pre, du1, du_scale1, accumulate, scratch, grad,
                             stream, &sg);
  }
  int rc = mlp_backward_impl(N1, C, X1, W2, W3, dropout_p, h1d, h2d, o_pre, du1, du_scale1, accumulate, scratch, grad,
                             stream);
  if (rc != WGSR_OK || N2 == 0) return rc;
  return mlp_backward_impl(N2, C, X2, W2, W3, dropout_p, h1d + (size_t)N1 * kHid, h2d + (size_t)N1 * kHid,
                           o_pre + N1, du2, du_scale2, 1, scratch, grad, stream);
}

}  // extern "C"
