// The uncertainty-aware mapping loss around the rasteriser, gfx950 (SURVEY.md
// 8(f) row f2: get_loss_mapping_uncertainty, src/utils/slam_utils.py:146-258,
// and compute_mapping_loss_components, src/utils/dyn_uncertainty/
// mapping_utils.py:206-323 -- the reference's DEFAULT mapping loss,
// uncertainty_params.activate: True, configs/wildgs_slam.yaml:64-77).
//
// The reference runs ~60 torch kernels per iteration here (exposure, masks,
// L1 maps, a full-image median, four F.interpolate resamples, the SSIM
// components, a 5x5 MedianPool2d through unfold, the weight map and the
// index_put re-weighting of the depth L1).  Only two full-resolution passes
// are needed:
//
//   unc_fwd    per pixel: exposure-corrected image, the uncertainty weight
//              w = 0.5 / r^2 (r = bilinear upsample of the detached, clipped
//              MLP output, annealed by data_rate; w < 0.1 -> 0) evaluated on
//              the fly from the small map, and per-block partial sums of
//              w * rgb L1, w (the SSIM term's weight) and the re-weighted
//              depth L1.
//   unc_small  per pixel of the small (feature-resolution) map: the four
//              downsamples the uncertainty loss needs (bilinear: opacity and
//              the clipped SSIM-component loss; bicubic: clipped depth L1 and
//              the reference depth), sampled straight from the full-resolution
//              inputs -- nothing full-resolution is materialised.
//   unc_loss   per small pixel: reflect-padded 5x5 median of the SSIM loss,
//              the uncertainty loss, its per-block sums and its gradient with
//              respect to the MLP output (fed back into the torch MLP).
//   unc_bwd    per pixel: dL/dimage (rgb L1 + the scaled SSIM gradient) and
//              dL/ddepth with the same weights, exposure-gradient partials.
//
// Floating-point expressions keep the reference's evaluation order with FMA
// contraction off (torch eager rounds every elementwise op).
#include "wgsr_common.h"
#include "wgsr_internal.h"

#pragma clang fp contract(off)

namespace wgsr {

namespace {

constexpr int kUBlock = 256;

__device__ __forceinline__ float ublock_sum(float v, float* sred) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) sred[w] = v;
  __syncthreads();
  float r = 0.f;
  if (threadIdx.x == 0)
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) r += sred[k];
  __syncthreads();
  return r;  // valid in thread 0
}

__device__ __forceinline__ float usgn(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

// F.interpolate(mode="bilinear", align_corners=False) source coordinate
// (ATen area_pixel_compute_source_index, non-cubic: clamped at 0)
__device__ __forceinline__ void lin_src(float scale, int dst, int in, int& i0, int& i1, float& l1) {
  float s = scale * ((float)dst + 0.5f) - 0.5f;
  s = s < 0.f ? 0.f : s;
  i0 = (int)s;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = s - (float)i0;
}

// bilinear sample of an [in_h, in_w] map at output pixel (oy, ox) of [out_h, out_w]
// (ATen upsample_bilinear2d_out_frame's expression)
template <class F>
__device__ __forceinline__ float bilinear_at(F&& at, int in_h, int in_w, int out_h, int out_w, int oy, int ox) {
  const float sh = (float)in_h / (float)out_h, sw = (float)in_w / (float)out_w;
  int y0, y1, x0, x1;
  float ly, lx;
  lin_src(sh, oy, in_h, y0, y1, ly);
  lin_src(sw, ox, in_w, x0, x1, lx);
  const float hy = 1.f - ly, hx = 1.f - lx;
  return hy * (hx * at(y0, x0) + lx * at(y0, x1)) + ly * (hx * at(y1, x0) + lx * at(y1, x1));
}

// bicubic (A = -0.75, indices clamped), ATen upsample_bicubic2d
__device__ __forceinline__ float cc1(float x) {
  const float A = -0.75f;
  return ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f;
}
__device__ __forceinline__ float cc2(float x) {
  const float A = -0.75f;
  return ((A * x - 5.f * A) * x + 8.f * A) * x - 4.f * A;
}
__device__ __forceinline__ float cubic1d(float x0, float x1, float x2, float x3, float t) {
  const float c0 = cc2(t + 1.f), c1 = cc1(t), c2 = cc1(1.f - t), c3 = cc2((1.f - t) + 1.f);
  return x0 * c0 + x1 * c1 + x2 * c2 + x3 * c3;
}
template <class F>
__device__ __forceinline__ float bicubic_at(F&& at, int in_h, int in_w, int out_h, int out_w, int oy, int ox) {
  const float sh = (float)in_h / (float)out_h, sw = (float)in_w / (float)out_w;
  const float ry = sh * ((float)oy + 0.5f) - 0.5f, rx = sw * ((float)ox + 0.5f) - 0.5f;
  // ATen guard_index_and_lambda
  const int iy = min((int)floorf(ry), in_h - 1), ix = min((int)floorf(rx), in_w - 1);
  const float ty = fminf(fmaxf(ry - (float)iy, 0.f), 1.f), tx = fminf(fmaxf(rx - (float)ix, 0.f), 1.f);
  float c[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int y = min(max(iy - 1 + k, 0), in_h - 1);
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = at(y, min(max(ix - 1 + j, 0), in_w - 1));
    c[k] = cubic1d(v[0], v[1], v[2], v[3], tx);
  }
  return cubic1d(c[0], c[1], c[2], c[3], ty);
}

struct UParams {
  int H, W, h, w;
  float rgb_th, data_rate, ssim_weight, opacity_th, depth_mult;
  int init;
  int pre;  // pre_exposed: the correction is applied twice (mapper.py:1127 + slam_utils.py:179-181)
};

__device__ __forceinline__ UParams uparams(const wgsr_uncer_params& p) {
  return UParams{p.H, p.W, p.h, p.w, p.rgb_threshold, p.data_rate, p.ssim_weight, p.opacity_th,
                 p.uncer_depth_mult, p.initialization,
                 p.initialization ? 0 : p.pre_exposed};
}

// processed_uncertainty = clip(u, min=0.1) + 1e-3 (mapping_utils.py:262)
__device__ __forceinline__ float processed(float u) { return fmaxf(u, 0.1f) + 1e-3f; }

// the per-pixel weight of slam_utils.py:231-234 at full-resolution pixel (y, x)
__device__ __forceinline__ float weight_at(const UParams& q, const float* __restrict__ unc, int y, int x) {
  float r = bilinear_at([&](int yy, int xx) { return processed(unc[yy * q.w + xx]); }, q.h, q.w, q.H, q.W, y, x);
  r = (r - 0.1f) * q.data_rate + 0.1f;  // mapping_utils.py:268
  const float wgt = (1.f / (r * r)) * 0.5f;  // torch's 0.5 / t is t.reciprocal() * 0.5
  return wgt < 0.1f ? 0.f : wgt;
}

// depth_threshold = min(10 * median(ref_depth), 50) (mapping_utils.py:252)
__device__ __forceinline__ float depth_threshold(const float* __restrict__ med) { return fminf(10.f * med[0], 50.f); }

__global__ __launch_bounds__(kUBlock) void k_unc_fwd(wgsr_uncer_params prm, const float* __restrict__ image,
                                                     const float* __restrict__ gt, const float* __restrict__ depth,
                                                     const float* __restrict__ ref, const float* __restrict__ expo_a,
                                                     const float* __restrict__ expo_b, const float* __restrict__ unc,
                                                     const float* __restrict__ med, float* __restrict__ image_ab,
                                                     float* __restrict__ part) {
  __shared__ float sred[kUBlock / 64];
  const UParams q = uparams(prm);
  const int HW = q.H * q.W;
  const int p = blockIdx.x * kUBlock + threadIdx.x;
  const float ea = q.init ? 1.f : expf(expo_a[0]), b = q.init ? 0.f : expo_b[0];
  float swl1 = 0.f, sw = 0.f, sd = 0.f;
  if (p < HW) {
    const int y = p / q.W, x = p - y * q.W;
    const float wgt = weight_at(q, unc, y, x);
    const float g0 = gt[p], g1 = gt[HW + p], g2 = gt[2 * HW + p];
    const float m = ((g0 + g1) + g2) > q.rgb_th ? 1.f : 0.f;
    float a0 = image[p], a1 = image[HW + p], a2 = image[2 * HW + p];
    if (q.pre) {  // the mapper's own torch.exp(a) * image + b, in its op order
      a0 = __fadd_rn(__fmul_rn(ea, a0), b);
      a1 = __fadd_rn(__fmul_rn(ea, a1), b);
      a2 = __fadd_rn(__fmul_rn(ea, a2), b);
    }
    if (!q.init) {
      a0 = ea * a0 + b;
      a1 = ea * a1 + b;
      a2 = ea * a2 + b;
    }
    image_ab[p] = a0;
    image_ab[HW + p] = a1;
    image_ab[2 * HW + p] = a2;
    // rgb_loss = w * ((1 - l) l1 + l ssim_loss): sum_c w l1_c and sum w (x3 channels)
    swl1 = wgt * fabsf(a0 * m - g0 * m) + wgt * fabsf(a1 * m - g1 * m) + wgt * fabsf(a2 * m - g2 * m);
    sw = wgt;
    const float rd = ref[p], d = depth[p];
    const float thr = depth_threshold(med);
    const float dm = (rd > 0.01f && rd < thr) ? 1.f : 0.f;
    float l1d = fabsf(d * dm - rd * dm);
    if (rd < d + 1.f) l1d = wgt * l1d;  // slam_utils.py:244-245
    sd = l1d;
  }
  const float s0 = ublock_sum(swl1, sred);
  const float s1 = ublock_sum(sw, sred);
  const float s2 = ublock_sum(sd, sred);
  if (threadIdx.x == 0) {
    part[3 * blockIdx.x] = s0;
    part[3 * blockIdx.x + 1] = s1;
    part[3 * blockIdx.x + 2] = s2;
  }
}

__global__ __launch_bounds__(kUBlock) void k_unc_small(wgsr_uncer_params prm, const float* __restrict__ opac,
                                                       const float* __restrict__ depth, const float* __restrict__ ref,
                                                       const float* __restrict__ med, const float* __restrict__ lum,
                                                       const float* __restrict__ con, const float* __restrict__ str,
                                                       float* __restrict__ s_ssim, float* __restrict__ s_dl,
                                                       float* __restrict__ s_op) {
  const UParams q = uparams(prm);
  const int i = blockIdx.x * kUBlock + threadIdx.x;
  if (i >= q.h * q.w) return;
  const int oy = i / q.w, ox = i - oy * q.w;
  const int W = q.W;
  const float thr = depth_threshold(med);
  // small_opacity (mapping_utils.py:272)
  s_op[i] = bilinear_at([&](int y, int x) { return opac[y * W + x]; }, q.H, q.W, q.h, q.w, oy, ox);
  // ssim_loss = clip(opacity * ssim_weight * (1 - l)(1 - s)(1 - c), max 5) (:279-287), then bilinear (:290)
  s_ssim[i] = bilinear_at(
      [&](int y, int x) {
        const int p = y * W + x;
        const float v = opac[p] * q.ssim_weight * (1.f - lum[p]) * (1.f - str[p]) * (1.f - con[p]);
        return fminf(v, 5.f);
      },
      q.H, q.W, q.h, q.w, oy, ox);
  // small_depth_loss: bicubic of clip(depth L1, max 5) (:296-300), zero where the
  // bicubic reference depth exceeds the threshold (:301-305)
  float dl = bicubic_at(
      [&](int y, int x) {
        const int p = y * W + x;
        const float rd = ref[p];
        const float dm = (rd > 0.01f && rd < thr) ? 1.f : 0.f;
        return fminf(fabsf(depth[p] * dm - rd * dm), 5.f);
      },
      q.H, q.W, q.h, q.w, oy, ox);
  const float sd = bicubic_at([&](int y, int x) { return ref[y * W + x]; }, q.H, q.W, q.h, q.w, oy, ox);
  if (sd > thr) dl = 0.f;
  s_dl[i] = dl;
}

// torch.median of 25 values: the lower median (13th smallest) -- for 25
// values the median itself.  A 99-comparator selection network (min / max
// pairs, ~200 VALU instead of the 625 compares of counting ranks); checked
// on all 2^25 zero-one inputs (the zero-one principle then covers every
// input).
__device__ __forceinline__ float median25(const float (&v)[25]) {
  constexpr int kNet[99][2] = {
    {0, 1}, {3, 4}, {2, 4}, {2, 3}, {6, 7}, {5, 7}, {5, 6}, {9, 10},
    {8, 10}, {8, 9}, {12, 13}, {11, 13}, {11, 12}, {15, 16}, {14, 16}, {14, 15},
    {18, 19}, {17, 19}, {17, 18}, {21, 22}, {20, 22}, {20, 21}, {23, 24}, {2, 5},
    {3, 6}, {0, 6}, {0, 3}, {4, 7}, {1, 7}, {1, 4}, {11, 14}, {8, 14},
    {8, 11}, {12, 15}, {9, 15}, {9, 12}, {13, 16}, {10, 16}, {10, 13}, {20, 23},
    {17, 23}, {17, 20}, {21, 24}, {18, 24}, {18, 21}, {19, 22}, {8, 17}, {9, 18},
    {0, 18}, {0, 9}, {10, 19}, {1, 19}, {1, 10}, {11, 20}, {2, 20}, {2, 11},
    {12, 21}, {3, 21}, {3, 12}, {13, 22}, {4, 22}, {4, 13}, {14, 23}, {5, 23},
    {5, 14}, {15, 24}, {6, 24}, {6, 15}, {7, 16}, {7, 19}, {13, 21}, {15, 23},
    {7, 13}, {7, 15}, {1, 9}, {3, 11}, {5, 17}, {11, 17}, {9, 17}, {4, 10},
    {6, 12}, {7, 14}, {4, 6}, {4, 7}, {12, 14}, {10, 14}, {6, 7}, {10, 12},
    {6, 10}, {6, 17}, {12, 17}, {7, 17}, {7, 10}, {12, 18}, {7, 12}, {10, 18},
    {12, 20}, {10, 20}, {10, 12}};
  float p[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) p[i] = v[i];
#pragma unroll
  for (int k = 0; k < 99; ++k) {
    const float a = p[kNet[k][0]], b = p[kNet[k][1]];
    p[kNet[k][0]] = fminf(a, b);
    p[kNet[k][1]] = fmaxf(a, b);
  }
  return p[12];
}

__device__ __forceinline__ int reflect(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * (n - 1) - i : i;
}

__global__ __launch_bounds__(kUBlock) void k_unc_loss(wgsr_uncer_params prm, const float* __restrict__ unc,
                                                      const float* __restrict__ s_ssim, const float* __restrict__ s_dl,
                                                      const float* __restrict__ s_op, float grad_scale,
                                                      float* __restrict__ loss_map, float* __restrict__ part,
                                                      float* __restrict__ d_unc) {
  __shared__ float sred[kUBlock / 64];
  const UParams q = uparams(prm);
  const int i = blockIdx.x * kUBlock + threadIdx.x;
  float L = 0.f;
  if (i < q.h * q.w) {
    const int oy = i / q.w, ox = i - oy * q.w;
    // MedianPool2d(5, stride 1, same=True): reflect padding 2 on every side
    float v[25];
#pragma unroll
    for (int dy = 0; dy < 5; ++dy)
#pragma unroll
      for (int dx = 0; dx < 5; ++dx)
        v[dy * 5 + dx] = s_ssim[reflect(oy + dy - 2, q.h) * q.w + reflect(ox + dx - 2, q.w)];
    const float f = median25(v);
    const float u = unc[i];
    const float pu = processed(u);
    const float pu2 = pu * pu;
    const float dl = s_dl[i];
    L = f / pu2 + 0.5f * logf(pu) + q.depth_mult * dl / pu2;  // mapping_utils.py:308-313
    const bool keep = !(s_op[i] < q.opacity_th);                // :314-316
    L = keep ? L : 0.f;
    if (loss_map) loss_map[i] = L;
    if (d_unc) {
      // d/dpu of f pu^-2 + 0.5 log pu + k dl pu^-2, through clip(min 0.1)
      const float pu3 = pu2 * pu;
      const float g = -2.f * f / pu3 + 0.5f / pu - 2.f * q.depth_mult * dl / pu3;
      d_unc[i] = (keep && u >= 0.1f) ? grad_scale * g : 0.f;
    }
  }
  const float s = ublock_sum(L, sred);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(kUBlock) void k_unc_bwd(wgsr_uncer_params prm, const float* __restrict__ image,
                                                     const float* __restrict__ image_ab, const float* __restrict__ gt,
                                                     const float* __restrict__ depth, const float* __restrict__ ref,
                                                     const float* __restrict__ expo_a,
                                                     const float* __restrict__ expo_b, const float* __restrict__ unc,
                                                     const float* __restrict__ med, float w_rgb, float w_depth,
                                                     const float* __restrict__ lgrad,
                                                     const float* __restrict__ ssim_grad, float* __restrict__ d_image,
                                                     float* __restrict__ d_depth, float* __restrict__ part) {
  __shared__ float sred[kUBlock / 64];
  const UParams q = uparams(prm);
  const int HW = q.H * q.W;
  const int p = blockIdx.x * kUBlock + threadIdx.x;
  const float ea = q.init ? 1.f : expf(expo_a[0]);
  const float b1 = q.pre ? expo_b[0] : 0.f;
  const float lg = lgrad ? lgrad[0] : 1.f;  // upstream dL/dloss
  w_rgb = w_rgb * lg;
  w_depth = w_depth * lg;
  float da = 0.f, db = 0.f;
  if (p < HW) {
    const int y = p / q.W, x = p - y * q.W;
    const float wgt = weight_at(q, unc, y, x);
    const float g[3] = {gt[p], gt[HW + p], gt[2 * HW + p]};
    const float m = ((g[0] + g[1]) + g[2]) > q.rgb_th ? 1.f : 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const size_t k = (size_t)c * HW + p;
      float gab = w_rgb * wgt * usgn(image_ab[k] * m - g[c] * m) * m;
      if (ssim_grad) gab += ssim_grad[k];
      if (q.pre) {
        // x2 = ea x1 + b, x1 = ea x + b:  dx2/dx = ea^2, dx2/da = ea (x1 + ea x), dx2/db = ea + 1
        const float x = image[k];
        const float x1 = __fadd_rn(__fmul_rn(ea, x), b1);
        d_image[k] = (gab * ea) * ea;
        da += gab * ea * (x1 + ea * x);
        db += gab * (ea + 1.f);
      } else {
        d_image[k] = gab * ea;
        da += gab * image[k] * ea;
        db += gab;
      }
    }
    const float rd = ref[p], d = depth[p];
    const float thr = depth_threshold(med);
    const float dm = (rd > 0.01f && rd < thr) ? 1.f : 0.f;
    const float wd = (rd < d + 1.f) ? wgt : 1.f;
    d_depth[p] = w_depth * wd * usgn(d * dm - rd * dm) * dm;
  }
  const float s0 = ublock_sum(da, sred);
  const float s1 = ublock_sum(db, sred);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s0;
    part[2 * blockIdx.x + 1] = s1;
  }
}

// One workgroup: the scalar epilogue of the loss (fixed-order partial sums,
// the loss value, the SSIM backward's per-plane scale) -- one launch instead
// of ~15 tiny torch ops per iteration.  1024 threads read the partial arrays
// in one strided pass (5 running sums each), then one fixed-order block
// reduction of all five.
constexpr int kCombine = 1024;

__global__ __launch_bounds__(kCombine) void k_unc_combine(int HW, int hw, const float* __restrict__ lpart, int nb,
                                                          const float* __restrict__ upart, int nbs,
                                                          const float* __restrict__ ssim_mean,
                                                          const float* __restrict__ extra, int nextra, float w_extra,
                                                          float alpha, float lam, float ssim_mult, int ssim_loss,
                                                          float* __restrict__ loss, float* __restrict__ sums,
                                                          float* __restrict__ ssim_scale,
                                                          const float* __restrict__ ssim_partials, int ssim_tiles,
                                                          float* __restrict__ ssim_mean_out) {
  __shared__ float sred[5][kCombine / 64];
  __shared__ double s_dred[256];
  const int t = threadIdx.x;
  // (ssim_partials: the SSIM forward's 3-plane tile partials, reduced here
  // as k_ssim_reduce would -- one launch fewer)
  float smean = 0.f;
  if (ssim_partials) smean = ssim_partials_mean(ssim_partials, 3, ssim_tiles, 1.0 / (double)HW, nullptr, s_dred);
  float v[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  for (int i = t; i < nb; i += kCombine) {
    v[0] += lpart[3 * i];
    v[1] += lpart[3 * i + 1];
    v[2] += lpart[3 * i + 2];
  }
  for (int i = t; i < nbs; i += kCombine) v[3] += upart[i];
  if (extra)
    for (int i = t; i < nextra; i += kCombine) v[4] += extra[i];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    v[k] = wave_sum(v[k]);
    if ((t & 63) == 0) sred[k][t >> 6] = v[k];
  }
  __syncthreads();
  if (t != 0) return;
  float r[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    r[k] = 0.f;
    for (int w = 0; w < kCombine / 64; ++w) r[k] += sred[k][w];
  }
  const float s0 = r[0], s1 = r[1], s2 = r[2], u = r[3], x = r[4];
  const float n3 = 3.f * (float)HW;
  if (ssim_partials && ssim_mean_out) ssim_mean_out[0] = smean;
  const float sm = ssim_partials ? smean : (ssim_loss ? ssim_mean[0] : 0.f);
  const float rgb = ssim_loss ? ((1.f - lam) * s0 + 3.f * lam * (1.f - sm) * s1) / n3 : s0 / n3;
  loss[0] = alpha * rgb + (1.f - alpha) * s2 / (float)HW + ssim_mult * (u / (float)hw) + w_extra * x;
  sums[0] = s0;
  sums[1] = s1;
  sums[2] = s2;
  // dL/dS per pixel of the SSIM map: -alpha lambda (sum w) / HW / (3 HW)
  const float sc = s1 * (-alpha * lam / ((float)HW * n3));
  ssim_scale[0] = sc;
  ssim_scale[1] = sc;
  ssim_scale[2] = sc;
}

int ublocks(int64_t n) { return n > 0 ? (int)((n + kUBlock - 1) / kUBlock) : 0; }

int check_params(const wgsr_uncer_params* p, const char* who) {
  if (!p) return set_error(WGSR_EINVAL, "%s: null params", who);
  if (p->H <= 0 || p->W <= 0 || p->h <= 2 || p->w <= 2)
    return set_error(WGSR_EINVAL, "%s: bad sizes (image %dx%d, uncertainty %dx%d; reflect padding needs > 2)", who,
                     p->H, p->W, p->h, p->w);
  if ((int64_t)p->H * p->W > (int64_t)INT32_MAX / 3) return set_error(WGSR_EINVAL, "%s: image too large", who);
  return WGSR_OK;
}

}  // namespace
}  // namespace wgsr

using namespace wgsr;

#define UNCCHK(name)                                                                         \
  do {                                                                                       \
    const hipError_t _e = hipGetLastError();                                                 \
    if (_e != hipSuccess) return set_error(WGSR_EHIP, "%s: %s", name, hipGetErrorString(_e)); \
  } while (0)

extern "C" {

int wgsr_uncer_blocks(int64_t n) { return ublocks(n); }

int wgsr_uncer_loss_forward(const wgsr_uncer_params* prm, const float* image, const float* gt_image,
                            const float* depth, const float* ref_depth, const float* exposure_a,
                            const float* exposure_b, const float* uncertainty, const float* median_depth,
                            float* image_ab, float* partials, void* stream) {
  if (int e = check_params(prm, "wgsr_uncer_loss_forward")) return e;
  if (!image || !gt_image || !depth || !ref_depth || !uncertainty || !median_depth || !image_ab || !partials ||
      (!prm->initialization && (!exposure_a || !exposure_b)))
    return set_error(WGSR_EINVAL, "wgsr_uncer_loss_forward: null pointer");
  const int HW = prm->H * prm->W;
  hipLaunchKernelGGL(k_unc_fwd, dim3(ublocks(HW)), dim3(kUBlock), 0, (hipStream_t)stream, *prm, image, gt_image,
                     depth, ref_depth, exposure_a, exposure_b, uncertainty, median_depth, image_ab, partials);
  UNCCHK("wgsr_uncer_loss_forward");
  return WGSR_OK;
}

int wgsr_uncer_small_maps(const wgsr_uncer_params* prm, const float* opacity, const float* depth,
                          const float* ref_depth, const float* median_depth, const float* luminance,
                          const float* contrast, const float* structure, float* small_ssim_loss,
                          float* small_depth_loss, float* small_opacity, void* stream) {
  if (int e = check_params(prm, "wgsr_uncer_small_maps")) return e;
  if (!opacity || !depth || !ref_depth || !median_depth || !luminance || !contrast || !structure ||
      !small_ssim_loss || !small_depth_loss || !small_opacity)
    return set_error(WGSR_EINVAL, "wgsr_uncer_small_maps: null pointer");
  const int hw = prm->h * prm->w;
  hipLaunchKernelGGL(k_unc_small, dim3(ublocks(hw)), dim3(kUBlock), 0, (hipStream_t)stream, *prm, opacity, depth,
                     ref_depth, median_depth, luminance, contrast, structure, small_ssim_loss, small_depth_loss,
                     small_opacity);
  UNCCHK("wgsr_uncer_small_maps");
  return WGSR_OK;
}

int wgsr_uncer_loss_small(const wgsr_uncer_params* prm, const float* uncertainty, const float* small_ssim_loss,
                          const float* small_depth_loss, const float* small_opacity, float grad_scale,
                          float* loss_map, float* partials, float* dL_duncertainty, void* stream) {
  if (int e = check_params(prm, "wgsr_uncer_loss_small")) return e;
  if (!uncertainty || !small_ssim_loss || !small_depth_loss || !small_opacity || !partials)
    return set_error(WGSR_EINVAL, "wgsr_uncer_loss_small: null pointer");
  const int hw = prm->h * prm->w;
  hipLaunchKernelGGL(k_unc_loss, dim3(ublocks(hw)), dim3(kUBlock), 0, (hipStream_t)stream, *prm, uncertainty,
                     small_ssim_loss, small_depth_loss, small_opacity, grad_scale, loss_map, partials,
                     dL_duncertainty);
  UNCCHK("wgsr_uncer_loss_small");
  return WGSR_OK;
}

int wgsr_uncer_loss_combine(const wgsr_uncer_params* prm, const float* partials, const float* small_partials,
                            const float* ssim_mean, const float* extra_partials, int n_extra, float extra_weight,
                            float alpha, float lambda_dssim, float ssim_mult, int ssim_loss, float* loss,
                            float* sums, float* ssim_scale, void* stream) {
  if (int e = check_params(prm, "wgsr_uncer_loss_combine")) return e;
  if (!partials || !small_partials || !loss || !sums || !ssim_scale || (ssim_loss && !ssim_mean) ||
      (n_extra > 0 && !extra_partials))
    return set_error(WGSR_EINVAL, "wgsr_uncer_loss_combine: null pointer");
  hipLaunchKernelGGL(k_unc_combine, dim3(1), dim3(kCombine), 0, (hipStream_t)stream, prm->H * prm->W,
                     prm->h * prm->w, partials, ublocks((int64_t)prm->H * prm->W), small_partials,
                     ublocks((int64_t)prm->h * prm->w), ssim_mean, n_extra > 0 ? extra_partials : nullptr, n_extra,
                     extra_weight, alpha, lambda_dssim, ssim_mult, ssim_loss, loss, sums, ssim_scale, nullptr, 0,
                     nullptr);
  UNCCHK("wgsr_uncer_loss_combine");
  return WGSR_OK;
}

int wgsr_uncer_loss_combine_ssim(const wgsr_uncer_params* prm, const float* partials, const float* small_partials,
                                 const float* ssim_partials, float* ssim_mean, const float* extra_partials,
                                 int n_extra, float extra_weight, float alpha, float lambda_dssim, float ssim_mult,
                                 float* loss, float* sums, float* ssim_scale, void* stream) {
  if (int e = check_params(prm, "wgsr_uncer_loss_combine_ssim")) return e;
  if (!partials || !small_partials || !ssim_partials || !loss || !sums || !ssim_scale ||
      (n_extra > 0 && !extra_partials))
    return set_error(WGSR_EINVAL, "wgsr_uncer_loss_combine_ssim: null pointer");
  const int tiles = wgsr_ssim_tiles(prm->H, prm->W);
  hipLaunchKernelGGL(k_unc_combine, dim3(1), dim3(kCombine), 0, (hipStream_t)stream, prm->H * prm->W,
                     prm->h * prm->w, partials, ublocks((int64_t)prm->H * prm->W), small_partials,
                     ublocks((int64_t)prm->h * prm->w), nullptr, n_extra > 0 ? extra_partials : nullptr, n_extra,
                     extra_weight, alpha, lambda_dssim, ssim_mult, 1, loss, sums, ssim_scale, ssim_partials, tiles,
                     ssim_mean);
  UNCCHK("wgsr_uncer_loss_combine_ssim");
  return WGSR_OK;
}

int wgsr_uncer_loss_backward(const wgsr_uncer_params* prm, const float* image, const float* image_ab,
                             const float* gt_image, const float* depth, const float* ref_depth,
                             const float* exposure_a, const float* exposure_b, const float* uncertainty,
                             const float* median_depth, float w_rgb, float w_depth, const float* loss_grad, const float* ssim_grad, float* dL_dimage,
                             float* dL_ddepth, float* partials, void* stream) {
  if (int e = check_params(prm, "wgsr_uncer_loss_backward")) return e;
  if (!image || !image_ab || !gt_image || !depth || !ref_depth || !uncertainty || !median_depth || !dL_dimage ||
      !dL_ddepth || !partials || (!prm->initialization && !exposure_a) ||
      (!prm->initialization && prm->pre_exposed && !exposure_b))
    return set_error(WGSR_EINVAL, "wgsr_uncer_loss_backward: null pointer");
  const int HW = prm->H * prm->W;
  hipLaunchKernelGGL(k_unc_bwd, dim3(ublocks(HW)), dim3(kUBlock), 0, (hipStream_t)stream, *prm, image, image_ab,
                     gt_image, depth, ref_depth, exposure_a, exposure_b, uncertainty, median_depth, w_rgb, w_depth,
                     loss_grad,
                     ssim_grad, dL_dimage, dL_ddepth, partials);
  UNCCHK("wgsr_uncer_loss_backward");
  return WGSR_OK;
}

}  // extern "C"
