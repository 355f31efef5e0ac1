// The mapping iteration around the rasteriser, gfx950 (SURVEY.md 8(f) rows
// f1/f2: what src/mapper.py:1083-1219 runs before and after the rasteriser
// every iteration, as few fused launches instead of ~100 small torch kernels).
//
//   activate      GaussianModel's activations (gaussian_model.py:
//                 get_opacity / get_scaling / get_rotation: sigmoid, exp,
//                 F.normalize) for one forward, plus the per-block partial
//                 sums of mapper.py's isotropic scale loss
//                 |exp(s) - mean_row(exp(s))| (mapper.py:1167-1169).
//   activate_bwd  the chain rule back to the raw parameters, with the
//                 isotropic loss gradient folded in.
//   loss fwd/bwd  get_loss_mapping_rgbd (slam_utils.py:107-143) minus its
//                 SSIM (wgsr_ssim_*): exposure correction exp(a) I + b, the
//                 boundary-masked rgb L1 and the masked depth L1 as per-block
//                 partial sums; the backward combines the L1 terms with the
//                 SSIM gradient into dL/dimage, dL/ddepth and the exposure
//                 gradients' partial sums.
//   densify_stats mapper.py:1177-1183 + add_densification_stats
//                 (gaussian_model.py:745-749) for one view: max_radii2D,
//                 sum ||dL/dmeans2D[:2]|| and the visibility count, without
//                 boolean indexing.
// Partial sums are per workgroup, reduced afterwards in a fixed order
// (deterministic).
#include "wgsr_common.h"
#include "wgsr_internal.h"

namespace wgsr {

namespace {

constexpr int kMapBlock = 256;

__device__ __forceinline__ float block_sum(float v, float* sred) {
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

__global__ __launch_bounds__(kMapBlock) void k_activate(int P, const float* __restrict__ o_raw,
                                                        const float* __restrict__ s_raw,
                                                        const float* __restrict__ r_raw, float* __restrict__ opac,
                                                        float* __restrict__ scales, float* __restrict__ rots,
                                                        float* __restrict__ iso_part) {
  __shared__ float sred[kMapBlock / 64];
  const int i = blockIdx.x * kMapBlock + threadIdx.x;
  float iso = 0.f;
  if (i < P) {
    opac[i] = 1.f / (1.f + expf(-o_raw[i]));
    const float e0 = expf(s_raw[3 * (size_t)i]), e1 = expf(s_raw[3 * (size_t)i + 1]),
                e2 = expf(s_raw[3 * (size_t)i + 2]);
    scales[3 * (size_t)i] = e0;
    scales[3 * (size_t)i + 1] = e1;
    scales[3 * (size_t)i + 2] = e2;
    const float m = (e0 + e1 + e2) / 3.f;
    iso = fabsf(e0 - m) + fabsf(e1 - m) + fabsf(e2 - m);
    const float4 q = reinterpret_cast<const float4*>(r_raw)[i];
    const float n = fmaxf(sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w), 1e-12f);
    reinterpret_cast<float4*>(rots)[i] = make_float4(q.x / n, q.y / n, q.z / n, q.w / n);
  }
  const float s = block_sum(iso, sred);
  if (threadIdx.x == 0) iso_part[blockIdx.x] = s;
}

__device__ __forceinline__ float sgn(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

// the densification statistics of k_densify_stats, fused into the
// activation backward's pass over the Gaussians (radii null: none)
struct DensifyJob {
  const int32_t* radii;
  const float* m2d_grad;
  float* max_radii;
  float* accum;
  float* denom;
  // a capacity-mode forward's overflow word (counts[3] / ImageLayout::meta[1];
  // null: none): set, the iteration left no gradient and the statistics keep
  // their values (the render backward wrote only the zero fill)
  const uint32_t* skip;
};
__device__ __forceinline__ void densify_stats_one(int i, const DensifyJob& J) {
  const int r = J.radii[i];
  if (r <= 0) return;
  J.max_radii[i] = fmaxf(J.max_radii[i], (float)r);
  const float gx = J.m2d_grad[3 * (size_t)i], gy = J.m2d_grad[3 * (size_t)i + 1];
  J.accum[i] += sqrtf(gx * gx + gy * gy);
  J.denom[i] += 1.f;
}

__global__ __launch_bounds__(kMapBlock) void k_activate_bwd(int P, const float* __restrict__ o_raw,
                                                            const float* __restrict__ s_raw,
                                                            const float* __restrict__ r_raw,
                                                            const float* __restrict__ g_op,
                                                            const float* __restrict__ g_sc,
                                                            const float* __restrict__ g_rot, float iso_w,
                                                            float* __restrict__ d_o, float* __restrict__ d_s,
                                                            float* __restrict__ d_r, const DensifyJob dj) {
  const int i = blockIdx.x * kMapBlock + threadIdx.x;
  if (i >= P) return;
  if (dj.radii && !(dj.skip && *dj.skip)) densify_stats_one(i, dj);
  // sigmoid: grad * (1 - y) * y
  const float y = 1.f / (1.f + expf(-o_raw[i]));
  d_o[i] = g_op[i] * (1.f - y) * y;
  // exp, with the isotropic term 10 * mean|e - mean_row(e)| folded in
  const size_t i3 = 3 * (size_t)i;
  const float e[3] = {expf(s_raw[i3]), expf(s_raw[i3 + 1]), expf(s_raw[i3 + 2])};
  const float m = (e[0] + e[1] + e[2]) / 3.f;
  const float sg[3] = {sgn(e[0] - m), sgn(e[1] - m), sgn(e[2] - m)};
  const float sm = (sg[0] + sg[1] + sg[2]) / 3.f;
#pragma unroll
  for (int k = 0; k < 3; ++k) d_s[i3 + k] = (g_sc[i3 + k] + iso_w * (sg[k] - sm)) * e[k];
  // F.normalize: y = x / max(|x|, eps) -> (g - y (y . g)) / |x| above eps
  const float4 q = reinterpret_cast<const float4*>(r_raw)[i];
  const float4 g = reinterpret_cast<const float4*>(g_rot)[i];
  const float nr = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  float4 d;
  if (nr > 1e-12f) {
    const float inv = 1.f / nr;
    const float4 u = make_float4(q.x * inv, q.y * inv, q.z * inv, q.w * inv);
    const float ug = u.x * g.x + u.y * g.y + u.z * g.z + u.w * g.w;
    d = make_float4((g.x - u.x * ug) * inv, (g.y - u.y * ug) * inv, (g.z - u.z * ug) * inv, (g.w - u.w * ug) * inv);
  } else {
    d = make_float4(g.x / 1e-12f, g.y / 1e-12f, g.z / 1e-12f, g.w / 1e-12f);
  }
  reinterpret_cast<float4*>(d_r)[i] = d;
}

// Forward terms per pixel p of the [3,H,W] image / [1,H,W] depth.
__global__ __launch_bounds__(kMapBlock) void k_map_loss_fwd(int HW, const float* __restrict__ image,
                                                            const float* __restrict__ gt,
                                                            const float* __restrict__ depth,
                                                            const float* __restrict__ gt_depth,
                                                            const float* __restrict__ expo_a,
                                                            const float* __restrict__ expo_b, float rgb_th,
                                                            float* __restrict__ image_ab, float* __restrict__ part) {
  __shared__ float sred[kMapBlock / 64];
  const int p = blockIdx.x * kMapBlock + threadIdx.x;
  const float ea = expf(expo_a[0]), b = expo_b[0];
  float l1 = 0.f, l1d = 0.f;
  if (p < HW) {
    const float g0 = gt[p], g1 = gt[HW + p], g2 = gt[2 * HW + p];
    const float m = ((g0 + g1) + g2) > rgb_th ? 1.f : 0.f;
    const float a0 = ea * image[p] + b, a1 = ea * image[HW + p] + b, a2 = ea * image[2 * HW + p] + b;
    image_ab[p] = a0;
    image_ab[HW + p] = a1;
    image_ab[2 * HW + p] = a2;
    l1 = fabsf(a0 * m - g0 * m) + fabsf(a1 * m - g1 * m) + fabsf(a2 * m - g2 * m);
    const float gd = gt_depth[p];
    const float dm = gd > 0.01f ? 1.f : 0.f;
    l1d = fabsf(depth[p] * dm - gd * dm);
  }
  const float s0 = block_sum(l1, sred);
  const float s1 = block_sum(l1d, sred);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s0;
    part[2 * blockIdx.x + 1] = s1;
  }
}

// dL/dimage_ab = w_rgb sign(.) m + ssim_grad (already scaled); dL/dimage =
// exp(a) dL/dimage_ab; partial sums of dL/da = sum dL/dimage_ab image exp(a)
// and dL/db = sum dL/dimage_ab; dL/ddepth = w_depth sign(.) dm.
__global__ __launch_bounds__(kMapBlock) void k_map_loss_bwd(
    int HW, const float* __restrict__ image, const float* __restrict__ image_ab, const float* __restrict__ gt,
    const float* __restrict__ depth, const float* __restrict__ gt_depth, const float* __restrict__ expo_a,
    float rgb_th, float w_rgb, float w_depth, const float* __restrict__ ssim_grad, float* __restrict__ d_image,
    float* __restrict__ d_depth, float* __restrict__ part) {
  __shared__ float sred[kMapBlock / 64];
  const int p = blockIdx.x * kMapBlock + threadIdx.x;
  const float ea = expf(expo_a[0]);
  float da = 0.f, db = 0.f;
  if (p < HW) {
    const float g[3] = {gt[p], gt[HW + p], gt[2 * HW + p]};
    const float m = ((g[0] + g[1]) + g[2]) > rgb_th ? 1.f : 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const size_t q = (size_t)c * HW + p;
      float gab = w_rgb * sgn(image_ab[q] * m - g[c] * m) * m;
      if (ssim_grad) gab += ssim_grad[q];
      d_image[q] = gab * ea;
      da += gab * image[q] * ea;
      db += gab;
    }
    const float gd = gt_depth[p];
    const float dm = gd > 0.01f ? 1.f : 0.f;
    d_depth[p] = w_depth * sgn(depth[p] * dm - gd * dm) * dm;
  }
  const float s0 = block_sum(da, sred);
  const float s1 = block_sum(db, sred);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s0;
    part[2 * blockIdx.x + 1] = s1;
  }
}

__global__ __launch_bounds__(kMapBlock) void k_densify_stats(int P, const int32_t* __restrict__ radii,
                                                             const float* __restrict__ m2d_grad,
                                                             float* __restrict__ max_radii, float* __restrict__ accum,
                                                             float* __restrict__ denom) {
  const int i = blockIdx.x * kMapBlock + threadIdx.x;
  if (i >= P) return;
  densify_stats_one(i, DensifyJob{radii, m2d_grad, max_radii, accum, denom, nullptr});
}

}  // namespace
}  // namespace wgsr

using namespace wgsr;

#define MAPCHK(name)                                                                         \
  do {                                                                                       \
    const hipError_t _e = hipGetLastError();                                                 \
    if (_e != hipSuccess) return set_error(WGSR_EHIP, "%s: %s", name, hipGetErrorString(_e)); \
  } while (0)

extern "C" {

int wgsr_map_blocks(int64_t n) { return n > 0 ? (int)((n + kMapBlock - 1) / kMapBlock) : 0; }

int wgsr_gaussian_activate(int P, const float* opacity_raw, const float* scaling_raw, const float* rotation_raw,
                           float* opacity, float* scales, float* rotations, float* iso_partials, void* stream) {
  if (P < 0) return set_error(WGSR_EINVAL, "wgsr_gaussian_activate: negative P");
  if (P == 0) return WGSR_OK;
  if (!opacity_raw || !scaling_raw || !rotation_raw || !opacity || !scales || !rotations || !iso_partials)
    return set_error(WGSR_EINVAL, "wgsr_gaussian_activate: null pointer");
  hipLaunchKernelGGL(k_activate, dim3(wgsr_map_blocks(P)), dim3(kMapBlock), 0, (hipStream_t)stream, P, opacity_raw,
                     scaling_raw, rotation_raw, opacity, scales, rotations, iso_partials);
  MAPCHK("wgsr_gaussian_activate");
  return WGSR_OK;
}

int wgsr_gaussian_activate_backward(int P, const float* opacity_raw, const float* scaling_raw,
                                    const float* rotation_raw, const float* dL_dopacity, const float* dL_dscales,
                                    const float* dL_drotations, float iso_weight, float* dL_dopacity_raw,
                                    float* dL_dscaling_raw, float* dL_drotation_raw, void* stream) {
  if (P < 0) return set_error(WGSR_EINVAL, "wgsr_gaussian_activate_backward: negative P");
  if (P == 0) return WGSR_OK;
  if (!opacity_raw || !scaling_raw || !rotation_raw || !dL_dopacity || !dL_dscales || !dL_drotations ||
      !dL_dopacity_raw || !dL_dscaling_raw || !dL_drotation_raw)
    return set_error(WGSR_EINVAL, "wgsr_gaussian_activate_backward: null pointer");
  hipLaunchKernelGGL(k_activate_bwd, dim3(wgsr_map_blocks(P)), dim3(kMapBlock), 0, (hipStream_t)stream, P,
                     opacity_raw, scaling_raw, rotation_raw, dL_dopacity, dL_dscales, dL_drotations, iso_weight,
                     dL_dopacity_raw, dL_dscaling_raw, dL_drotation_raw,
                     DensifyJob{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr});
  MAPCHK("wgsr_gaussian_activate_backward");
  return WGSR_OK;
}

int wgsr_gaussian_activate_backward_stats(int P, const float* opacity_raw, const float* scaling_raw,
                                          const float* rotation_raw, const float* dL_dopacity,
                                          const float* dL_dscales, const float* dL_drotations, float iso_weight,
                                          float* dL_dopacity_raw, float* dL_dscaling_raw, float* dL_drotation_raw,
                                          const int32_t* radii, const float* dL_dmeans2D, float* max_radii2D,
                                          float* grad_accum, float* denom, const uint32_t* skip, void* stream) {
  if (P < 0) return set_error(WGSR_EINVAL, "wgsr_gaussian_activate_backward_stats: negative P");
  if (P == 0) return WGSR_OK;
  if (!opacity_raw || !scaling_raw || !rotation_raw || !dL_dopacity || !dL_dscales || !dL_drotations ||
      !dL_dopacity_raw || !dL_dscaling_raw || !dL_drotation_raw || !radii || !dL_dmeans2D || !max_radii2D ||
      !grad_accum || !denom)
    return set_error(WGSR_EINVAL, "wgsr_gaussian_activate_backward_stats: null pointer");
  hipLaunchKernelGGL(k_activate_bwd, dim3(wgsr_map_blocks(P)), dim3(kMapBlock), 0, (hipStream_t)stream, P,
                     opacity_raw, scaling_raw, rotation_raw, dL_dopacity, dL_dscales, dL_drotations, iso_weight,
                     dL_dopacity_raw, dL_dscaling_raw, dL_drotation_raw,
                     DensifyJob{radii, dL_dmeans2D, max_radii2D, grad_accum, denom, skip});
  MAPCHK("wgsr_gaussian_activate_backward_stats");
  return WGSR_OK;
}

int wgsr_mapping_loss_forward(int H, int W, const float* image, const float* gt_image, const float* depth,
                              const float* gt_depth, const float* exposure_a, const float* exposure_b,
                              float rgb_threshold, float* image_ab, float* partials, void* stream) {
  if (H <= 0 || W <= 0) return set_error(WGSR_EINVAL, "wgsr_mapping_loss_forward: bad image size");
  if (!image || !gt_image || !depth || !gt_depth || !exposure_a || !exposure_b || !image_ab || !partials)
    return set_error(WGSR_EINVAL, "wgsr_mapping_loss_forward: null pointer");
  const int HW = H * W;
  hipLaunchKernelGGL(k_map_loss_fwd, dim3(wgsr_map_blocks(HW)), dim3(kMapBlock), 0, (hipStream_t)stream, HW, image,
                     gt_image, depth, gt_depth, exposure_a, exposure_b, rgb_threshold, image_ab, partials);
  MAPCHK("wgsr_mapping_loss_forward");
  return WGSR_OK;
}

int wgsr_mapping_loss_backward(int H, int W, const float* image, const float* image_ab, const float* gt_image,
                               const float* depth, const float* gt_depth, const float* exposure_a,
                               float rgb_threshold, float w_rgb, float w_depth, const float* ssim_grad,
                               float* dL_dimage, float* dL_ddepth, float* partials, void* stream) {
  if (H <= 0 || W <= 0) return set_error(WGSR_EINVAL, "wgsr_mapping_loss_backward: bad image size");
  if (!image || !image_ab || !gt_image || !depth || !gt_depth || !exposure_a || !dL_dimage || !dL_ddepth ||
      !partials)
    return set_error(WGSR_EINVAL, "wgsr_mapping_loss_backward: null pointer");
  const int HW = H * W;
  hipLaunchKernelGGL(k_map_loss_bwd, dim3(wgsr_map_blocks(HW)), dim3(kMapBlock), 0, (hipStream_t)stream, HW, image,
                     image_ab, gt_image, depth, gt_depth, exposure_a, rgb_threshold, w_rgb, w_depth, ssim_grad,
                     dL_dimage, dL_ddepth, partials);
  MAPCHK("wgsr_mapping_loss_backward");
  return WGSR_OK;
}

int wgsr_densification_stats(int P, const int32_t* radii, const float* dL_dmeans2D, float* max_radii2D,
                             float* grad_accum, float* denom, void* stream) {
  if (P < 0) return set_error(WGSR_EINVAL, "wgsr_densification_stats: negative P");
  if (P == 0) return WGSR_OK;
  if (!radii || !dL_dmeans2D || !max_radii2D || !grad_accum || !denom)
    return set_error(WGSR_EINVAL, "wgsr_densification_stats: null pointer");
  hipLaunchKernelGGL(k_densify_stats, dim3(wgsr_map_blocks(P)), dim3(kMapBlock), 0, (hipStream_t)stream, P, radii,
                     dL_dmeans2D, max_radii2D, grad_accum, denom);
  MAPCHK("wgsr_densification_stats");
  return WGSR_OK;
}

}  // extern "C"
