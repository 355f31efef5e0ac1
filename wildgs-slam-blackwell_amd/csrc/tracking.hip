// The mapper's pose-refinement loss around the rasteriser, gfx950 (SURVEY.md
// 8(f) row f2, the tracking half: src/mapper.py:856-911 runs 100 iterations of
// render -> get_loss_tracking -> backward -> pose/exposure Adam per refined
// keyframe).
//
//   track_loss  get_loss_tracking / get_loss_tracking_rgb (src/utils/
//               slam_utils.py:47-82): exposure-corrected image, boundary mask
//               x the keyframe's gradient mask, opacity-weighted L1, optional
//               uncertainty weights.  The loss is a weighted L1 whose weights
//               do not depend on the parameters, so ONE pass writes the loss
//               partial sums and every gradient (image, opacity, exposure).
//   grad_mask   Camera.compute_grad_mask (src/utils/camera_utils.py:157-180
//               with slam_utils.image_gradient / image_gradient_mask :10-44):
//               Scharr gradient magnitude of the grey image where the whole
//               reflect-padded 3x3 neighbourhood is above eps, then a 32 x 32
//               grid of blocks thresholded at 4 x the block median.  The
//               reference runs ~3000 small kernels per keyframe for this (a
//               Python loop of 1024 medians); here it is two launches.
#include <math.h>

#include "wgsr_common.h"
#include "wgsr_internal.h"

#pragma clang fp contract(off)

namespace wgsr {

namespace {

constexpr int kTBlock = 256;

__device__ __forceinline__ float tblock_sum(float v, float* sred) {
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

__device__ __forceinline__ float tsgn(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

__global__ __launch_bounds__(kTBlock) void k_track_loss(int HW, const float* __restrict__ image,
                                                        const float* __restrict__ gt,
                                                        const float* __restrict__ opacity,
                                                        const float* __restrict__ grad_mask,
                                                        const float* __restrict__ unc,
                                                        const float* __restrict__ expo_a,
                                                        const float* __restrict__ expo_b, float rgb_th, float inv_n,
                                                        float* __restrict__ d_image, float* __restrict__ d_opacity,
                                                        float* __restrict__ part) {
  __shared__ float sred[kTBlock / 64];
  const int p = blockIdx.x * kTBlock + threadIdx.x;
  const float ea = expf(expo_a[0]), b = expo_b[0];
  float ls = 0.f, da = 0.f, db = 0.f;
  if (p < HW) {
    const float g[3] = {gt[p], gt[HW + p], gt[2 * HW + p]};
    float m = ((g[0] + g[1]) + g[2]) > rgb_th ? 1.f : 0.f;
    if (grad_mask) m = m * grad_mask[p];  // rgb_pixel_mask * viewpoint.grad_mask
    float wgt = 1.f;
    if (unc) {
      const float u = unc[p];
      wgt = (1.f / (u * u)) * 0.5f;  // torch's 0.5 / t is t.reciprocal() * 0.5
      wgt = wgt < 0.1f ? 0.f : wgt;
    }
    const float op = opacity[p];
    float dop = 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const size_t k = (size_t)c * HW + p;
      const float x = image[k];
      const float a = ea * x + b;
      const float r = a * m - g[c] * m;
      float l1 = op * fabsf(r);
      float ad = fabsf(r);
      if (unc) {
        l1 = l1 * wgt;
        ad = ad * wgt;
      }
      ls += l1;
      dop += ad;
      float gab = inv_n * op * tsgn(r) * m;
      if (unc) gab = gab * wgt;
      d_image[k] = gab * ea;
      da += gab * x * ea;
      db += gab;
    }
    if (d_opacity) d_opacity[p] = inv_n * dop;
  }
  const float s0 = tblock_sum(ls, sred);
  const float s1 = tblock_sum(da, sred);
  const float s2 = tblock_sum(db, sred);
  if (threadIdx.x == 0) {
    part[3 * blockIdx.x] = s0;
    part[3 * blockIdx.x + 1] = s1;
    part[3 * blockIdx.x + 2] = s2;
  }
}

__device__ __forceinline__ int refl(int i, int n) {  // F.pad(mode="reflect") by one pixel
  return i < 0 ? -i : (i >= n ? 2 * (n - 1) - i : i);
}

__device__ __forceinline__ float grey_at(const float* __restrict__ img, int HW, int W, int y, int x) {
  const int p = y * W + x;
  return ((img[p] + img[HW + p]) + img[2 * HW + p]) * (1.f / 3.f);  // mean(dim=0): sum x (1/3)
}

// Scharr gradient magnitude with the eps neighbourhood mask, every pixel
// (the pixels outside the 32 x 32 grid of blocks keep it).
__global__ __launch_bounds__(kTBlock) void k_grad_intensity(int H, int W, const float* __restrict__ img, float eps,
                                                            float* __restrict__ out) {
  const int p = blockIdx.x * kTBlock + threadIdx.x;
  if (p >= H * W) return;
  const int HW = H * W;
  const int y = p / W, x = p - y * W;
  float v[3][3];
  bool all = true;
#pragma unroll
  for (int dy = 0; dy < 3; ++dy)
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      v[dy][dx] = grey_at(img, HW, W, refl(y + dy - 1, H), refl(x + dx - 1, W));
      all = all && (fabsf(v[dy][dx]) > eps);
    }
  // conv2d (cross-correlation) with conv_x = [[3,10,3],[0,0,0],[-3,-10,-3]]
  // and conv_y = [[3,0,-3],[10,0,-10],[3,0,-3]], scaled by 1/32
  const float cx = 3.f * v[0][0] + 10.f * v[0][1] + 3.f * v[0][2] - 3.f * v[2][0] - 10.f * v[2][1] - 3.f * v[2][2];
  const float cy = 3.f * v[0][0] - 3.f * v[0][2] + 10.f * v[1][0] - 10.f * v[1][2] + 3.f * v[2][0] - 3.f * v[2][2];
  const float m = all ? 1.f : 0.f;
  const float gv = (0.03125f * cx) * m, gh = (0.03125f * cy) * m;
  out[p] = sqrtf(gv * gv + gh * gh);
}

// One workgroup per grid block: lower median of the block's intensities
// (bitonic sort in LDS), then the reference's two masked assignments.
constexpr int kMaskSort = 8192;

__global__ __launch_bounds__(kTBlock) void k_grad_block(int H, int W, int bh, int bw, float multiplier,
                                                        float* __restrict__ out) {
  __shared__ float s[kMaskSort];
  const int r = blockIdx.x / 32, c = blockIdx.x % 32;
  const int n = bh * bw;
  int np = 1;
  while (np < n) np <<= 1;
  for (int i = threadIdx.x; i < np; i += kTBlock) {
    float v = __int_as_float(0x7f800000);  // +inf padding sorts last
    if (i < n) v = out[(r * bh + i / bw) * W + c * bw + i % bw];
    s[i] = v;
  }
  __syncthreads();
  for (int k = 2; k <= np; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < np; i += kTBlock) {
        const int l = i ^ j;
        if (l > i) {
          const float a = s[i], b = s[l];
          const bool up = (i & k) == 0;
          if ((a > b) == up) {
            s[i] = b;
            s[l] = a;
          }
        }
      }
      __syncthreads();
    }
  const float t = s[(n - 1) / 2] * multiplier;  // torch.median: the lower median
  const float hi = (1.f <= t) ? 0.f : 1.f;      // block[v > t] = 1, then block[v <= t] = 0
  for (int i = threadIdx.x; i < n; i += kTBlock) {
    float* q = &out[(r * bh + i / bw) * W + c * bw + i % bw];
    *q = (*q > t) ? hi : 0.f;
  }
}

// ---- one pose-refinement update (mapper.py:884-906 after the backward) ----
// state (floats): [0,9) R row-major | [9,12) T | 12 exposure_a | 13 exposure_b |
// [16,24) Adam exp_avg of (rot 3, trans 3, exposure_a, exposure_b) | [24,32)
// exp_avg_sq | [32,48) viewmatrix | [48,64) projmatrix | [64,67) campos |
// 67 |tau| of the update.  The viewmatrix / projmatrix / campos are the
// rasteriser inputs of the NEXT iteration (Camera.world_view_transform,
// full_proj_transform, camera_center).
constexpr int kPoseState = 68;

__device__ __forceinline__ void mat3_mul(const float A[9], const float B[9], float C[9]) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

// rasteriser camera fields from (R, T) and the stored projection matrix
__device__ void pose_camera(const float R[9], const float T[3], const float* __restrict__ proj_t, float* st) {
  float Wv[16];
  // getWorld2View2(R, T).transpose(0, 1) = [[R^T, 0], [T^T, 1]]
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j) Wv[4 * i + j] = R[3 * j + i];
    Wv[4 * i + 3] = 0.f;
  }
  Wv[12] = T[0]; Wv[13] = T[1]; Wv[14] = T[2]; Wv[15] = 1.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) st[32 + k] = Wv[k];
  // full_proj_transform = world_view_transform @ projection_matrix
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      st[48 + 4 * i + j] = Wv[4 * i] * proj_t[j] + Wv[4 * i + 1] * proj_t[4 + j] + Wv[4 * i + 2] * proj_t[8 + j] +
                           Wv[4 * i + 3] * proj_t[12 + j];
  // camera_center = inverse(world_view_transform)[3, :3] = -T^T R
#pragma unroll
  for (int j = 0; j < 3; ++j) st[64 + j] = -(T[0] * R[j] + T[1] * R[3 + j] + T[2] * R[6 + j]);
}

constexpr int kPoseThreads = 1024;

__global__ __launch_bounds__(kPoseThreads) void k_pose_step(float* __restrict__ st, const float* __restrict__ dtau,
                                                  const float* __restrict__ part, int nb,
                                                  const float* __restrict__ proj_t, float lr_rot, float lr_trans,
                                                  float lr_expo, float beta1, float beta2, float eps, float bc1,
                                                  float bc2_sqrt, float conv_th, int* __restrict__ converged,
                                                  int camera_only) {
  __shared__ float sred[2][kPoseThreads / 64];
  const int t = threadIdx.x;
  float ga = 0.f, gb = 0.f;
  for (int b = t; b < nb; b += kPoseThreads) {  // exposure gradients: fixed-order sums of the loss partials
    ga += part[3 * b + 1];
    gb += part[3 * b + 2];
  }
  ga = wave_sum(ga);
  gb = wave_sum(gb);
  if ((t & 63) == 0) {
    sred[0][t >> 6] = ga;
    sred[1][t >> 6] = gb;
  }
  __syncthreads();
  if (t != 0) return;
  ga = gb = 0.f;
  for (int w = 0; w < kPoseThreads / 64; ++w) {
    ga += sred[0][w];
    gb += sred[1][w];
  }
  float R[9], T[3];
#pragma unroll
  for (int k = 0; k < 9; ++k) R[k] = st[k];
  T[0] = st[9]; T[1] = st[10]; T[2] = st[11];
  if (camera_only) {
    pose_camera(R, T, proj_t, st);
    return;
  }
  // Adam over (cam_rot_delta, cam_trans_delta, exposure_a, exposure_b), whose
  // deltas are 0 at every step start (update_pose resets them)
  const float g[8] = {dtau[3], dtau[4], dtau[5], dtau[0], dtau[1], dtau[2], ga, gb};
  const float lr[8] = {lr_rot, lr_rot, lr_rot, lr_trans, lr_trans, lr_trans, lr_expo, lr_expo};
  float pnew[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float m = beta1 * st[16 + k] + (1.f - beta1) * g[k];
    const float v = beta2 * st[24 + k] + (1.f - beta2) * g[k] * g[k];
    st[16 + k] = m;
    st[24 + k] = v;
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    const float p0 = k < 6 ? 0.f : st[12 + (k - 6)];
    pnew[k] = p0 - (lr[k] / bc1) * (m / denom);
  }
  st[12] = pnew[6];
  st[13] = pnew[7];
  // update_pose (pose_utils.py:81-98): tau = [trans, rot], new_w2c = SE3_exp(tau) @ w2c
  const float rho[3] = {pnew[3], pnew[4], pnew[5]}, th[3] = {pnew[0], pnew[1], pnew[2]};
  const float Wm[9] = {0.f, -th[2], th[1], th[2], 0.f, -th[0], -th[1], th[0], 0.f};
  float W2[9];
  mat3_mul(Wm, Wm, W2);
  const float angle = sqrtf(th[0] * th[0] + th[1] * th[1] + th[2] * th[2]);
  float Rx[9], Vm[9];
  if (angle < 1e-5f) {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const float I = (k % 4 == 0) ? 1.f : 0.f;
      Rx[k] = I + Wm[k] + 0.5f * W2[k];
      Vm[k] = I + 0.5f * Wm[k] + (1.f / 6.f) * W2[k];
    }
  } else {
    const float sa = sinf(angle), ca = cosf(angle), a2 = angle * angle;
    const float c1 = sa / angle, c2 = (1.f - ca) / a2, c3 = (angle - sa) / (a2 * angle);
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const float I = (k % 4 == 0) ? 1.f : 0.f;
      Rx[k] = I + c1 * Wm[k] + c2 * W2[k];
      Vm[k] = I + Wm[k] * c2 + W2[k] * c3;
    }
  }
  float Rn[9];
  mat3_mul(Rx, R, Rn);
  float Tn[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float t = Vm[3 * i] * rho[0] + Vm[3 * i + 1] * rho[1] + Vm[3 * i + 2] * rho[2];
    Tn[i] = Rx[3 * i] * T[0] + Rx[3 * i + 1] * T[1] + Rx[3 * i + 2] * T[2] + t;
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) st[k] = Rn[k];
  st[9] = Tn[0]; st[10] = Tn[1]; st[11] = Tn[2];
  const float tn = sqrtf(rho[0] * rho[0] + rho[1] * rho[1] + rho[2] * rho[2] + th[0] * th[0] + th[1] * th[1] +
                         th[2] * th[2]);
  st[67] = tn;
  converged[0] = tn < conv_th ? 1 : 0;
  pose_camera(Rn, Tn, proj_t, st);
}

}  // namespace
}  // namespace wgsr

using namespace wgsr;

#define TRKCHK(name)                                                                         \
  do {                                                                                       \
    const hipError_t _e = hipGetLastError();                                                 \
    if (_e != hipSuccess) return set_error(WGSR_EHIP, "%s: %s", name, hipGetErrorString(_e)); \
  } while (0)

extern "C" {

int wgsr_track_blocks(int64_t n) { return n > 0 ? (int)((n + kTBlock - 1) / kTBlock) : 0; }

int wgsr_tracking_loss(int H, int W, const float* image, const float* gt_image, const float* opacity,
                       const float* grad_mask, const float* uncertainty, const float* exposure_a,
                       const float* exposure_b, float rgb_threshold, float* dL_dimage, float* dL_dopacity,
                       float* partials, void* stream) {
  if (H <= 0 || W <= 0 || (int64_t)H * W > (int64_t)INT32_MAX / 3)
    return set_error(WGSR_EINVAL, "wgsr_tracking_loss: bad image size %dx%d", H, W);
  if (!image || !gt_image || !opacity || !exposure_a || !exposure_b || !dL_dimage || !partials)
    return set_error(WGSR_EINVAL, "wgsr_tracking_loss: null pointer");
  const int HW = H * W;
  hipLaunchKernelGGL(k_track_loss, dim3(wgsr_track_blocks(HW)), dim3(kTBlock), 0, (hipStream_t)stream, HW, image,
                     gt_image, opacity, grad_mask, uncertainty, exposure_a, exposure_b, rgb_threshold,
                     1.f / (3.f * (float)HW), dL_dimage, dL_dopacity, partials);
  TRKCHK("wgsr_tracking_loss");
  return WGSR_OK;
}

int wgsr_grad_mask(int H, int W, const float* image, float edge_threshold, float* grad_mask, void* stream) {
  if (H < 2 || W < 2 || (int64_t)H * W > (int64_t)INT32_MAX / 3)
    return set_error(WGSR_EINVAL, "wgsr_grad_mask: bad image size %dx%d (reflect padding needs >= 2)", H, W);
  if (!image || !grad_mask) return set_error(WGSR_EINVAL, "wgsr_grad_mask: null pointer");
  const int bh = H / 32, bw = W / 32;
  if ((int64_t)bh * bw > kMaskSort)
    return set_error(WGSR_EINVAL, "wgsr_grad_mask: %dx%d blocks exceed %d pixels", bh, bw, kMaskSort);
  hipLaunchKernelGGL(k_grad_intensity, dim3(wgsr_track_blocks((int64_t)H * W)), dim3(kTBlock), 0,
                     (hipStream_t)stream, H, W, image, 0.01f, grad_mask);
  if (bh > 0 && bw > 0)
    hipLaunchKernelGGL(k_grad_block, dim3(32 * 32), dim3(kTBlock), 0, (hipStream_t)stream, H, W, bh, bw,
                       edge_threshold, grad_mask);
  TRKCHK("wgsr_grad_mask");
  return WGSR_OK;
}

int wgsr_pose_state_floats(void) { return kPoseState; }

int wgsr_pose_step(float* state, const float* dtau, const float* loss_partials, int n_partials,
                   const float* projection_matrix, float lr_rot, float lr_trans, float lr_exposure, float beta1,
                   float beta2, float eps, int step, float converged_threshold, int* converged, int camera_only,
                   void* stream) {
  if (!state || !projection_matrix || (!camera_only && (!dtau || !loss_partials || !converged || step < 1)))
    return set_error(WGSR_EINVAL, "wgsr_pose_step: bad arguments");
  const double bc1 = camera_only ? 1.0 : 1.0 - pow((double)beta1, step);
  const double bc2 = camera_only ? 1.0 : 1.0 - pow((double)beta2, step);
  hipLaunchKernelGGL(k_pose_step, dim3(1), dim3(kPoseThreads), 0, (hipStream_t)stream, state, dtau, loss_partials,
                     camera_only ? 0 : n_partials, projection_matrix, lr_rot, lr_trans, lr_exposure, beta1, beta2,
                     eps, (float)bc1, (float)sqrt(bc2), converged_threshold, converged, camera_only);
  TRKCHK("wgsr_pose_step");
  return WGSR_OK;
}

}  // extern "C"
