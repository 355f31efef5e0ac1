// SSIM for the mapping loss, gfx950.
//
//  * wgsr_ssim_forward / wgsr_ssim_backward: loss_utils.ssim (thirdparty/
//    gaussian_splatting/utils/loss_utils.py:61-101), the `1 - ssim(rendered,
//    gt)` term of every mapping iteration (src/utils/slam_utils.py:130, 200).
//    The reference runs 5 depthwise conv2d + ~15 elementwise kernels forward
//    and their adjoints backward; here one launch each way.  The forward
//    keeps, per pixel, dS/dmu1, dS/dE[x^2] and dS/dE[xy] (S = the SSIM map,
//    mu1 = E[x], E = the Gaussian window average); the backward convolves
//    those three maps with the (symmetric) window -- the adjoint of the
//    zero-padded forward conv -- and forms
//        dL/dx = s_plane * (W*dmu1 + 2 x W*dE11 + y W*dE12).
//  * wgsr_ssim_components: compute_ssim_components (src/utils/dyn_uncertainty/
//    mapping_utils.py:99-204): clipped luminance / contrast / structure maps
//    averaged over channels, forward only (the reference detaches them,
//    mapping_utils.py:294).
//
// Layout: images are planes of H x W fp32 (any leading dims flattened).  A
// workgroup owns a 64 x 16 output tile of one plane: the (16+2R) x (64+2R)
// input window is staged in LDS (all global loads issued before the LDS
// writes), the horizontal 1-D pass writes 5 (or 3) row sums per column to
// LDS, and each thread finishes 4 vertically adjacent pixels of one column
// (a wave covers 64 consecutive columns: conflict-free LDS, 256-B stores).
// HBM bound: 8 B read + 12 B written per plane pixel forward, 20 B read + 4 B
// written backward.
#include <math.h>

#include "wgsr_common.h"
#include "wgsr_internal.h"

namespace wgsr {

namespace {

constexpr int kTW = 64, kTH = 16, kRowsPerThread = 4;
constexpr int kMaxWindow = 11;
// Python-float constants as torch rounds them for fp32 tensors
constexpr float kC1 = (float)(0.01 * 0.01);
constexpr float kC2 = (float)(0.03 * 0.03);
constexpr float kC3 = (float)(0.03 * 0.03 / 2);
constexpr float kEps = 1.1920928955078125e-07f;  // torch.finfo(torch.float32).eps
constexpr float kClip = 0.98f;

struct Window {
  float g[kMaxWindow];
};

// 1-D window exactly as loss_utils.gaussian / mapping_utils.generate_gaussian_kernel:
// exp() in double, stored as fp32, divided by the fp32 sum (torch's sum of
// these <= 11 floats equals the exactly rounded sum for every window size).
Window make_window(int ws) {
  Window w{};
  double sum = 0.0;
  for (int x = 0; x < ws; ++x) {
    const double d = (double)(x - ws / 2);
    w.g[x] = (float)exp(-(d * d) / (2.0 * 1.5 * 1.5));
    sum += (double)w.g[x];
  }
  const float fsum = (float)sum;
  for (int x = 0; x < ws; ++x) w.g[x] /= fsum;
  return w;
}

template <int R>
struct Stage {
  static constexpr int IW = kTW + 2 * R, IH = kTH + 2 * R;
  static constexpr int kLoads = (IH * IW + 255) / 256;
  static constexpr int kHItems = (IH * kTW + 255) / 256;
};

// Stage NI input planes (with a zero halo of R) into LDS: all loads first.
template <int R, int NI>
__device__ __forceinline__ void load_window(const float* const (&src)[NI], int H, int W, int gx0, int gy0,
                                            float (*lds)[Stage<R>::IH][Stage<R>::IW]) {
  using S = Stage<R>;
  const int t = threadIdx.x;
  float v[S::kLoads][NI];
#pragma unroll
  for (int k = 0; k < S::kLoads; ++k) {
    const int i = t + 256 * k;
    const int r = i / S::IW, c = i - r * S::IW;
    const int gy = gy0 + r, gx = gx0 + c;
    const bool in = i < S::IH * S::IW && gy >= 0 && gy < H && gx >= 0 && gx < W;
#pragma unroll
    for (int q = 0; q < NI; ++q) v[k][q] = in ? src[q][(int64_t)gy * W + gx] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < S::kLoads; ++k) {
    const int i = t + 256 * k;
    if (i < S::IH * S::IW) {
      const int r = i / S::IW, c = i - r * S::IW;
#pragma unroll
      for (int q = 0; q < NI; ++q) lds[q][r][c] = v[k][q];
    }
  }
}

// Horizontal pass.  Forward (kProducts): the 5 statistics x, y, x^2, y^2, xy
// of the two staged planes; backward: the 3 staged planes as they are.
template <int R, int NQ, bool kProducts>
__device__ __forceinline__ void hpass(const Window& win, float (*in)[Stage<R>::IH][Stage<R>::IW],
                                      float (*hs)[Stage<R>::IH][kTW]) {
  using S = Stage<R>;
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < S::kHItems; ++k) {
    const int i = t + 256 * k;
    if (i >= S::IH * kTW) break;
    const int r = i / kTW, c = i - r * kTW;
    float acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = 0.f;
#pragma unroll
    for (int j = 0; j <= 2 * R; ++j) {
      const float g = win.g[j];
      if constexpr (kProducts) {
        const float a = in[0][r][c + j], b = in[1][r][c + j];
        acc[0] += g * a;
        acc[1] += g * b;
        acc[2] += g * (a * a);
        acc[3] += g * (b * b);
        acc[4] += g * (a * b);
      } else {
#pragma unroll
        for (int q = 0; q < NQ; ++q) acc[q] += g * in[q][r][c + j];
      }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) hs[q][r][c] = acc[q];
  }
}

// Vertical pass: thread (tx, ty) finishes rows 4 ty .. 4 ty + 3 of column tx.
template <int R, int NQ>
__device__ __forceinline__ void vpass(const Window& win, float (*hs)[Stage<R>::IH][kTW],
                                      float (&acc)[kRowsPerThread][NQ]) {
  const int tx = threadIdx.x & (kTW - 1), ty = threadIdx.x / kTW;
#pragma unroll
  for (int o = 0; o < kRowsPerThread; ++o)
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[o][q] = 0.f;
#pragma unroll
  for (int i = 0; i < kRowsPerThread + 2 * R; ++i) {
    float v[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) v[q] = hs[q][kRowsPerThread * ty + i][tx];
#pragma unroll
    for (int o = 0; o < kRowsPerThread; ++o) {
      const int j = i - o;
      if (j >= 0 && j <= 2 * R)
#pragma unroll
        for (int q = 0; q < NQ; ++q) acc[o][q] += win.g[j] * v[q];
    }
  }
}

__device__ __forceinline__ float block_sum_256(float v, float* s_red) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
  __syncthreads();
  return s_red[0] + s_red[1] + s_red[2] + s_red[3];
}

template <int R>
__global__ __launch_bounds__(256) void k_ssim_fwd(const float* __restrict__ img1, const float* __restrict__ img2,
                                                  int H, int W, Window win, float* __restrict__ dmap,
                                                  int64_t plane_stride_all, float* __restrict__ partial) {
  using S = Stage<R>;
  __shared__ float s_in[2][S::IH][S::IW];
  __shared__ float s_h[5][S::IH][kTW];
  __shared__ float s_red[4];
  const int64_t plane = blockIdx.z;
  const int64_t poff = plane * (int64_t)H * W;
  const int tx0 = blockIdx.x * kTW, ty0 = blockIdx.y * kTH;
  const float* const src[2] = {img1 + poff, img2 + poff};
  load_window<R, 2>(src, H, W, tx0 - R, ty0 - R, s_in);
  __syncthreads();
  hpass<R, 5, true>(win, s_in, s_h);
  __syncthreads();
  float acc[kRowsPerThread][5];
  vpass<R, 5>(win, s_h, acc);
  const int gx = tx0 + (threadIdx.x & (kTW - 1));
  const int gyb = ty0 + kRowsPerThread * (threadIdx.x / kTW);
  float ssum = 0.f;
#pragma unroll
  for (int o = 0; o < kRowsPerThread; ++o) {
    const int gy = gyb + o;
    if (gx >= W || gy >= H) continue;
    // loss_utils.py:72-99, in the reference's operation order
    const float mu1 = acc[o][0], mu2 = acc[o][1];
    const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu1_mu2 = mu1 * mu2;
    const float s11 = acc[o][2] - mu1_sq, s22 = acc[o][3] - mu2_sq, s12 = acc[o][4] - mu1_mu2;
    const float A = 2.f * mu1_mu2 + kC1, B = 2.f * s12 + kC2;
    const float C = mu1_sq + mu2_sq + kC1, D = s11 + s22 + kC2;
    const float S_ = (A * B) / (C * D);
    ssum += S_;
    if (dmap) {
      const float iCD = 1.f / (C * D);
      const int64_t p = poff + (int64_t)gy * W + gx;
      dmap[p] = 2.f * mu2 * (B - A) * iCD - 2.f * mu1 * S_ * (1.f / C - 1.f / D);  // dS/dmu1
      dmap[plane_stride_all + p] = -S_ / D;                                    // dS/dE[x^2]
      dmap[2 * plane_stride_all + p] = 2.f * A * iCD;                          // dS/dE[xy]
    }
  }
  const float tot = block_sum_256(ssum, s_red);
  if (threadIdx.x == 0) partial[(plane * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] = tot;
}

// per-plane sums of the tile partials in a fixed order (double), the plane
// means and the mean over everything
__global__ __launch_bounds__(256) void k_ssim_reduce(const float* __restrict__ partial, int64_t planes,
                                                     int tiles, double inv_plane_px, float* __restrict__ plane_mean,
                                                     float* __restrict__ mean) {
  __shared__ double s_red[256];
  const float m = ssim_partials_mean(partial, planes, tiles, inv_plane_px, plane_mean, s_red);
  if (threadIdx.x == 0) mean[0] = m;
}

template <int R>
__global__ __launch_bounds__(256) void k_ssim_bwd(const float* __restrict__ img1, const float* __restrict__ img2,
                                                  const float* __restrict__ dmap, int64_t plane_stride_all,
                                                  const float* __restrict__ plane_scale, int H, int W, Window win,
                                                  float* __restrict__ grad1) {
  using S = Stage<R>;
  __shared__ float s_in[3][S::IH][S::IW];
  __shared__ float s_h[3][S::IH][kTW];
  const int64_t plane = blockIdx.z;
  const int64_t poff = plane * (int64_t)H * W;
  const int tx0 = blockIdx.x * kTW, ty0 = blockIdx.y * kTH;
  const float* const src[3] = {dmap + poff, dmap + plane_stride_all + poff, dmap + 2 * plane_stride_all + poff};
  load_window<R, 3>(src, H, W, tx0 - R, ty0 - R, s_in);
  __syncthreads();
  hpass<R, 3, false>(win, s_in, s_h);
  __syncthreads();
  float acc[kRowsPerThread][3];
  vpass<R, 3>(win, s_h, acc);
  const float scale = plane_scale[plane];
  const int gx = tx0 + (threadIdx.x & (kTW - 1));
  const int gyb = ty0 + kRowsPerThread * (threadIdx.x / kTW);
#pragma unroll
  for (int o = 0; o < kRowsPerThread; ++o) {
    const int gy = gyb + o;
    if (gx >= W || gy >= H) continue;
    const int64_t p = poff + (int64_t)gy * W + gx;
    grad1[p] = scale * (acc[o][0] + 2.f * img1[p] * acc[o][1] + img2[p] * acc[o][2]);
  }
}

// mapping_utils.py:125-204 for all channels of one image: channel means of
// the clipped luminance / contrast / structure maps
template <int R>
__global__ __launch_bounds__(256) void k_ssim_components(const float* __restrict__ img1,
                                                         const float* __restrict__ img2, int channels, int H, int W,
                                                         Window win, float* __restrict__ lum,
                                                         float* __restrict__ con, float* __restrict__ str) {
  using S = Stage<R>;
  __shared__ float s_in[2][S::IH][S::IW];
  __shared__ float s_h[5][S::IH][kTW];
  const int64_t img = blockIdx.z;
  const int64_t plane_px = (int64_t)H * W;
  const int tx0 = blockIdx.x * kTW, ty0 = blockIdx.y * kTH;
  const int gx = tx0 + (threadIdx.x & (kTW - 1));
  const int gyb = ty0 + kRowsPerThread * (threadIdx.x / kTW);
  float ls[kRowsPerThread] = {}, cs[kRowsPerThread] = {}, ss[kRowsPerThread] = {};
  for (int ch = 0; ch < channels; ++ch) {
    const int64_t poff = (img * channels + ch) * plane_px;
    const float* const src[2] = {img1 + poff, img2 + poff};
    if (ch) __syncthreads();  // the previous channel's vertical pass is done with s_h
    load_window<R, 2>(src, H, W, tx0 - R, ty0 - R, s_in);
    __syncthreads();
    hpass<R, 5, true>(win, s_in, s_h);
    __syncthreads();
    float acc[kRowsPerThread][5];
    vpass<R, 5>(win, s_h, acc);
#pragma unroll
    for (int o = 0; o < kRowsPerThread; ++o) {
      const float mu1 = acc[o][0], mu2 = acc[o][1];
      const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu1_mu2 = mu1 * mu2;
      const float s11 = fmaxf(kEps, acc[o][2] - mu1_sq);
      const float s22 = fmaxf(kEps, acc[o][3] - mu2_sq);
      float s12 = acc[o][4] - mu1_mu2;
      const float lim = sqrtf(s11 * s22);
      s12 = s12 > 0.f ? fminf(lim, s12) : (s12 < 0.f ? -fminf(lim, -s12) : 0.f);
      const float sd1 = sqrtf(s11), sd2 = sqrtf(s22);
      const float l = (2.f * mu1_mu2 + kC1) / (mu1_sq + mu2_sq + kC1);
      const float c = fminf((2.f * sd1 * sd2 + kC2) / (s11 + s22 + kC2), kClip);
      const float s = fminf((s12 + kC3) / (sd1 * sd2 + kC3), kClip);
      ls[o] += l;
      cs[o] += c;
      ss[o] += s;
    }
  }
#pragma unroll
  for (int o = 0; o < kRowsPerThread; ++o) {
    const int gy = gyb + o;
    if (gx >= W || gy >= H) continue;
    const int64_t p = img * plane_px + (int64_t)gy * W + gx;
    // torch's mean(1): the channel sum divided by the count
    lum[p] = ls[o] / (float)channels;
    con[p] = cs[o] / (float)channels;
    str[p] = ss[o] / (float)channels;
  }
}

bool window_ok(int ws) { return ws == 3 || ws == 5 || ws == 7 || ws == 9 || ws == 11; }

}  // namespace

}  // namespace wgsr

using namespace wgsr;

#define WGSR_SSIM_DISPATCH(ws, KERNEL, ...)                                                  \
  switch (ws) {                                                                            \
    case 3: hipLaunchKernelGGL(KERNEL<1>, __VA_ARGS__); break;                             \
    case 5: hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__); break;                             \
    case 7: hipLaunchKernelGGL(KERNEL<3>, __VA_ARGS__); break;                             \
    case 9: hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__); break;                             \
    default: hipLaunchKernelGGL(KERNEL<5>, __VA_ARGS__); break;                            \
  }

extern "C" {

size_t wgsr_ssim_scratch_bytes(int64_t planes, int H, int W) {
  if (planes <= 0 || H <= 0 || W <= 0) return 0;
  const int64_t tiles = (int64_t)((W + kTW - 1) / kTW) * ((H + kTH - 1) / kTH);
  return (size_t)(4 * planes * tiles);
}

int wgsr_ssim_forward(const float* img1, const float* img2, int64_t planes, int H, int W, int window_size,
                      float* dmap, float* plane_mean, float* mean, wgsr_alloc_fn scratch_alloc, void* ctx,
                      void* stream) {
  if (planes <= 0 || H <= 0 || W <= 0 || planes > 65535 || !window_ok(window_size))
    return set_error(WGSR_EINVAL, "wgsr_ssim_forward: bad shape (%lld planes of %dx%d) or window %d",
                     (long long)planes, H, W, window_size);
  if (!img1 || !img2 || !mean) return set_error(WGSR_EINVAL, "wgsr_ssim_forward: null pointer");
  const dim3 grid((W + kTW - 1) / kTW, (H + kTH - 1) / kTH, (unsigned)planes);
  float* partial = static_cast<float*>(scratch_alloc(ctx, wgsr_ssim_scratch_bytes(planes, H, W)));
  if (!partial) return set_error(WGSR_EALLOC, "wgsr_ssim_forward: scratch allocation failed");
  hipStream_t s = (hipStream_t)stream;
  const Window win = make_window(window_size);
  const int64_t all = planes * (int64_t)H * W;
  WGSR_SSIM_DISPATCH(window_size, k_ssim_fwd, grid, dim3(256), 0, s, img1, img2, H, W, win, dmap, all, partial);
  hipLaunchKernelGGL(k_ssim_reduce, dim3(1), dim3(256), 0, s, partial, planes, (int)(grid.x * grid.y),
                     1.0 / ((double)H * W), plane_mean, mean);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? WGSR_OK : set_error(WGSR_EHIP, "wgsr_ssim_forward: %s", hipGetErrorString(e));
}

int wgsr_ssim_forward_partials(const float* img1, const float* img2, int64_t planes, int H, int W, int window_size,
                               float* dmap, float* partials, void* stream) {
  if (planes <= 0 || H <= 0 || W <= 0 || planes > 65535 || !window_ok(window_size))
    return set_error(WGSR_EINVAL, "wgsr_ssim_forward_partials: bad shape or window %d", window_size);
  if (!img1 || !img2 || !partials) return set_error(WGSR_EINVAL, "wgsr_ssim_forward_partials: null pointer");
  const dim3 grid((W + kTW - 1) / kTW, (H + kTH - 1) / kTH, (unsigned)planes);
  const Window win = make_window(window_size);
  const int64_t all = planes * (int64_t)H * W;
  WGSR_SSIM_DISPATCH(window_size, k_ssim_fwd, grid, dim3(256), 0, (hipStream_t)stream, img1, img2, H, W, win, dmap,
                     all, partials);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? WGSR_OK : set_error(WGSR_EHIP, "wgsr_ssim_forward_partials: %s", hipGetErrorString(e));
}

int wgsr_ssim_tiles(int H, int W) { return (H > 0 && W > 0) ? ((W + kTW - 1) / kTW) * ((H + kTH - 1) / kTH) : 0; }

int wgsr_ssim_backward(const float* img1, const float* img2, int64_t planes, int H, int W, int window_size,
                       const float* dmap, const float* plane_scale, float* grad_img1, void* stream) {
  if (planes <= 0 || H <= 0 || W <= 0 || planes > 65535 || !window_ok(window_size))
    return set_error(WGSR_EINVAL, "wgsr_ssim_backward: bad shape or window %d", window_size);
  if (!img1 || !img2 || !dmap || !plane_scale || !grad_img1)
    return set_error(WGSR_EINVAL, "wgsr_ssim_backward: null pointer");
  const dim3 grid((W + kTW - 1) / kTW, (H + kTH - 1) / kTH, (unsigned)planes);
  hipStream_t s = (hipStream_t)stream;
  const Window win = make_window(window_size);
  const int64_t all = planes * (int64_t)H * W;
  WGSR_SSIM_DISPATCH(window_size, k_ssim_bwd, grid, dim3(256), 0, s, img1, img2, dmap, all, plane_scale, H, W, win,
                     grad_img1);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? WGSR_OK : set_error(WGSR_EHIP, "wgsr_ssim_backward: %s", hipGetErrorString(e));
}

int wgsr_ssim_components(const float* img1, const float* img2, int64_t images, int channels, int H, int W,
                         int window_size, float* luminance, float* contrast, float* structure, void* stream) {
  if (images <= 0 || images > 65535 || channels <= 0 || H <= 0 || W <= 0 || !window_ok(window_size))
    return set_error(WGSR_EINVAL, "wgsr_ssim_components: bad shape or window %d", window_size);
  if (!img1 || !img2 || !luminance || !contrast || !structure)
    return set_error(WGSR_EINVAL, "wgsr_ssim_components: null pointer");
  const dim3 grid((W + kTW - 1) / kTW, (H + kTH - 1) / kTH, (unsigned)images);
  hipStream_t s = (hipStream_t)stream;
  const Window win = make_window(window_size);
  WGSR_SSIM_DISPATCH(window_size, k_ssim_components, grid, dim3(256), 0, s, img1, img2, channels, H, W, win,
                     luminance, contrast, structure);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? WGSR_OK : set_error(WGSR_EHIP, "wgsr_ssim_components: %s", hipGetErrorString(e));
}

}  // extern "C"
