// Map deformation on the device, gfx950:
// Mapper._update_keyframes_from_frontend -> _update_mapping_points
// (src/mapper.py:365-558) for EVERY keyframe whose pose / depth changed, in
// one pass over the GaussianStore rows instead of ~25 torch launches per
// keyframe (boolean masks, cat, two 4x4 GEMMs over the masked rows, gathers,
// scatters and three replace_tensor_to_optimizer re-allocations).
//
// Per keyframe k with at least one row anchored to it (unique_kfIDs == k):
//   T_k = inv(inv(w2c_old) @ w2c_new)            (host, 4x4)
//   q_k = rotation_matrix_to_quaternion(T_k)      (host, general_utils.py:138-162)
//   rigid:  xyz <- (T_k [xyz, 1])[:3]
//   depth:  pc = (w2c_old [xyz, 1])[:3]; pix = K pc; (u, v) = trunc(pix.xy /
//           pix.z) clamped to the image; d, d_old = the new / old depth at
//           (v, u); s = 1 + (1 / pc.z) (d - d_old), s = 1 where d == 0 or
//           d_old == 0 or s <= 0; xyz <- (T_k [(c2w_old [s pc, 1])[:3], 1])[:3];
//           scaling (raw, log) += log(s)
//   rotation (both): raw <- q_k (x) normalize(raw)
// and, once any keyframe has rows (the reference returns early otherwise):
//   EVERY row's raw rotation <- normalize(raw) (the reference writes
//   get_rotation -- the activated tensor -- back as the new parameter), the
//   Adam moments of xyz and rotation -> 0 (replace_tensor_to_optimizer,
//   gaussian_model.py:495-508), and those of scaling too when a depth-branch
//   keyframe had rows.  A row belongs to one keyframe, so applying every
//   keyframe in one pass equals the reference's sequence of calls up to the
//   repeated normalisation's rounding.
//
// Two launches: k_deform_any (which branches have rows: one ballot + one
// atomic per wave into a 2-word flag block) and k_deform_apply (every row;
// the whole grid exits at once when no branch has rows).
#include "wgsr_common.h"
#include "wgsr_internal.h"

namespace wgsr {

namespace {

constexpr int kDefBlock = 256;

__device__ __forceinline__ float fmul(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float fadd(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float fsub(float a, float b) { return __fsub_rn(a, b); }

// rows 0..2 of a row-major 4x4 applied to [x, y, z, 1] (a GEMM row: k = 0..3)
__device__ __forceinline__ void affine(const float* M, float x, float y, float z, float& ox, float& oy, float& oz) {
  ox = fmaf(M[2], z, fmaf(M[1], y, fmul(M[0], x))) + M[3];
  oy = fmaf(M[6], z, fmaf(M[5], y, fmul(M[4], x))) + M[7];
  oz = fmaf(M[10], z, fmaf(M[9], y, fmul(M[8], x))) + M[11];
}

// torch's float -> int64 (CUDA semantics: saturating, NaN -> 0), then clamp
__device__ __forceinline__ int pix_index(float f, int n) {
  if (!(f == f)) return 0;
  const float t = truncf(f);
  if (t <= 0.f) return 0;
  if (t >= (float)(n - 1)) return n - 1;
  return (int)t;
}

__global__ __launch_bounds__(kDefBlock) void k_deform_any(int64_t P, const int32_t* __restrict__ kf_id,
                                                         const int32_t* __restrict__ lut, int lut_size,
                                                         const wgsr_deform_frame* __restrict__ frames,
                                                         uint32_t* __restrict__ flags) {
  const int64_t i = (int64_t)blockIdx.x * kDefBlock + threadIdx.x;
  int method = -1;
  if (i < P) {
    const int k = kf_id[i];
    const int f = (k >= 0 && k < lut_size) ? lut[k] : -1;
    if (f >= 0) method = frames[f].method;
  }
  const uint64_t rigid = wave_ballot(method == 0), depth = wave_ballot(method == 1);
  if ((threadIdx.x & 63) == 0) {
    if (rigid) atomicOr(&flags[0], 1u);
    if (depth) atomicOr(&flags[1], 1u);
  }
}

__global__ __launch_bounds__(kDefBlock) void k_deform_apply(int64_t P, wgsr_gaussian_bank bank,
                                                           const int32_t* __restrict__ lut, int lut_size,
                                                           const wgsr_deform_frame* __restrict__ frames,
                                                           const uint32_t* __restrict__ flags) {
  const uint32_t any_rigid = flags[0], any_depth = flags[1];
  if (!(any_rigid | any_depth)) return;   // the reference's early return: nothing changes
  const int64_t i = (int64_t)blockIdx.x * kDefBlock + threadIdx.x;
  if (i >= P) return;
  const int k = bank.kf_id[i];
  const int f = (k >= 0 && k < lut_size) ? lut[k] : -1;

  // get_rotation = F.normalize(raw, dim=1): x / max(||x||, 1e-12)
  float4 q = reinterpret_cast<const float4*>(bank.rotation)[i];
  {
    const float n2 = fadd(fadd(fadd(fmul(q.x, q.x), fmul(q.y, q.y)), fmul(q.z, q.z)), fmul(q.w, q.w));
    const float nrm = fmaxf(sqrtf(n2), 1e-12f);
    q = make_float4(q.x / nrm, q.y / nrm, q.z / nrm, q.w / nrm);
  }
  if (f >= 0) {
    const wgsr_deform_frame& F = frames[f];
    float* xyz = bank.xyz + 3 * i;
    float x = xyz[0], y = xyz[1], z = xyz[2];
    if (F.method == 1) {
      float cx, cy, cz;
      affine(F.w2c_old, x, y, z, cx, cy, cz);
      const float* K = F.K;
      const float px = fmaf(K[2], cz, fmaf(K[1], cy, fmul(K[0], cx)));
      const float py = fmaf(K[5], cz, fmaf(K[4], cy, fmul(K[3], cx)));
      const float pz = fmaf(K[8], cz, fmaf(K[7], cy, fmul(K[6], cx)));
      const int u = pix_index(px / pz, F.W), v = pix_index(py / pz, F.H);
      const float d = F.depth[(int64_t)v * F.W + u], d_old = F.depth_old[(int64_t)v * F.W + u];
      float s = fadd(1.0f, fmul(1.0f / cz, fsub(d, d_old)));
      if (d == 0.f || d_old == 0.f || s <= 0.f) s = 1.0f;
      affine(F.c2w_old, fmul(s, cx), fmul(s, cy), fmul(s, cz), x, y, z);
      float* sc = bank.scaling + 3 * i;
      const float ls = logf(s);
      sc[0] = fadd(sc[0], ls);
      sc[1] = fadd(sc[1], ls);
      sc[2] = fadd(sc[2], ls);
    }
    float ox, oy, oz;
    affine(F.T, x, y, z, ox, oy, oz);
    xyz[0] = ox;
    xyz[1] = oy;
    xyz[2] = oz;
    // quaternion_multiply(q_k, q) (general_utils.py:164-175), one rounding per op
    const float w1 = F.q[0], x1 = F.q[1], y1 = F.q[2], z1 = F.q[3];
    const float w2 = q.x, x2 = q.y, y2 = q.z, z2 = q.w;
    q = make_float4(fsub(fsub(fsub(fmul(w1, w2), fmul(x1, x2)), fmul(y1, y2)), fmul(z1, z2)),
                    fsub(fadd(fadd(fmul(w1, x2), fmul(x1, w2)), fmul(y1, z2)), fmul(z1, y2)),
                    fsub(fadd(fadd(fmul(w1, y2), fmul(y1, w2)), fmul(z1, x2)), fmul(x1, z2)),
                    fsub(fadd(fadd(fmul(w1, z2), fmul(z1, w2)), fmul(x1, y2)), fmul(y1, x2)));
  }
  reinterpret_cast<float4*>(bank.rotation)[i] = q;
  // replace_tensor_to_optimizer: zeroed moments (order: xyz 0, rotation 4, scaling 3)
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  reinterpret_cast<float4*>(bank.exp_avg[4])[i] = z4;
  reinterpret_cast<float4*>(bank.exp_avg_sq[4])[i] = z4;
  for (int c = 0; c < 3; ++c) {
    bank.exp_avg[0][3 * i + c] = 0.f;
    bank.exp_avg_sq[0][3 * i + c] = 0.f;
  }
  if (any_depth) {
    for (int c = 0; c < 3; ++c) {
      bank.exp_avg[3][3 * i + c] = 0.f;
      bank.exp_avg_sq[3][3 * i + c] = 0.f;
    }
  }
}

inline unsigned def_blocks(int64_t n) { return (unsigned)((n + kDefBlock - 1) / kDefBlock); }

}  // namespace

}  // namespace wgsr

using namespace wgsr;

extern "C" {

int wgsr_deform_points(int64_t P, const wgsr_gaussian_bank* bank, const wgsr_deform_frame* frames, int nframes,
                       const int32_t* lut, int lut_size, uint32_t* flags, void* stream) {
  if (P < 0 || nframes < 0 || lut_size < 0) return set_error(WGSR_EINVAL, "wgsr_deform_points: bad sizes");
  if (P == 0 || nframes == 0 || lut_size == 0) return WGSR_OK;
  if (!bank || !frames || !lut || !flags || !bank->xyz || !bank->rotation || !bank->scaling || !bank->kf_id)
    return set_error(WGSR_EINVAL, "wgsr_deform_points: null pointer");
  for (int k = 0; k < 5; ++k)
    if (!bank->exp_avg[k] || !bank->exp_avg_sq[k]) return set_error(WGSR_EINVAL, "wgsr_deform_points: null moments");
  const hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(flags, 0, 2 * sizeof(uint32_t), s);
  if (e != hipSuccess) return set_error(WGSR_EHIP, "wgsr_deform_points: %s", hipGetErrorString(e));
  hipLaunchKernelGGL(k_deform_any, dim3(def_blocks(P)), dim3(kDefBlock), 0, s, P, bank->kf_id, lut, lut_size, frames,
                     flags);
  hipLaunchKernelGGL(k_deform_apply, dim3(def_blocks(P)), dim3(kDefBlock), 0, s, P, *bank, lut, lut_size, frames,
                     (const uint32_t*)flags);
  e = hipGetLastError();
  if (e != hipSuccess) return set_error(WGSR_EHIP, "wgsr_deform_points: %s", hipGetErrorString(e));
  return WGSR_OK;
}

}  // extern "C"
