// PLY vertex records <-> the Gaussian SoA tensors on the device, gfx950
// (GaussianModel.save_ply / load_ply,
// thirdparty/gaussian_splatting/scene/gaussian_model.py:338-493).
//
// The file body is an array of P fixed-size records (binary_little_endian
// float32 properties: x y z nx ny nz f_dc_* f_rest_* opacity scale_* rot_*
// for the reference's writer, any order for the reader).  The reference
// builds it on the host with one Python tuple per Gaussian
// (gaussian_model.py:382, list(map(tuple, attributes))) and reads it back
// column by column into float64 arrays.  Here the records are assembled /
// taken apart on the device, so the host only moves one contiguous block
// between the file and HBM.
//
// Both kernels transpose through LDS: a workgroup owns 64 records; the
// record side is read / written as one contiguous run (coalesced) and each
// tensor's 64 rows likewise, with the column permutation applied in LDS.
// HBM bound: 2 x 4 x ncol bytes per Gaussian.
#include "wgsr_common.h"
#include "wgsr_internal.h"

namespace wgsr {

namespace {

constexpr int kRecsPerBlock = 64;

struct PlyMap {
  float* t[WGSR_PLY_MAX_TENSORS];
  int32_t tcols[WGSR_PLY_MAX_TENSORS];
  int32_t tstart[WGSR_PLY_MAX_TENSORS];  // offset of tensor i's columns in col[]
  int16_t col[WGSR_PLY_MAX_COLS];        // record column of each tensor column
  int32_t ntens, ncol;
};

__global__ __launch_bounds__(256) void k_ply_pack(PlyMap m, int64_t P, float* __restrict__ rec) {
  __shared__ float s[kRecsPerBlock * WGSR_PLY_MAX_COLS];
  const int64_t v0 = (int64_t)blockIdx.x * kRecsPerBlock;
  const int nv = (int)min<int64_t>(kRecsPerBlock, P - v0);
  const int n = nv * m.ncol;
  for (int i = threadIdx.x; i < n; i += 256) s[i] = 0.f;  // columns no tensor maps (normals)
  __syncthreads();
  for (int k = 0; k < m.ntens; ++k) {
    const int tc = m.tcols[k];
    const float* src = m.t[k] + v0 * tc;
    const int16_t* col = m.col + m.tstart[k];
    for (int i = threadIdx.x; i < nv * tc; i += 256) {
      const int v = i / tc, c = i - v * tc;
      s[v * m.ncol + col[c]] = src[i];
    }
  }
  __syncthreads();
  float* dst = rec + v0 * m.ncol;
  for (int i = threadIdx.x; i < n; i += 256) dst[i] = s[i];
}

__global__ __launch_bounds__(256) void k_ply_unpack(PlyMap m, int64_t P, const float* __restrict__ rec) {
  __shared__ float s[kRecsPerBlock * WGSR_PLY_MAX_COLS];
  const int64_t v0 = (int64_t)blockIdx.x * kRecsPerBlock;
  const int nv = (int)min<int64_t>(kRecsPerBlock, P - v0);
  const int n = nv * m.ncol;
  const float* src = rec + v0 * m.ncol;
  for (int i = threadIdx.x; i < n; i += 256) s[i] = src[i];
  __syncthreads();
  for (int k = 0; k < m.ntens; ++k) {
    const int tc = m.tcols[k];
    float* dst = m.t[k] + v0 * tc;
    const int16_t* col = m.col + m.tstart[k];
    for (int i = threadIdx.x; i < nv * tc; i += 256) {
      const int v = i / tc, c = i - v * tc;
      dst[i] = s[v * m.ncol + col[c]];
    }
  }
}

int build_map(const wgsr_ply_column_set* sets, int ntens, int ncol, PlyMap& m, const char* who) {
  if (ntens < 1 || ntens > WGSR_PLY_MAX_TENSORS || ncol < 1 || ncol > WGSR_PLY_MAX_COLS)
    return set_error(WGSR_EINVAL, "%s: 1..%d tensors and 1..%d record columns", who, WGSR_PLY_MAX_TENSORS,
                     WGSR_PLY_MAX_COLS);
  m = PlyMap{};
  m.ntens = ntens;
  m.ncol = ncol;
  int used = 0;
  for (int k = 0; k < ntens; ++k) {
    const wgsr_ply_column_set& cs = sets[k];
    if (!cs.data || cs.cols < 1 || used + cs.cols > WGSR_PLY_MAX_COLS || !cs.record_col)
      return set_error(WGSR_EINVAL, "%s: tensor %d has no data / columns", who, k);
    m.t[k] = cs.data;
    m.tcols[k] = cs.cols;
    m.tstart[k] = used;
    for (int c = 0; c < cs.cols; ++c) {
      const int rc = cs.record_col[c];
      if (rc < 0 || rc >= ncol) return set_error(WGSR_EINVAL, "%s: tensor %d column %d maps outside the record", who, k, c);
      m.col[used + c] = (int16_t)rc;
    }
    used += cs.cols;
  }
  return WGSR_OK;
}

}  // namespace

}  // namespace wgsr

using namespace wgsr;

extern "C" {

int wgsr_ply_pack(const wgsr_ply_column_set* sets, int ntens, int64_t P, int ncol, float* records, void* stream) {
  if (P < 0) return set_error(WGSR_EINVAL, "wgsr_ply_pack: negative P");
  PlyMap m;
  const int rc = build_map(sets, ntens, ncol, m, "wgsr_ply_pack");
  if (rc != WGSR_OK) return rc;
  if (P == 0) return WGSR_OK;
  if (!records) return set_error(WGSR_EINVAL, "wgsr_ply_pack: null records");
  hipLaunchKernelGGL(k_ply_pack, dim3((unsigned)((P + kRecsPerBlock - 1) / kRecsPerBlock)), dim3(256), 0,
                     (hipStream_t)stream, m, P, records);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? WGSR_OK : set_error(WGSR_EHIP, "wgsr_ply_pack: %s", hipGetErrorString(e));
}

int wgsr_ply_unpack(const float* records, int64_t P, int ncol, const wgsr_ply_column_set* sets, int ntens,
                    void* stream) {
  if (P < 0) return set_error(WGSR_EINVAL, "wgsr_ply_unpack: negative P");
  PlyMap m;
  const int rc = build_map(sets, ntens, ncol, m, "wgsr_ply_unpack");
  if (rc != WGSR_OK) return rc;
  if (P == 0) return WGSR_OK;
  if (!records) return set_error(WGSR_EINVAL, "wgsr_ply_unpack: null records");
  hipLaunchKernelGGL(k_ply_unpack, dim3((unsigned)((P + kRecsPerBlock - 1) / kRecsPerBlock)), dim3(256), 0,
                     (hipStream_t)stream, m, P, records);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? WGSR_OK : set_error(WGSR_EHIP, "wgsr_ply_unpack: %s", hipGetErrorString(e));
}

}  // extern "C"
