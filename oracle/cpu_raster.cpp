// ORACLE (test infrastructure only) -- fp32 tile-based CPU restatement of the
// diff-gaussian-rasterization-w-pose forward/backward and simple-knn distCUDA2.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
// this library, and only as the checker / timed CPU baseline; the product path
// (wildgs-slam-blackwell_amd/) never links it.
//
// The CUDA sources it restates are NOT in the reference snapshot
// (thirdparty/diff-gaussian-rasterization-w-pose and thirdparty/simple-knn are
// empty gitlinks, .gitmodules:7-12).  The algorithm follows SURVEY.md
// Appendix A (rasteriser) and Appendix B (distCUDA2); formulas keep the upstream
// operation order where it is known.  This restatement is itself checked
// against the float64 autograd oracle (oracle/dense.py) in tests/.
//
// Callers: gaussian_renderer/__init__.py:130-141 (rasteriser) and
// scene/gaussian_model.py:201-207 (distCUDA2).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <vector>
#include <omp.h>

namespace {

constexpr int BX = 16, BY = 16;
constexpr float SH_C0 = 0.28209479177387814f;
constexpr float SH_C1 = 0.4886025119029199f;
constexpr float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                            -1.0925484305920792f, 0.5462742152960396f};
constexpr float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                            0.3731763325901154f,  -0.4570457994644658f, 1.445305721320277f,
                            -0.5900435899266435f};

struct V3 { float x, y, z; };
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator*(float s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }

// column-major 4x4 storage of the row-vector matrices the caller passes
// (world_view_transform / full_proj_transform, camera_utils.py:137-147).
inline V3 xform43(const float* m, V3 p) {
  return {m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
          m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]};
}
inline void xform44(const float* m, V3 p, float out[4]) {
  out[0] = m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12];
  out[1] = m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13];
  out[2] = m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14];
  out[3] = m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15];
}
inline float ndc2pix(float v, int S) { return (float)(((v + 1.0) * S - 1.0) * 0.5); }

// Standard rotation of q = (w, x, y, z), not re-normalised (A.2 step 3).
inline void quat_rot(const float* q, float R[3][3]) {
  float r = q[0], x = q[1], y = q[2], z = q[3];
  R[0][0] = 1.f - 2.f * (y * y + z * z); R[0][1] = 2.f * (x * y - r * z); R[0][2] = 2.f * (x * z + r * y);
  R[1][0] = 2.f * (x * y + r * z); R[1][1] = 1.f - 2.f * (x * x + z * z); R[1][2] = 2.f * (y * z - r * x);
  R[2][0] = 2.f * (x * z - r * y); R[2][1] = 2.f * (y * z + r * x); R[2][2] = 1.f - 2.f * (x * x + y * y);
}

inline void cov3d(const float* s, float mod, const float* q, float out[6]) {
  float R[3][3];
  quat_rot(q, R);
  float sx = mod * s[0], sy = mod * s[1], sz = mod * s[2];
  float s2[3] = {sx * sx, sy * sy, sz * sz};
  // Sigma = R diag(s^2) R^T
  int idx = 0;
  for (int i = 0; i < 3; ++i)
    for (int j = i; j < 3; ++j) {
      float acc = 0.f;
      for (int k = 0; k < 3; ++k) acc += R[i][k] * s2[k] * R[j][k];
      out[idx++] = acc;
    }
}

inline void sym3(const float* c6, float S[3][3]) {
  S[0][0] = c6[0]; S[0][1] = c6[1]; S[0][2] = c6[2];
  S[1][0] = c6[1]; S[1][1] = c6[3]; S[1][2] = c6[4];
  S[2][0] = c6[2]; S[2][1] = c6[4]; S[2][2] = c6[5];
}

struct Cam {
  int W, H;
  float tanx, tany, fx, fy;
  const float* view;   // 16
  const float* proj;   // 16
  const float* praw;   // 16
  V3 campos;
  float Rw[3][3];      // world->camera rotation (row-major math)
};

inline void cam_init(Cam& c) {
  for (int r = 0; r < 3; ++r)
    for (int k = 0; k < 3; ++k) c.Rw[r][k] = c.view[4 * k + r];
}

// T = J Rw (2x3) and the clamped camera-space mean.
inline void ewa_T(const Cam& c, V3 t, float T[2][3], V3& tc, float& xmul, float& ymul) {
  const float limx = 1.3f * c.tanx, limy = 1.3f * c.tany;
  const float txtz = t.x / t.z, tytz = t.y / t.z;
  tc = {std::min(limx, std::max(-limx, txtz)) * t.z, std::min(limy, std::max(-limy, tytz)) * t.z, t.z};
  xmul = (txtz < -limx || txtz > limx) ? 0.f : 1.f;
  ymul = (tytz < -limy || tytz > limy) ? 0.f : 1.f;
  float J00 = c.fx / tc.z, J02 = -(c.fx * tc.x) / (tc.z * tc.z);
  float J11 = c.fy / tc.z, J12 = -(c.fy * tc.y) / (tc.z * tc.z);
  for (int k = 0; k < 3; ++k) {
    T[0][k] = J00 * c.Rw[0][k] + J02 * c.Rw[2][k];
    T[1][k] = J11 * c.Rw[1][k] + J12 * c.Rw[2][k];
  }
}

inline void cov2d(const float T[2][3], const float S[3][3], float& a, float& b, float& cc) {
  float ST0[3], ST1[3];
  for (int i = 0; i < 3; ++i) {
    ST0[i] = S[i][0] * T[0][0] + S[i][1] * T[0][1] + S[i][2] * T[0][2];
    ST1[i] = S[i][0] * T[1][0] + S[i][1] * T[1][1] + S[i][2] * T[1][2];
  }
  a = T[0][0] * ST0[0] + T[0][1] * ST0[1] + T[0][2] * ST0[2] + 0.3f;
  b = T[0][0] * ST1[0] + T[0][1] * ST1[1] + T[0][2] * ST1[2];
  cc = T[1][0] * ST1[0] + T[1][1] * ST1[1] + T[1][2] * ST1[2] + 0.3f;
}

inline V3 sh_color(int deg, int M, const float* sh, V3 dir, bool clamped[3]) {
  const float* s = sh;
  auto C = [&](int k) { return V3{s[3 * k], s[3 * k + 1], s[3 * k + 2]}; };
  V3 r = SH_C0 * C(0);
  if (deg > 0) {
    float x = dir.x, y = dir.y, z = dir.z;
    r = r - (SH_C1 * y) * C(1) + (SH_C1 * z) * C(2) - (SH_C1 * x) * C(3);
    if (deg > 1) {
      float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
      r = r + (SH_C2[0] * xy) * C(4) + (SH_C2[1] * yz) * C(5) + (SH_C2[2] * (2.f * zz - xx - yy)) * C(6) +
          (SH_C2[3] * xz) * C(7) + (SH_C2[4] * (xx - yy)) * C(8);
      if (deg > 2) {
        r = r + (SH_C3[0] * y * (3.f * xx - yy)) * C(9) + (SH_C3[1] * xy * z) * C(10) +
            (SH_C3[2] * y * (4.f * zz - xx - yy)) * C(11) + (SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy)) * C(12) +
            (SH_C3[4] * x * (4.f * zz - xx - yy)) * C(13) + (SH_C3[5] * z * (xx - yy)) * C(14) +
            (SH_C3[6] * x * (xx - 3.f * yy)) * C(15);
      }
    }
  }
  (void)M;
  r = r + V3{0.5f, 0.5f, 0.5f};
  clamped[0] = r.x < 0; clamped[1] = r.y < 0; clamped[2] = r.z < 0;
  return {std::max(r.x, 0.f), std::max(r.y, 0.f), std::max(r.z, 0.f)};
}

// dL/dsh and dL/dmean through the view direction (upstream computeColorFromSH bwd).
inline V3 sh_backward(int deg, const float* sh, V3 pos, V3 campos, const bool clamped[3], V3 dL_dRGB, float* dsh) {
  V3 dir_orig = pos - campos;
  float len = std::sqrt(dot(dir_orig, dir_orig));
  V3 dir{dir_orig.x / len, dir_orig.y / len, dir_orig.z / len};
  auto C = [&](int k) { return V3{sh[3 * k], sh[3 * k + 1], sh[3 * k + 2]}; };
  auto put = [&](int k, float w) { dsh[3 * k] = w * dL_dRGB.x; dsh[3 * k + 1] = w * dL_dRGB.y; dsh[3 * k + 2] = w * dL_dRGB.z; };
  dL_dRGB.x *= clamped[0] ? 0.f : 1.f;
  dL_dRGB.y *= clamped[1] ? 0.f : 1.f;
  dL_dRGB.z *= clamped[2] ? 0.f : 1.f;
  V3 dx{0, 0, 0}, dy{0, 0, 0}, dz{0, 0, 0};
  float x = dir.x, y = dir.y, z = dir.z;
  put(0, SH_C0);
  if (deg > 0) {
    put(1, -SH_C1 * y); put(2, SH_C1 * z); put(3, -SH_C1 * x);
    dx = (-SH_C1) * C(3); dy = (-SH_C1) * C(1); dz = SH_C1 * C(2);
    if (deg > 1) {
      float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
      put(4, SH_C2[0] * xy); put(5, SH_C2[1] * yz); put(6, SH_C2[2] * (2.f * zz - xx - yy));
      put(7, SH_C2[3] * xz); put(8, SH_C2[4] * (xx - yy));
      dx = dx + (SH_C2[0] * y) * C(4) + (SH_C2[2] * 2.f * -x) * C(6) + (SH_C2[3] * z) * C(7) + (SH_C2[4] * 2.f * x) * C(8);
      dy = dy + (SH_C2[0] * x) * C(4) + (SH_C2[1] * z) * C(5) + (SH_C2[2] * 2.f * -y) * C(6) + (SH_C2[4] * 2.f * -y) * C(8);
      dz = dz + (SH_C2[1] * y) * C(5) + (SH_C2[2] * 2.f * 2.f * z) * C(6) + (SH_C2[3] * x) * C(7);
      if (deg > 2) {
        put(9, SH_C3[0] * y * (3.f * xx - yy)); put(10, SH_C3[1] * xy * z);
        put(11, SH_C3[2] * y * (4.f * zz - xx - yy)); put(12, SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy));
        put(13, SH_C3[4] * x * (4.f * zz - xx - yy)); put(14, SH_C3[5] * z * (xx - yy));
        put(15, SH_C3[6] * x * (xx - 3.f * yy));
        dx = dx + (SH_C3[0] * 3.f * 2.f * xy) * C(9) + (SH_C3[1] * yz) * C(10) + (SH_C3[2] * -2.f * xy) * C(11) +
             (SH_C3[3] * -3.f * 2.f * xz) * C(12) + (SH_C3[4] * (-3.f * xx + 4.f * zz - yy)) * C(13) +
             (SH_C3[5] * 2.f * xz) * C(14) + (SH_C3[6] * 3.f * (xx - yy)) * C(15);
        dy = dy + (SH_C3[0] * 3.f * (xx - yy)) * C(9) + (SH_C3[1] * xz) * C(10) +
             (SH_C3[2] * (-3.f * yy + 4.f * zz - xx)) * C(11) + (SH_C3[3] * -3.f * 2.f * yz) * C(12) +
             (SH_C3[4] * -2.f * xy) * C(13) + (SH_C3[5] * -2.f * yz) * C(14) + (SH_C3[6] * -3.f * 2.f * xy) * C(15);
        dz = dz + (SH_C3[1] * xy) * C(10) + (SH_C3[2] * 4.f * 2.f * yz) * C(11) +
             (SH_C3[3] * 3.f * (2.f * zz - xx - yy)) * C(12) + (SH_C3[4] * 4.f * 2.f * xz) * C(13) +
             (SH_C3[5] * (xx - yy)) * C(14);
      }
    }
  }
  V3 dL_ddir{dot(dx, dL_dRGB), dot(dy, dL_dRGB), dot(dz, dL_dRGB)};
  // d normalize(v)/dv
  V3 v = dir_orig;
  float sum2 = dot(v, v);
  float invsum32 = 1.0f / std::sqrt(sum2 * sum2 * sum2);
  return {((sum2 - v.x * v.x) * dL_ddir.x - v.y * v.x * dL_ddir.y - v.z * v.x * dL_ddir.z) * invsum32,
          (-v.x * v.y * dL_ddir.x + (sum2 - v.y * v.y) * dL_ddir.y - v.z * v.y * dL_ddir.z) * invsum32,
          (-v.x * v.z * dL_ddir.x - v.y * v.z * dL_ddir.y + (sum2 - v.z * v.z) * dL_ddir.z) * invsum32};
}

struct State {
  int P, D, M, W, H, gx, gy;
  bool has_sh, has_cov, has_colors;
  Cam cam;
  float scale_mod;
  const float *bg, *means, *colors, *opac, *scales, *rots, *cov_pre, *sh;
  std::vector<float> xy, depth, conic_o, rgb, cov;   // per Gaussian
  std::vector<uint8_t> clamped;
  std::vector<int> radii;
  std::vector<uint32_t> tiles;
  std::vector<int> rect;                 // 4 per Gaussian
  std::vector<uint32_t> order;           // visible Gaussians by (depth, id)
  std::vector<uint64_t> slot_off;        // per depth rank: first slot
  std::vector<uint32_t> tile_start;      // ntiles + 1
  std::vector<uint32_t> list;            // sorted entry -> Gaussian id
  std::vector<uint32_t> slot_pos;        // pre-sort slot -> sorted entry
  std::vector<float> final_T;
  std::vector<uint32_t> n_contrib;
  size_t N = 0;
};

}  // namespace

extern "C" {

// Forward.  Output arrays are caller-owned; `state` must be released with
// cr_free.  Arguments mirror _C.rasterize_gaussians.
void* cr_forward(int P, int D, int M, const float* bg, const float* means3D, const float* colors,
                 const float* opacity, const float* scales, const float* rotations, float scale_modifier,
                 const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                 const float* projmatrix_raw, float tan_fovx, float tan_fovy, int H, int W, const float* sh,
                 const float* campos, float* out_color, float* out_depth, float* out_opacity, int* radii,
                 int* n_touched, long long* num_rendered, int* n_touched_firm, int* n_touched_soft) {
  State* s = new State();
  s->P = P; s->D = D; s->M = M; s->W = W; s->H = H;
  s->gx = (W + BX - 1) / BX; s->gy = (H + BY - 1) / BY;
  s->has_sh = sh != nullptr; s->has_cov = cov3D_precomp != nullptr; s->has_colors = colors != nullptr;
  s->cam = Cam{W, H, tan_fovx, tan_fovy, W / (2.0f * tan_fovx), H / (2.0f * tan_fovy),
               viewmatrix, projmatrix, projmatrix_raw, V3{campos[0], campos[1], campos[2]}, {}};
  cam_init(s->cam);
  s->scale_mod = scale_modifier;
  s->bg = bg; s->means = means3D; s->colors = colors; s->opac = opacity; s->scales = scales; s->rots = rotations;
  s->cov_pre = cov3D_precomp; s->sh = sh;
  s->xy.assign(2 * (size_t)P, 0.f); s->depth.assign(P, 0.f); s->conic_o.assign(4 * (size_t)P, 0.f);
  s->rgb.assign(3 * (size_t)P, 0.f); s->cov.assign(6 * (size_t)P, 0.f); s->clamped.assign(3 * (size_t)P, 0);
  s->radii.assign(P, 0); s->tiles.assign(P, 0); s->rect.assign(4 * (size_t)P, 0);
  const Cam& c = s->cam;
  const int gx = s->gx, gy = s->gy;

  // ---- preprocess (A.2)
#pragma omp parallel for schedule(static)
  for (int i = 0; i < P; ++i) {
    V3 p{means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]};
    float hom[4];
    xform44(c.proj, p, hom);
    float pw = 1.0f / (hom[3] + 0.0000001f);
    V3 pproj{hom[0] * pw, hom[1] * pw, hom[2] * pw};
    V3 pv = xform43(c.view, p);
    if (pv.z <= 0.2f) continue;
    float* cv = &s->cov[6 * (size_t)i];
    if (cov3D_precomp) std::memcpy(cv, cov3D_precomp + 6 * (size_t)i, 6 * sizeof(float));
    else cov3d(scales + 3 * (size_t)i, scale_modifier, rotations + 4 * (size_t)i, cv);
    float S[3][3]; sym3(cv, S);
    float T[2][3]; V3 tc; float xm, ym;
    ewa_T(c, pv, T, tc, xm, ym);
    float a, b, cc;
    cov2d(T, S, a, b, cc);
    float det = a * cc - b * b;
    if (det == 0.0f) continue;
    float det_inv = 1.f / det;
    float mid = 0.5f * (a + cc);
    float l1 = mid + std::sqrt(std::max(0.1f, mid * mid - det));
    float l2 = mid - std::sqrt(std::max(0.1f, mid * mid - det));
    float my_radius = std::ceil(3.f * std::sqrt(std::max(l1, l2)));
    float px = ndc2pix(pproj.x, W), py = ndc2pix(pproj.y, H);
    int r = (int)my_radius;
    int x0 = std::min(gx, std::max(0, (int)((px - r) / BX)));
    int y0 = std::min(gy, std::max(0, (int)((py - r) / BY)));
    int x1 = std::min(gx, std::max(0, (int)((px + r + BX - 1) / BX)));
    int y1 = std::min(gy, std::max(0, (int)((py + r + BY - 1) / BY)));
    if ((x1 - x0) * (y1 - y0) == 0) continue;
    if (!colors) {
      bool cl[3];
      V3 dir = p - c.campos;
      float len = std::sqrt(dot(dir, dir));
      dir = V3{dir.x / len, dir.y / len, dir.z / len};
      V3 col = sh_color(D, M, sh + 3 * (size_t)M * i, dir, cl);
      s->rgb[3 * i] = col.x; s->rgb[3 * i + 1] = col.y; s->rgb[3 * i + 2] = col.z;
      for (int k = 0; k < 3; ++k) s->clamped[3 * i + k] = cl[k];
    } else {
      for (int k = 0; k < 3; ++k) s->rgb[3 * i + k] = colors[3 * i + k];
    }
    s->depth[i] = pv.z;
    s->radii[i] = r;
    s->xy[2 * i] = px; s->xy[2 * i + 1] = py;
    s->conic_o[4 * i] = cc * det_inv; s->conic_o[4 * i + 1] = -b * det_inv;
    s->conic_o[4 * i + 2] = a * det_inv; s->conic_o[4 * i + 3] = opacity[i];
    s->tiles[i] = (uint32_t)((x1 - x0) * (y1 - y0));
    int* rc = &s->rect[4 * (size_t)i];
    rc[0] = x0; rc[1] = y0; rc[2] = x1; rc[3] = y1;
  }

  // ---- binning: depth order (stable by id), then a stable tile scatter.
  for (int i = 0; i < P; ++i) if (s->tiles[i]) s->order.push_back(i);
  std::stable_sort(s->order.begin(), s->order.end(), [&](uint32_t a, uint32_t b) {
    uint32_t ka, kb;
    std::memcpy(&ka, &s->depth[a], 4); std::memcpy(&kb, &s->depth[b], 4);
    return ka < kb;
  });
  const size_t V = s->order.size();
  s->slot_off.assign(V + 1, 0);
  for (size_t r = 0; r < V; ++r) s->slot_off[r + 1] = s->slot_off[r] + s->tiles[s->order[r]];
  const size_t N = s->slot_off[V];
  s->N = N;
  const int ntiles = gx * gy;
  const int nt = omp_get_max_threads();
  std::vector<uint32_t> cnt((size_t)nt * ntiles, 0);
  auto chunk = [&](int t, size_t& b, size_t& e) { b = V * t / nt; e = V * (t + 1) / nt; };
#pragma omp parallel num_threads(nt)
  {
    int t = omp_get_thread_num();
    size_t b, e; chunk(t, b, e);
    uint32_t* my = &cnt[(size_t)t * ntiles];
    for (size_t r = b; r < e; ++r) {
      const int* rc = &s->rect[4 * (size_t)s->order[r]];
      for (int y = rc[1]; y < rc[3]; ++y)
        for (int x = rc[0]; x < rc[2]; ++x) my[y * gx + x]++;
    }
  }
  s->tile_start.assign(ntiles + 1, 0);
  {
    uint32_t run = 0;
    for (int tl = 0; tl < ntiles; ++tl) {
      s->tile_start[tl] = run;
      for (int t = 0; t < nt; ++t) {
        uint32_t v = cnt[(size_t)t * ntiles + tl];
        cnt[(size_t)t * ntiles + tl] = run;
        run += v;
      }
    }
    s->tile_start[ntiles] = run;
  }
  s->list.assign(N, 0);
  s->slot_pos.assign(N, 0);
#pragma omp parallel num_threads(nt)
  {
    int t = omp_get_thread_num();
    size_t b, e; chunk(t, b, e);
    uint32_t* my = &cnt[(size_t)t * ntiles];
    for (size_t r = b; r < e; ++r) {
      uint32_t g = s->order[r];
      const int* rc = &s->rect[4 * (size_t)g];
      size_t k = s->slot_off[r];
      for (int y = rc[1]; y < rc[3]; ++y)
        for (int x = rc[0]; x < rc[2]; ++x, ++k) {
          uint32_t pos = my[y * gx + x]++;
          s->list[pos] = g;
          s->slot_pos[k] = pos;
        }
    }
  }

  // ---- render (A.3)
  s->final_T.assign((size_t)W * H, 0.f);
  s->n_contrib.assign((size_t)W * H, 0);
  std::vector<int> touched(P, 0), firm(P, 0), soft(P, 0);
  // n_touched counts blends with T > 0.5 after the blend.  Besides the plain
  // count, each decision is classified: FIRM when the oracle's T is away from
  // 0.5 by more than the slack rounding could explain, SOFT otherwise.  The
  // slack starts at 1e-5 (relative) and grows by the opacity of every entry
  // whose inclusion itself sits on a threshold (power ~ 0, alpha ~ 1/255):
  // another exp() rounding may include or skip it, moving T by that factor.
  // Such an ambiguous entry is a SOFT candidate itself.  A correct
  // implementation therefore has firm <= n_touched <= firm + soft, and equals
  // the oracle exactly wherever soft == 0 (then n_touched == firm).
#pragma omp parallel
  {
#pragma omp for schedule(dynamic, 4)
    for (int tl = 0; tl < ntiles; ++tl) {
      int tx = tl % gx, ty = tl / gx;
      uint32_t b = s->tile_start[tl], e = s->tile_start[tl + 1];
      for (int py = ty * BY; py < std::min(H, ty * BY + BY); ++py)
        for (int px = tx * BX; px < std::min(W, tx * BX + BX); ++px) {
          float T = 1.f, C[3] = {0, 0, 0}, Dp = 0.f;
          float slack = 1e-5f;
          uint32_t contributor = 0, last = 0;
          for (uint32_t j = b; j < e; ++j) {
            contributor++;
            uint32_t g = s->list[j];
            float dx = s->xy[2 * g] - (float)px, dy = s->xy[2 * g + 1] - (float)py;
            const float* co = &s->conic_o[4 * (size_t)g];
            float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
            float a_any = std::min(0.99f, co[3] * std::exp(std::min(power, 0.0f)));
            bool amb = std::fabs(power) < 1e-5f ||
                       std::fabs(a_any - 1.0f / 255.0f) <= 1e-4f * (1.0f / 255.0f);
            if (amb) {
              slack += std::max(a_any, 1.0f / 255.0f);
              if (T * (1 - a_any) > 0.5f * (1.0f - 1.02f * slack)) {
#pragma omp atomic
                soft[g]++;
              }
            }
            if (power > 0.0f) continue;
            float alpha = std::min(0.99f, co[3] * std::exp(power));
            if (alpha < 1.0f / 255.0f) continue;
            float test_T = T * (1 - alpha);
            if (test_T < 0.0001f) break;
            for (int ch = 0; ch < 3; ++ch) C[ch] += s->rgb[3 * g + ch] * alpha * T;
            Dp += s->depth[g] * alpha * T;
            if (test_T > 0.5f) {
#pragma omp atomic
              touched[g]++;
            }
            if (!amb) {
              if (std::fabs(test_T - 0.5f) <= 0.5f * 1.02f * slack) {
#pragma omp atomic
                soft[g]++;
              } else if (test_T > 0.5f) {
#pragma omp atomic
                firm[g]++;
              }
            }
            T = test_T;
            last = contributor;
          }
          size_t pid = (size_t)py * W + px;
          s->final_T[pid] = T;
          s->n_contrib[pid] = last;
          for (int ch = 0; ch < 3; ++ch) out_color[ch * (size_t)H * W + pid] = C[ch] + T * bg[ch];
          out_depth[pid] = Dp;
          out_opacity[pid] = 1 - T;
        }
    }
  }
  for (int i = 0; i < P; ++i) { radii[i] = s->radii[i]; n_touched[i] = touched[i]; }
  if (n_touched_firm)
    for (int i = 0; i < P; ++i) n_touched_firm[i] = firm[i];
  if (n_touched_soft)
    for (int i = 0; i < P; ++i) n_touched_soft[i] = soft[i];
  *num_rendered = (long long)N;
  return s;
}

// Backward.  Output arrays are caller-owned and fully written (zeros for
// culled Gaussians).  Layout = _C.rasterize_gaussians_backward's outputs.
void cr_backward(void* handle, const float* dL_dpix, const float* dL_ddepth_pix, float* dL_dmeans2D,
                 float* dL_dcolors, float* dL_dopacity, float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh,
                 float* dL_dscales, float* dL_drot, float* dL_dtau) {
  State* s = (State*)handle;
  const int P = s->P, W = s->W, H = s->H, gx = s->gx;
  const int ntiles = gx * s->gy;
  const Cam& c = s->cam;
  // per sorted entry partials: dmean2D.xy, dconic.xyw, dopacity, dcolor rgb, ddepth
  std::vector<float> part(10 * s->N, 0.f);
  const float ddelx_dx = 0.5f * W, ddely_dy = 0.5f * H;
#pragma omp parallel for schedule(dynamic, 4)
  for (int tl = 0; tl < ntiles; ++tl) {
    int tx = tl % gx, ty = tl / gx;
    uint32_t b = s->tile_start[tl], e = s->tile_start[tl + 1];
    for (int py = ty * BY; py < std::min(H, ty * BY + BY); ++py)
      for (int px = tx * BX; px < std::min(W, tx * BX + BX); ++px) {
        size_t pid = (size_t)py * W + px;
        const float T_final = s->final_T[pid];
        float T = T_final;
        const uint32_t last = s->n_contrib[pid];
        float dpix[3] = {dL_dpix[pid], dL_dpix[(size_t)H * W + pid], dL_dpix[2 * (size_t)H * W + pid]};
        float dpd = dL_ddepth_pix[pid];
        float acc[3] = {0, 0, 0}, acc_d = 0.f, last_alpha = 0.f, last_c[3] = {0, 0, 0}, last_d = 0.f;
        float bg_dot = s->bg[0] * dpix[0] + s->bg[1] * dpix[1] + s->bg[2] * dpix[2];
        for (uint32_t jj = std::min<uint32_t>(e - b, last); jj-- > 0;) {
          uint32_t j = b + jj;
          uint32_t g = s->list[j];
          float dx = s->xy[2 * g] - (float)px, dy = s->xy[2 * g + 1] - (float)py;
          const float* co = &s->conic_o[4 * (size_t)g];
          float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
          if (power > 0.0f) continue;
          float G = std::exp(power);
          float alpha = std::min(0.99f, co[3] * G);
          if (alpha < 1.0f / 255.0f) continue;
          T = T / (1.f - alpha);
          float w = alpha * T;
          float dL_dalpha = 0.f;
          float* pp = &part[10 * (size_t)j];
          for (int ch = 0; ch < 3; ++ch) {
            float col = s->rgb[3 * g + ch];
            acc[ch] = last_alpha * last_c[ch] + (1.f - last_alpha) * acc[ch];
            last_c[ch] = col;
            dL_dalpha += (col - acc[ch]) * dpix[ch];
            pp[6 + ch] += w * dpix[ch];
          }
          float cd = s->depth[g];
          acc_d = last_alpha * last_d + (1.f - last_alpha) * acc_d;
          last_d = cd;
          dL_dalpha += (cd - acc_d) * dpd;
          pp[9] += w * dpd;
          dL_dalpha *= T;
          last_alpha = alpha;
          dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
          float dL_dG = co[3] * dL_dalpha;
          float gdx = G * dx, gdy = G * dy;
          float dG_ddelx = -gdx * co[0] - gdy * co[1];
          float dG_ddely = -gdy * co[2] - gdx * co[1];
          pp[0] += dL_dG * dG_ddelx * ddelx_dx;
          pp[1] += dL_dG * dG_ddely * ddely_dy;
          pp[2] += -0.5f * gdx * dx * dL_dG;
          pp[3] += -0.5f * gdx * dy * dL_dG;
          pp[4] += -0.5f * gdy * dy * dL_dG;
          pp[5] += G * dL_dalpha;
        }
      }
  }

  const size_t V = s->order.size();
  std::vector<int> rank_of(P, -1);
  for (size_t r = 0; r < V; ++r) rank_of[s->order[r]] = (int)r;
  const int M = s->M, D = s->D;
#pragma omp parallel for schedule(static)
  for (int i = 0; i < P; ++i) {
    float* o2 = dL_dmeans2D + 3 * (size_t)i;
    float* ocol = dL_dcolors + 3 * (size_t)i;
    float* om = dL_dmeans3D + 3 * (size_t)i;
    float* ocov = dL_dcov3D + 6 * (size_t)i;
    float* osc = dL_dscales ? dL_dscales + 3 * (size_t)i : nullptr;
    float* orot = dL_drot ? dL_drot + 4 * (size_t)i : nullptr;
    float* otau = dL_dtau + 6 * (size_t)i;
    float* osh = dL_dsh ? dL_dsh + 3 * (size_t)M * i : nullptr;
    for (int k = 0; k < 3; ++k) { o2[k] = 0; ocol[k] = 0; om[k] = 0; if (osc) osc[k] = 0; }
    for (int k = 0; k < 6; ++k) { ocov[k] = 0; otau[k] = 0; }
    if (orot) for (int k = 0; k < 4; ++k) orot[k] = 0;
    if (osh) for (int k = 0; k < 3 * M; ++k) osh[k] = 0;
    dL_dopacity[i] = 0;
    if (!(s->radii[i] > 0)) continue;
    // reduce this Gaussian's per-entry partials in slot order
    float g[10] = {0};
    int r = rank_of[i];
    for (uint64_t k = s->slot_off[r]; k < s->slot_off[r + 1]; ++k) {
      const float* pp = &part[10 * (size_t)s->slot_pos[k]];
      for (int q = 0; q < 10; ++q) g[q] += pp[q];
    }
    o2[0] = g[0]; o2[1] = g[1];
    dL_dopacity[i] = g[5];
    ocol[0] = g[6]; ocol[1] = g[7]; ocol[2] = g[8];
    const float dcx = g[2], dcy = g[3], dcw = g[4], ddepth = g[9];

    // ---- computeCov2D backward
    V3 mean{s->means[3 * i], s->means[3 * i + 1], s->means[3 * i + 2]};
    V3 t = xform43(c.view, mean);
    const float* cv = &s->cov[6 * (size_t)i];
    float S[3][3]; sym3(cv, S);
    float T[2][3]; V3 tc; float xm, ym;
    ewa_T(c, t, T, tc, xm, ym);
    float a, b, cc;
    cov2d(T, S, a, b, cc);
    float denom = a * cc - b * b;
    float dL_da = 0, dL_db = 0, dL_dc = 0;
    float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    if (denom2inv != 0) {
      dL_da = denom2inv * (-cc * cc * dcx + 2 * b * cc * dcy + (denom - a * cc) * dcw);
      dL_dc = denom2inv * (-a * a * dcw + 2 * a * b * dcy + (denom - a * cc) * dcx);
      dL_db = denom2inv * 2 * (b * cc * dcx - (denom + 2 * b * b) * dcy + a * b * dcw);
      // diagonal
      ocov[0] = T[0][0] * T[0][0] * dL_da + T[0][0] * T[1][0] * dL_db + T[1][0] * T[1][0] * dL_dc;
      ocov[3] = T[0][1] * T[0][1] * dL_da + T[0][1] * T[1][1] * dL_db + T[1][1] * T[1][1] * dL_dc;
      ocov[5] = T[0][2] * T[0][2] * dL_da + T[0][2] * T[1][2] * dL_db + T[1][2] * T[1][2] * dL_dc;
      // off-diagonal (appears twice)
      ocov[1] = 2 * T[0][0] * T[0][1] * dL_da + (T[0][0] * T[1][1] + T[0][1] * T[1][0]) * dL_db + 2 * T[1][0] * T[1][1] * dL_dc;
      ocov[2] = 2 * T[0][0] * T[0][2] * dL_da + (T[0][0] * T[1][2] + T[0][2] * T[1][0]) * dL_db + 2 * T[1][0] * T[1][2] * dL_dc;
      ocov[4] = 2 * T[0][2] * T[0][1] * dL_da + (T[0][1] * T[1][2] + T[0][2] * T[1][1]) * dL_db + 2 * T[1][1] * T[1][2] * dL_dc;
    }
    float dT[2][3];
    for (int k = 0; k < 3; ++k) {
      float s0 = T[0][0] * S[k][0] + T[0][1] * S[k][1] + T[0][2] * S[k][2];
      float s1 = T[1][0] * S[k][0] + T[1][1] * S[k][1] + T[1][2] * S[k][2];
      dT[0][k] = 2 * s0 * dL_da + s1 * dL_db;
      dT[1][k] = 2 * s1 * dL_dc + s0 * dL_db;
    }
    const float (*Rw)[3] = c.Rw;
    float dJ00 = Rw[0][0] * dT[0][0] + Rw[0][1] * dT[0][1] + Rw[0][2] * dT[0][2];
    float dJ02 = Rw[2][0] * dT[0][0] + Rw[2][1] * dT[0][1] + Rw[2][2] * dT[0][2];
    float dJ11 = Rw[1][0] * dT[1][0] + Rw[1][1] * dT[1][1] + Rw[1][2] * dT[1][2];
    float dJ12 = Rw[2][0] * dT[1][0] + Rw[2][1] * dT[1][1] + Rw[2][2] * dT[1][2];
    float tz = 1.f / tc.z, tz2 = tz * tz, tz3 = tz2 * tz;
    V3 dL_dt{xm * -c.fx * tz2 * dJ02, ym * -c.fy * tz2 * dJ12,
             -c.fx * tz2 * dJ00 - c.fy * tz2 * dJ11 + (2 * c.fx * tc.x) * tz3 * dJ02 + (2 * c.fy * tc.y) * tz3 * dJ12};
    // mean gradient through t = Rw mean + trans
    V3 dm{Rw[0][0] * dL_dt.x + Rw[1][0] * dL_dt.y + Rw[2][0] * dL_dt.z,
          Rw[0][1] * dL_dt.x + Rw[1][1] * dL_dt.y + Rw[2][1] * dL_dt.z,
          Rw[0][2] * dL_dt.x + Rw[1][2] * dL_dt.y + Rw[2][2] * dL_dt.z};
    // pose: translation part and rotation of the (clamped) camera point
    V3 tau_rho = dL_dt;
    V3 tau_theta = cross(tc, dL_dt);
    // pose: rotation W of the view entering T = J W
    float dRw[3][3];
    for (int k = 0; k < 3; ++k) {
      dRw[0][k] = (c.fx / tc.z) * dT[0][k];
      dRw[1][k] = (c.fy / tc.z) * dT[1][k];
      dRw[2][k] = (-(c.fx * tc.x) / (tc.z * tc.z)) * dT[0][k] + (-(c.fy * tc.y) / (tc.z * tc.z)) * dT[1][k];
    }
    for (int col = 0; col < 3; ++col) {
      V3 rc{Rw[0][col], Rw[1][col], Rw[2][col]};
      V3 gc{dRw[0][col], dRw[1][col], dRw[2][col]};
      tau_theta = tau_theta + cross(rc, gc);
    }

    // ---- preprocess backward: means2D (NDC) -> mean, depth, SH, cov3D
    V3 g2{g[0], g[1], 0.f};
    const float* pm = c.proj;
    float hom[4];
    xform44(pm, mean, hom);
    float m_w = 1.0f / (hom[3] + 0.0000001f);
    float mul1 = (pm[0] * mean.x + pm[4] * mean.y + pm[8] * mean.z + pm[12]) * m_w * m_w;
    float mul2 = (pm[1] * mean.x + pm[5] * mean.y + pm[9] * mean.z + pm[13]) * m_w * m_w;
    dm.x += (pm[0] * m_w - pm[3] * mul1) * g2.x + (pm[1] * m_w - pm[3] * mul2) * g2.y;
    dm.y += (pm[4] * m_w - pm[7] * mul1) * g2.x + (pm[5] * m_w - pm[7] * mul2) * g2.y;
    dm.z += (pm[8] * m_w - pm[11] * mul1) * g2.x + (pm[9] * m_w - pm[11] * mul2) * g2.y;
    // pose through the projection (upstream uses proj_raw's a, b, e only: V5)
    float alpha_ = m_w, beta_ = -hom[0] * m_w * m_w, gamma_ = -hom[1] * m_w * m_w;
    float pa = c.praw[0], pb = c.praw[5], pe = c.praw[11];
    V3 d1{alpha_ * pa, 0.f, beta_ * pe}, d2{0.f, alpha_ * pb, gamma_ * pe};
    V3 gp = g2.x * d1 + g2.y * d2;
    gp.z += ddepth;  // depth = p_C.z
    tau_rho = tau_rho + gp;
    tau_theta = tau_theta + cross(t, gp);
    dm.x += ddepth * c.view[2];
    dm.y += ddepth * c.view[6];
    dm.z += ddepth * c.view[10];
    if (s->has_sh) {
      bool cl[3] = {s->clamped[3 * i] != 0, s->clamped[3 * i + 1] != 0, s->clamped[3 * i + 2] != 0};
      V3 dmsh = sh_backward(D, s->sh + 3 * (size_t)M * i, mean, c.campos, cl, V3{g[6], g[7], g[8]}, osh);
      dm = dm + dmsh;
    }
    if (!s->has_cov) {
      // cov3D -> scale, rotation
      const float* sc = s->scales + 3 * (size_t)i;
      const float* q = s->rots + 4 * (size_t)i;
      float R[3][3]; quat_rot(q, R);
      float sv[3] = {s->scale_mod * sc[0], s->scale_mod * sc[1], s->scale_mod * sc[2]};
      float dS[3][3] = {{ocov[0], 0.5f * ocov[1], 0.5f * ocov[2]},
                        {0.5f * ocov[1], ocov[3], 0.5f * ocov[4]},
                        {0.5f * ocov[2], 0.5f * ocov[4], ocov[5]}};
      // Sigma = M^T M with M = diag(s) R^T ; dL/dM = 2 M dSigma
      float Mm[3][3], dM[3][3];
      for (int r0 = 0; r0 < 3; ++r0)
        for (int c0 = 0; c0 < 3; ++c0) Mm[r0][c0] = sv[r0] * R[c0][r0];
      for (int r0 = 0; r0 < 3; ++r0)
        for (int c0 = 0; c0 < 3; ++c0)
          dM[r0][c0] = 2.f * (Mm[r0][0] * dS[0][c0] + Mm[r0][1] * dS[1][c0] + Mm[r0][2] * dS[2][c0]);
      for (int k = 0; k < 3; ++k)
        // w.r.t. the modified scale (upstream omits the scale_modifier factor: V9)
        osc[k] = R[0][k] * dM[k][0] + R[1][k] * dM[k][1] + R[2][k] * dM[k][2];
      // dL/dR[j][k] = s_k dM[k][j]
      float G[3][3];
      for (int j = 0; j < 3; ++j)
        for (int k = 0; k < 3; ++k) G[j][k] = sv[k] * dM[k][j];
      float rr = q[0], x = q[1], y = q[2], z = q[3];
      orot[0] = 2 * z * (G[1][0] - G[0][1]) + 2 * y * (G[0][2] - G[2][0]) + 2 * x * (G[2][1] - G[1][2]);
      orot[1] = 2 * y * (G[1][0] + G[0][1]) + 2 * z * (G[2][0] + G[0][2]) + 2 * rr * (G[2][1] - G[1][2]) -
                4 * x * (G[2][2] + G[1][1]);
      orot[2] = 2 * x * (G[1][0] + G[0][1]) + 2 * rr * (G[0][2] - G[2][0]) + 2 * z * (G[2][1] + G[1][2]) -
                4 * y * (G[2][2] + G[0][0]);
      orot[3] = 2 * rr * (G[1][0] - G[0][1]) + 2 * x * (G[2][0] + G[0][2]) + 2 * y * (G[2][1] + G[1][2]) -
                4 * z * (G[1][1] + G[0][0]);
    }
    om[0] = dm.x; om[1] = dm.y; om[2] = dm.z;
    otau[0] = tau_rho.x; otau[1] = tau_rho.y; otau[2] = tau_rho.z;
    otau[3] = tau_theta.x; otau[4] = tau_theta.y; otau[5] = tau_theta.z;
  }
}

void cr_free(void* handle) { delete (State*)handle; }

// simple-knn distCUDA2 (Appendix B): mean of the 3 smallest squared distances
// to other points (self excluded by index; duplicates contribute 0; P < 4
// leaves FLT_MAX slots, so the mean overflows to inf).  Exact search over a
// uniform grid; distance evaluated as dx*dx + dy*dy + dz*dz, unfused.
void cr_distknn(int P, const float* pts, float* out) {
  if (P <= 0) return;
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int i = 0; i < P; ++i)
    for (int k = 0; k < 3; ++k) { mn[k] = std::min(mn[k], pts[3 * i + k]); mx[k] = std::max(mx[k], pts[3 * i + k]); }
  double ext[3], vol = 1.0;
  for (int k = 0; k < 3; ++k) { ext[k] = std::max<double>(mx[k] - mn[k], 1e-12); vol *= ext[k]; }
  double cell = std::cbrt(vol * 2.0 / P);
  int nc[3];
  for (int k = 0; k < 3; ++k) nc[k] = std::max(1, std::min(1024, (int)(ext[k] / cell) + 1));
  auto cidx = [&](const float* p, int k) {
    int v = (int)((p[k] - mn[k]) / ext[k] * nc[k]);
    return std::min(nc[k] - 1, std::max(0, v));
  };
  size_t ncell = (size_t)nc[0] * nc[1] * nc[2];
  std::vector<uint32_t> start(ncell + 1, 0), items(P);
  for (int i = 0; i < P; ++i) start[((size_t)cidx(pts + 3 * i, 2) * nc[1] + cidx(pts + 3 * i, 1)) * nc[0] + cidx(pts + 3 * i, 0) + 1]++;
  for (size_t q = 0; q < ncell; ++q) start[q + 1] += start[q];
  {
    std::vector<uint32_t> cur(start.begin(), start.end() - 1);
    for (int i = 0; i < P; ++i)
      items[cur[((size_t)cidx(pts + 3 * i, 2) * nc[1] + cidx(pts + 3 * i, 1)) * nc[0] + cidx(pts + 3 * i, 0)]++] = i;
  }
  double csz[3] = {ext[0] / nc[0], ext[1] / nc[1], ext[2] / nc[2]};
#pragma omp parallel for schedule(dynamic, 256)
  for (int i = 0; i < P; ++i) {
    const float* p = pts + 3 * i;
    float best[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
    int ci[3] = {cidx(p, 0), cidx(p, 1), cidx(p, 2)};
    int maxring = std::max(nc[0], std::max(nc[1], nc[2]));
    for (int ring = 0; ring <= maxring; ++ring) {
      // every point outside the (ring)-neighbourhood is at least this far away
      // (an axis whose cells the ring already spans bounds nothing: no point
      // lies outside the neighbourhood along it -- e.g. a flat or collinear
      // cloud's degenerate axis)
      double lo = DBL_MAX;
      for (int k = 0; k < 3; ++k) {
        if (ci[k] - ring <= 0 && ci[k] + ring >= nc[k] - 1) continue;
        double cmin = mn[k] + (ci[k] - ring) * csz[k], cmax = mn[k] + (ci[k] + ring + 1) * csz[k];
        lo = std::min(lo, std::min((double)p[k] - cmin, cmax - (double)p[k]));
      }
      for (int z = ci[2] - ring; z <= ci[2] + ring; ++z) {
        if (z < 0 || z >= nc[2]) continue;
        for (int y = ci[1] - ring; y <= ci[1] + ring; ++y) {
          if (y < 0 || y >= nc[1]) continue;
          for (int x = ci[0] - ring; x <= ci[0] + ring; ++x) {
            if (x < 0 || x >= nc[0]) continue;
            if (std::max(std::abs(x - ci[0]), std::max(std::abs(y - ci[1]), std::abs(z - ci[2]))) != ring) continue;
            size_t cell_id = ((size_t)z * nc[1] + y) * nc[0] + x;
            for (uint32_t u = start[cell_id]; u < start[cell_id + 1]; ++u) {
              uint32_t j = items[u];
              if ((int)j == i) continue;
              const float* o = pts + 3 * j;
              float dx = o[0] - p[0], dy = o[1] - p[1], dz = o[2] - p[2];
              float dist = dx * dx + dy * dy + dz * dz;  // built with -ffp-contract=off
              for (int k = 0; k < 3; ++k)
                if (best[k] > dist) { float tmp = best[k]; best[k] = dist; dist = tmp; }
            }
          }
        }
      }
      if (lo > 0 && best[2] < FLT_MAX && (double)best[2] <= lo * lo * 0.999999) break;
    }
    out[i] = (best[0] + best[1] + best[2]) / 3.0f;
  }
}

}  // extern "C"
