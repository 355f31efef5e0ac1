// diff_gaussian_rasterization._native: the three functions of upstream's
// pybind module (rasterize_points.cu of diff-gaussian-rasterization-w-pose,
// contract in SURVEY.md 8(b)) as a compiled torch extension over libwgsr's C
// ABI (include/wgsr.h).
//
// Same argument lists, return tuples, argument checks and error messages as
// the ctypes wrapper python/diff_gaussian_rasterization/_C.py, which stays the
// reference (and the path used when this module is not built).  What moves
// to C++ is the per-call host work around the kernels: output allocation,
// argument checks, the state-buffer allocation callbacks (torch uint8
// tensors, owned by the returned tuple) -- ~35 us of Python per backward
// call at TUM scale, time the GPU sat idle for whenever the kernels were
// shorter than the host path.
//
// libwgsr.so is not linked: _C.py hands over the entry points of the library
// it loaded (wgsr._lib, which honours WGSR_LIB), so both wrappers drive the
// same library.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include <exception>
#include <sstream>
#include <string>

#include "wgsr.h"

namespace {

using ForwardFn = int (*)(const wgsr_raster_args*, wgsr_alloc_fn, wgsr_alloc_fn, wgsr_alloc_fn, void*, float*, float*,
                          float*, int32_t*, int32_t*, int64_t*, void*);
using BackwardFn = int (*)(const wgsr_raster_args*, const int32_t*, const void*, void*, void*, int64_t, const float*,
                           const float*, wgsr_alloc_fn, void*, float*, float*, float*, float*, float*, float*, float*,
                           float*, float*, void*);
using MarkVisibleFn = int (*)(int, const float*, const float*, const float*, uint8_t*, void*);
using LastErrorFn = const char* (*)();

struct Lib {
  ForwardFn forward = nullptr;
  BackwardFn backward = nullptr;
  MarkVisibleFn mark_visible = nullptr;
  LastErrorFn last_error = nullptr;
} g_lib;

void bind(int64_t fwd, int64_t bwd, int64_t mv, int64_t err) {
  g_lib.forward = reinterpret_cast<ForwardFn>(fwd);
  g_lib.backward = reinterpret_cast<BackwardFn>(bwd);
  g_lib.mark_visible = reinterpret_cast<MarkVisibleFn>(mv);
  g_lib.last_error = reinterpret_cast<LastErrorFn>(err);
}

void need_lib() {
  if (!g_lib.forward || !g_lib.backward || !g_lib.mark_visible || !g_lib.last_error)
    throw std::runtime_error("diff_gaussian_rasterization._native: libwgsr entry points not bound");
}

void check(int code, const std::exception_ptr& alloc_failure = nullptr) {
  if (code == 3 /* WGSR_EALLOC */ && alloc_failure) std::rethrow_exception(alloc_failure);
  if (code != 0) {
    std::ostringstream s;
    s << "wgsr error " << code << ": " << g_lib.last_error();
    throw std::runtime_error(s.str());
  }
}

// python spelling of a dtype, as _C.py's f-strings print it
std::string dtype_name(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return "torch.float32";
    case at::kDouble: return "torch.float64";
    case at::kHalf: return "torch.float16";
    case at::kBFloat16: return "torch.bfloat16";
    case at::kInt: return "torch.int32";
    case at::kLong: return "torch.int64";
    case at::kShort: return "torch.int16";
    case at::kChar: return "torch.int8";
    case at::kByte: return "torch.uint8";
    case at::kBool: return "torch.bool";
    default: return std::string("torch.") + c10::toString(t);
  }
}

// _C._on: dtype, then device (a host pointer reaching a kernel faults the GPU)
at::Tensor on(const at::Tensor& t, const at::Device& dev, at::ScalarType dt, const char* name) {
  if (t.scalar_type() != dt)
    throw std::runtime_error(std::string(name) + ": expected " + dtype_name(dt) + ", got " +
                             dtype_name(t.scalar_type()));
  if (t.device() != dev || !t.device().is_cuda())
    throw std::runtime_error(std::string(name) + ": expected a tensor on " + dev.str() + ", got " +
                             t.device().str());
  return t.contiguous();
}

// _C._f32: absent (None or empty) -> undefined
at::Tensor f32(const c10::optional<at::Tensor>& t, const at::Device& dev, const char* name) {
  if (!t.has_value() || !t->defined() || t->numel() == 0) return at::Tensor();
  return on(*t, dev, at::kFloat, name);
}

const float* fp(const at::Tensor& t) { return t.defined() ? t.data_ptr<float>() : nullptr; }

// allocation callbacks: torch uint8 tensors kept in the context; a buffer of
// n bytes is the first n bytes of a max(n, 1)-byte tensor (as _lib._make_alloc)
// No exception may unwind through libwgsr's extern "C" frames: a failed
// allocation (e.g. torch's OutOfMemoryError) is kept and NULL returned, the
// library reports WGSR_EALLOC through its own error path, and check() then
// rethrows the original exception.
// A second call for the same buffer within one library call (the forward's
// predicted binning buffer was too small for the exact size) replaces the
// first allocation (wgsr.h: the library uses the pointer of the last call).
struct Alloc {
  at::Device dev;
  at::Tensor geom, binning, image, scratch;
  at::Tensor geom_b, binning_b, image_b, scratch_b;  // the allocations the slots view
  std::exception_ptr failure;
  explicit Alloc(const at::Device& d) : dev(d) {}
  void* take(at::Tensor& slot, at::Tensor& base, size_t n) noexcept {
    try {
      if (!base.defined() || base.numel() < (int64_t)(n > 0 ? n : 1))
        base = at::empty({(int64_t)(n > 0 ? n : 1)}, at::TensorOptions().dtype(at::kByte).device(dev));
      slot = base.narrow(0, 0, (int64_t)n);
      return base.data_ptr();
    } catch (...) {
      if (!failure) failure = std::current_exception();
      return nullptr;
    }
  }
};
void* alloc_geom(void* ctx, size_t n) { auto* a = static_cast<Alloc*>(ctx); return a->take(a->geom, a->geom_b, n); }
void* alloc_binning(void* ctx, size_t n) {
  auto* a = static_cast<Alloc*>(ctx);
  return a->take(a->binning, a->binning_b, n);
}
void* alloc_image(void* ctx, size_t n) { auto* a = static_cast<Alloc*>(ctx); return a->take(a->image, a->image_b, n); }
void* alloc_scratch(void* ctx, size_t n) {
  auto* a = static_cast<Alloc*>(ctx);
  return a->take(a->scratch, a->scratch_b, n);
}

wgsr_raster_args make_args(int P, int D, int M, int W, int H, const at::Tensor& bg, const at::Tensor& means3D,
                           const at::Tensor& colors, const at::Tensor& opacity, const at::Tensor& scales,
                           const at::Tensor& rotations, const at::Tensor& cov3D, const at::Tensor& sh,
                           const at::Tensor& view, const at::Tensor& proj, const at::Tensor& proj_raw,
                           const at::Tensor& campos, double scale_modifier, double tan_fovx, double tan_fovy,
                           bool prefiltered, bool debug) {
  wgsr_raster_args a{};
  a.P = P;
  a.D = D;
  a.M = M;
  a.W = W;
  a.H = H;
  a.bg = fp(bg);
  a.means3D = fp(means3D);
  a.colors = fp(colors);
  a.opacities = fp(opacity);
  a.scales = fp(scales);
  a.rotations = fp(rotations);
  a.cov3D_precomp = fp(cov3D);
  a.shs = fp(sh);
  a.viewmatrix = fp(view);
  a.projmatrix = fp(proj);
  a.projmatrix_raw = fp(proj_raw);
  a.campos = fp(campos);
  a.scale_modifier = (float)scale_modifier;
  a.tan_fovx = (float)tan_fovx;
  a.tan_fovy = (float)tan_fovy;
  a.prefiltered = prefiltered ? 1 : 0;
  a.debug = debug ? 1 : 0;
  return a;
}

void* stream_of(const at::Device& dev) { return at::hip::getCurrentHIPStream(dev.index()).stream(); }

using OptT = c10::optional<at::Tensor>;

std::tuple<int64_t, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor>
rasterize_gaussians(const OptT& background, const at::Tensor& means3D, const OptT& colors, const OptT& opacity,
                    const OptT& scales, const OptT& rotations, double scale_modifier, const OptT& cov3D_precomp,
                    const OptT& viewmatrix, const OptT& projmatrix, const OptT& projmatrix_raw, double tan_fovx,
                    double tan_fovy, int64_t image_height, int64_t image_width, const OptT& sh, int64_t degree,
                    const OptT& campos, bool prefiltered, bool debug) {
  if (means3D.dim() != 2 || means3D.size(1) != 3)
    throw std::runtime_error("means3D must have dimensions (num_points, 3)");
  need_lib();
  const at::Device dev = means3D.device();
  const int64_t P = means3D.size(0);
  const int64_t H = image_height, W = image_width;
  const auto fo = at::TensorOptions().dtype(at::kFloat).device(dev);
  const auto io = at::TensorOptions().dtype(at::kInt).device(dev);
  at::Tensor out_color = at::empty({3, H, W}, fo);
  at::Tensor out_depth = at::empty({1, H, W}, fo);
  at::Tensor out_opacity = at::empty({1, H, W}, fo);
  at::Tensor radii = at::empty({P}, io);
  at::Tensor n_touched = at::empty({P}, io);
  if (!dev.is_cuda()) throw std::runtime_error("means3D: expected a HIP device tensor, got " + dev.str());
  const at::Tensor shc = f32(sh, dev, "sh");
  const int M = shc.defined() ? (int)shc.size(1) : 0;
  const at::Tensor bg = f32(background, dev, "bg"), m = f32(means3D, dev, "means3D");
  const at::Tensor col = f32(colors, dev, "colors"), op = f32(opacity, dev, "opacity");
  const at::Tensor sc = f32(scales, dev, "scales"), rot = f32(rotations, dev, "rotations");
  const at::Tensor cov = f32(cov3D_precomp, dev, "cov3D_precomp");
  const at::Tensor vm = f32(viewmatrix, dev, "viewmatrix"), pm = f32(projmatrix, dev, "projmatrix");
  const at::Tensor pr = f32(projmatrix_raw, dev, "projmatrix_raw"), cp = f32(campos, dev, "campos");
  const wgsr_raster_args a = make_args((int)P, (int)degree, M, (int)W, (int)H, bg, m, col, op, sc, rot, cov, shc, vm,
                                       pm, pr, cp, scale_modifier, tan_fovx, tan_fovy, prefiltered, debug);
  const at::DeviceGuard guard(dev);
  Alloc al(dev);
  int64_t nr = 0;
  const int code = g_lib.forward(&a, alloc_geom, alloc_binning, alloc_image, &al, out_color.data_ptr<float>(),
                                 out_depth.data_ptr<float>(), out_opacity.data_ptr<float>(),
                                 P ? radii.data_ptr<int32_t>() : nullptr, P ? n_touched.data_ptr<int32_t>() : nullptr,
                                 &nr, stream_of(dev));
  check(code, al.failure);
  const at::Tensor empty = at::empty({0}, at::TensorOptions().dtype(at::kByte).device(dev));
  return {nr,
          out_color,
          radii,
          al.geom.defined() ? al.geom : empty,
          al.binning.defined() ? al.binning : empty,
          al.image.defined() ? al.image : empty,
          out_depth,
          out_opacity,
          n_touched};
}

// out_*: optional preallocated outputs (the `out` dict of _C.py) -- contiguous
// float32 of the output's shape on the device
at::Tensor take_out(const OptT& t, const at::Tensor& dflt, const at::Device& dev, const char* name) {
  if (!t.has_value() || !t->defined()) return dflt;
  if (t->sizes() != dflt.sizes() || t->scalar_type() != at::kFloat || !t->is_contiguous() || t->device() != dev) {
    // python's tuple spelling: (n,) or (a, b, ...)
    std::ostringstream s;
    s << "out['" << name << "'] must be a contiguous float32 (";
    for (int64_t i = 0; i < dflt.dim(); ++i) s << (i ? ", " : "") << dflt.size(i);
    s << (dflt.dim() == 1 ? ",)" : ")") << " on " << dev.str();
    throw std::runtime_error(s.str());
  }
  return *t;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor>
rasterize_gaussians_backward(const OptT& background, const at::Tensor& means3D, const at::Tensor& radii_in,
                             const OptT& colors, const OptT& scales, const OptT& rotations, double scale_modifier,
                             const OptT& cov3D_precomp, const OptT& viewmatrix, const OptT& projmatrix,
                             const OptT& projmatrix_raw, double tan_fovx, double tan_fovy,
                             const at::Tensor& dL_dout_color, const at::Tensor& dL_dout_depth, const OptT& sh,
                             int64_t degree, const OptT& campos, const at::Tensor& geomBuffer, int64_t R,
                             const at::Tensor& binningBuffer, const at::Tensor& imageBuffer, bool debug,
                             const OptT& out_means3D, const OptT& out_shs, const OptT& out_opacities,
                             const OptT& out_scales, const OptT& out_rotations) {
  need_lib();
  const at::Device dev = means3D.device();
  const int64_t P = means3D.size(0);
  const int64_t H = dL_dout_color.size(1), W = dL_dout_color.size(2);
  if (!dev.is_cuda()) throw std::runtime_error("means3D: expected a HIP device tensor, got " + dev.str());
  const at::Tensor shc = f32(sh, dev, "sh");
  const int64_t M = shc.defined() ? shc.size(1) : 0;
  const auto fo = at::TensorOptions().dtype(at::kFloat).device(dev);
  at::Tensor dL_dmeans2D = at::empty({P, 3}, fo);
  at::Tensor dL_dcolors = at::empty({P, 3}, fo);
  at::Tensor dL_dopacity = at::empty({P, 1}, fo);
  at::Tensor dL_dmeans3D = at::empty({P, 3}, fo);
  at::Tensor dL_dcov3D = at::empty({P, 6}, fo);
  at::Tensor dL_dsh = M == 0 ? at::zeros({P, M, 3}, fo) : at::empty({P, M, 3}, fo);
  at::Tensor dL_dscales = at::empty({P, 3}, fo);
  at::Tensor dL_drotations = at::empty({P, 4}, fo);
  dL_dmeans3D = take_out(out_means3D, dL_dmeans3D, dev, "means3D");
  dL_dsh = take_out(out_shs, dL_dsh, dev, "shs");
  dL_dopacity = take_out(out_opacities, dL_dopacity, dev, "opacities");
  dL_dscales = take_out(out_scales, dL_dscales, dev, "scales");
  dL_drotations = take_out(out_rotations, dL_drotations, dev, "rotations");
  at::Tensor dL_dtau = at::empty({P, 6}, fo);
  if (P == 0)
    return {dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations, dL_dtau};
  const at::Tensor m = f32(means3D, dev, "means3D");
  const at::Tensor radii = on(radii_in, dev, at::kInt, "radii");
  if (radii.numel() != P)
    throw std::runtime_error("radii: expected " + std::to_string(P) + " entries, got " +
                             std::to_string(radii.numel()));
  if (geomBuffer.numel()) on(geomBuffer, dev, at::kByte, "geomBuffer");
  if (binningBuffer.numel()) on(binningBuffer, dev, at::kByte, "binningBuffer");
  if (imageBuffer.numel()) on(imageBuffer, dev, at::kByte, "imageBuffer");
  // the backward does not read opacities (they live in the geometry buffer);
  // any valid device pointer satisfies the argument check
  const at::Tensor bg = f32(background, dev, "bg"), col = f32(colors, dev, "colors");
  const at::Tensor sc = f32(scales, dev, "scales"), rot = f32(rotations, dev, "rotations");
  const at::Tensor cov = f32(cov3D_precomp, dev, "cov3D_precomp");
  const at::Tensor vm = f32(viewmatrix, dev, "viewmatrix"), pm = f32(projmatrix, dev, "projmatrix");
  const at::Tensor pr = f32(projmatrix_raw, dev, "projmatrix_raw"), cp = f32(campos, dev, "campos");
  const wgsr_raster_args a = make_args((int)P, (int)degree, (int)M, (int)W, (int)H, bg, m, col, m, sc, rot, cov, shc,
                                       vm, pm, pr, cp, scale_modifier, tan_fovx, tan_fovy, false, debug);
  const at::Tensor gc = on(dL_dout_color, dev, at::kFloat, "dL_dout_color");
  const at::Tensor gd = on(dL_dout_depth, dev, at::kFloat, "dL_dout_depth");
  auto bp = [](const at::Tensor& t) -> void* { return t.numel() ? t.data_ptr() : nullptr; };
  const at::DeviceGuard guard(dev);
  Alloc al(dev);
  const int code = g_lib.backward(
      &a, radii.data_ptr<int32_t>(), bp(geomBuffer), bp(binningBuffer), bp(imageBuffer), R, gc.data_ptr<float>(),
      gd.data_ptr<float>(), alloc_scratch, &al, dL_dmeans2D.data_ptr<float>(), dL_dcolors.data_ptr<float>(),
      dL_dopacity.data_ptr<float>(), dL_dmeans3D.data_ptr<float>(), dL_dcov3D.data_ptr<float>(),
      dL_dsh.numel() ? dL_dsh.data_ptr<float>() : nullptr, dL_dscales.data_ptr<float>(),
      dL_drotations.data_ptr<float>(), dL_dtau.data_ptr<float>(), stream_of(dev));
  check(code, al.failure);
  return {dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations, dL_dtau};
}

at::Tensor mark_visible(const at::Tensor& means3D, const at::Tensor& viewmatrix, const at::Tensor& projmatrix) {
  need_lib();
  const at::Device dev = means3D.device();
  const int64_t P = means3D.size(0);
  if (!dev.is_cuda()) throw std::runtime_error("means3D: expected a HIP device tensor, got " + dev.str());
  at::Tensor present = at::empty({P}, at::TensorOptions().dtype(at::kBool).device(dev));
  const at::Tensor m = on(means3D, dev, at::kFloat, "means3D");
  const at::Tensor v = on(viewmatrix, dev, at::kFloat, "viewmatrix");
  const at::Tensor pm = on(projmatrix, dev, at::kFloat, "projmatrix");
  const at::DeviceGuard guard(dev);
  const int code = g_lib.mark_visible((int)P, m.data_ptr<float>(), v.data_ptr<float>(), pm.data_ptr<float>(),
                                      P ? reinterpret_cast<uint8_t*>(present.data_ptr()) : nullptr, stream_of(dev));
  check(code);
  return present;
}

}  // namespace

PYBIND11_MODULE(_native, mod) {
  mod.doc() = "diff_gaussian_rasterization entry points over libwgsr (compiled host wrapper)";
  mod.def("bind", &bind);
  mod.def("rasterize_gaussians", &rasterize_gaussians);
  mod.def("rasterize_gaussians_backward", &rasterize_gaussians_backward);
  mod.def("mark_visible", &mark_visible);
}
