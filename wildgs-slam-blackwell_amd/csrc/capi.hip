// C ABI of libwgsr (include/wgsr.h): host orchestration of the gfx950 stages.
//
// Mirrors upstream CudaRasterizer::Rasterizer::{forward, backward, markVisible}
// and SimpleKNN::knn with plain pointers: the caller owns all
// memory (allocation callbacks), every launch goes on the caller's stream, and
// the only host synchronisation is the num_rendered read in the forward.
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <immintrin.h>

#include "wgsr.h"
#include "wgsr_common.h"
#include "wgsr_internal.h"

namespace wgsr {

namespace {
thread_local char g_err[1024] = "";

// Pinned host landing zone for the forward's pair counts + the event that
// marks their arrival (one per host thread; never freed).
struct HostCounters {
  uint32_t* buf = nullptr;
  hipEvent_t ev = nullptr;
  // the D->H copy runs on a side stream behind `pre` (recorded after
  // k_preprocess), so the forward's stream goes straight on to the depth
  // sort instead of waiting out the copy and its host-visible release
  // (~10 us of the stream's time per forward; used when the Gaussian-level
  // depth sort runs, which the copy then overlaps)
  hipStream_t side = nullptr;
  hipEvent_t pre = nullptr;
  // per-bin default: k_publish_counts writes the block into `mbox` (coherent
  // pinned memory, kCounterBytes) and then `seq` into mbox_seq; the host
  // spins on that word instead of an event behind a blit-kernel copy (the
  // copy and its completion signal left the GPU idle ~6 us before the scan
  // and the host woke up later; measured in DESIGN.md section 8, round 6)
  uint4* mbox = nullptr;  // {seq << 8 | flags | 0x80 if > 32 bits, N_rect, N, N_bin}
  uint32_t seq = 0;
};
// one pinned block + event per (host thread, device): an event recorded on a
// stream must belong to that stream's device
constexpr int kMaxDevices = 64;
// The binning buffer's size is known only after the forward's one host wait;
// allocating it there put the allocation (~10 us of the caller's allocator)
// on the GPU's critical path.  The previous forward of the same shape on this
// thread predicts it: a buffer of that size (+1/16) is allocated BEFORE the
// wait, while k_preprocess runs, and only a forward that needs more allocates
// again after it.  (The binning layout is sized by num_rendered as always; a
// larger buffer just leaves its tail unused.)
struct BinningGuess {
  int P = -1, W = 0, H = 0, bshift = -1;
  size_t bytes = 0;
};
BinningGuess& binning_guess() {
  thread_local BinningGuess g[kMaxDevices];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) dev = 0;
  return g[dev];
}

// WGSR_PUBLISH_COUNTS=0: the blit-kernel copy + event wait for every forward
bool publish_counts() {
  static const bool on = [] {
    const char* e = getenv("WGSR_PUBLISH_COUNTS");
    return !(e && e[0] == '0');
  }();
  return on;
}

HostCounters& host_counters() {
  thread_local HostCounters per_dev[kMaxDevices];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) dev = 0;
  HostCounters& hc = per_dev[dev];
  if (!hc.buf) {
    void* p = nullptr;
    if (hipHostMalloc(&p, kCounterBytes, hipHostMallocDefault) != hipSuccess) p = nullptr;
    hc.buf = static_cast<uint32_t*>(p);
    if (hipEventCreateWithFlags(&hc.ev, hipEventDisableTiming) != hipSuccess) hc.ev = nullptr;
    if (hipStreamCreateWithFlags(&hc.side, hipStreamNonBlocking) != hipSuccess) hc.side = nullptr;
    if (hc.side && hipEventCreateWithFlags(&hc.pre, hipEventDisableTiming) != hipSuccess) hc.pre = nullptr;
    if (!hc.pre) hc.side = nullptr;
    void* m = nullptr;
    if (publish_counts() &&
        hipHostMalloc(&m, 256, hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess) {
      hc.mbox = static_cast<uint4*>(m);
      *hc.mbox = make_uint4(0u, 0u, 0u, 0u);
    }
  }
  return hc;
}

// The forward's counter block without a memset launch per call: two blocks
// per (host thread, device) in device memory.  A forward accumulates into one
// and its k_preprocess zeroes the other for the next forward on this thread.
// The previous forward's block was last touched by its D->H copy, which the
// host waited for before that call returned, so no stream (ours or another)
// can still be reading it.  (If the two blocks cannot be allocated, the
// geometry buffer's counter block is zeroed by a memset per call.)
struct DevCounters {
  uint32_t* buf = nullptr;  // 2 x kCounterBytes, zeroed once
  int parity = 0;
  bool failed = false;
};
// The per-bin depth sort emits the per-tile lists itself for small bins
// (2 x 2 tiles: TUM 512 x 384, 35.4 -> 33.8 us for sort + lists); with 4 x 4-
// tile bins (1080p) the 16-tile compaction inside the one-workgroup-per-CU
// sort costs more than k_expand_bins' 4x wider grid (140.8 vs 131.3 us).
bool bds_emit(int bshift) { return bshift <= 1; }


DevCounters* dev_counters(hipStream_t s) {
  thread_local DevCounters per_dev[kMaxDevices];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return nullptr;
  DevCounters& dc = per_dev[dev];
  if (!dc.buf && !dc.failed) {
    void* p = nullptr;
    // zeroed on the first forward's stream (ahead of its k_preprocess; any
    // later forward of this thread starts after this one's host wait)
    if (hipMalloc(&p, 2 * kCounterBytes) != hipSuccess || hipMemsetAsync(p, 0, 2 * kCounterBytes, s) != hipSuccess) {
      dc.failed = true;  // fall back to the per-call memset
      return nullptr;
    }
    dc.buf = static_cast<uint32_t*>(p);
  }
  return dc.buf ? &dc : nullptr;
}

}

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int num_bits(uint32_t n) {
  int b = 0;
  while (b < 32 && (1ull << b) < n) ++b;
  return b;
}

namespace {

// ---- optional per-stage timing with HIP events on the caller's stream -----
const char* const kStageNames[WGSR_NUM_STAGES] = {"preprocess", "depth_sort", "offsets_scan", "duplicate",
                                                  "tile_sort", "ranges", "render_fwd", "render_bwd",
                                                  "gauss_bwd", "dist_cuda2"};
struct Prof {
  uint32_t mask = 0;  // stages timed (bit i: stage i)
  struct Rec { int stage; hipEvent_t a, b; };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
  double ms[WGSR_NUM_STAGES] = {};
  int64_t count[WGSR_NUM_STAGES] = {};
  hipEvent_t get() {
    if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
  }
  void flush() {
    for (auto& r : recs) {
      float t = 0.f;
      if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&t, r.a, r.b) == hipSuccess) {
        ms[r.stage] += t;
        count[r.stage] += 1;
      }
      pool.push_back(r.a);
      pool.push_back(r.b);
    }
    recs.clear();
  }
};
Prof g_prof;  // process-wide; the bench is single-threaded per rank

struct StageTimer {
  int stage;
  hipStream_t s;
  hipEvent_t a = nullptr;
  StageTimer(int st, hipStream_t str) : stage(st), s(str) {
    if (((g_prof.mask >> st) & 1u) && (a = g_prof.get()) && hipEventRecord(a, s) != hipSuccess) a = nullptr;
  }
  ~StageTimer() {
    if (!a) return;
    hipEvent_t b = g_prof.get();
    if (b && hipEventRecord(b, s) == hipSuccess) g_prof.recs.push_back({stage, a, b});
    else g_prof.pool.push_back(a);
  }
};

struct Grid {
  int gx, gy, nt;
  explicit Grid(const wgsr_raster_args& a)
      : gx((a.W + kTile - 1) / kTile), gy((a.H + kTile - 1) / kTile), nt(gx * gy) {}
};

int tile_sort_bits(const Grid& g) { return num_bits((uint32_t)g.nt) > 0 ? num_bits((uint32_t)g.nt) : 1; }

// Sort-bin shift (Bins, wgsr_common.h): the duplicate + radix sort work on
// (Gaussian, bin) pairs of 2^s x 2^s tiles, and k_expand_bins cuts the sorted
// bin lists into the exact per-tile lists (the pair key carries the
// Gaussian's exact tile mask inside the bin).  Default 4 x 4 tiles: at 1080p
// 510 bins, ~1.3 sorted pairs per visible Gaussian instead of ~9.
// WGSR_BIN_SHIFT overrides (the backward finds the lists through the image
// buffer's meta word, so it never depends on the setting).
// Small frames (<= kSmallFrameTiles tiles) default to 2 x 2-tile bins: their
// expand step is launch-latency bound and finer bins shorten it (A/B, 100k
// Gaussians: 512x384 0.328 -> 0.324 ms, 640x480 0.342 -> 0.335 ms).
constexpr int kDefaultBinShift = 2;
constexpr int kSmallFrameTiles = 2048;
int bin_shift(const wgsr_raster_args& a) {
  const char* e = getenv("WGSR_BIN_SHIFT");
  const Grid g(a);
  int sh = e ? atoi(e) : (g.nt <= kSmallFrameTiles ? 1 : kDefaultBinShift);
  sh = sh < 0 ? 0 : (sh > kMaxBinShift ? kMaxBinShift : sh);
  // bin ids fit the key's low 16 bits, list lengths the packed scan's 16 bits
  return sh > 0 && g.nt > 65535 ? 0 : sh;
}
// WGSR_DEPTH_SORT=full: the depth sort as four 8-bit passes over the whole
// 32-bit keys (the reference schedule for A/B runs and the parity tests);
// default: three passes over the visible key range (launch_depth_sort)
bool depth_sort_full() {
  const char* e = getenv("WGSR_DEPTH_SORT");  // read per call: tests compare the modes
  return e && strcmp(e, "full") == 0;
}
// With sort bins the default orders each bin's entries by depth after the bin
// sort (k_bin_depth_sort: the pairs are duplicated in index order, no
// Gaussian depth order exists); WGSR_DEPTH_SORT=global|full keeps the
// Gaussian-level depth sort ahead of the duplication (the previous schedule,
// and the one whose depth order wgsr_depth_order_offset exposes).
// The default whenever sort bins are on (A/B, ms/step: 100k 512x384 SH0
// 0.218 -> 0.190; 200k / 500k / 1M at 1080p SH3 0.720 -> 0.674, 0.712 ->
// 0.696, 0.807 -> 0.801).  WGSR_DEPTH_SORT=global|full keeps the
// Gaussian-level sort.
// ... unless the bins average more than this many entries (the host sees the
// bin-pair count at its one wait and then falls back to the Gaussian-level
// sort; WGSR_BIN_DEPTH_MAX_AVG overrides)
size_t bin_depth_max_avg() {
  const char* e = getenv("WGSR_BIN_DEPTH_MAX_AVG");  // (per call: tests force the fallback)
  return e ? (size_t)strtoull(e, nullptr, 10) : (size_t)6144;
}
bool depth_sort_bins(const wgsr_raster_args& a, int bshift) {
  if (!bshift) return false;
  const char* e = getenv("WGSR_DEPTH_SORT");
  if (e && (strcmp(e, "full") == 0 || strcmp(e, "global") == 0)) return false;
  (void)a;
  return true;
}
constexpr int kDepthBits = 32;
constexpr bool kFullDepthInAlt = ((kDepthBits + 7) / 8) % 2 == 1;
// byte offset of the last forward's depth order (rank -> Gaussian) in its
// geometry buffer (wgsr_depth_order_offset)
thread_local int64_t g_depth_order_off = -1;  // -1: no depth order (bin_depth)

int validate(const wgsr_raster_args* a) {
  if (!a) return set_error(WGSR_EINVAL, "null args");
  if (a->P < 0) return set_error(WGSR_EINVAL, "means3D must have dimensions (num_points, 3)");
  if (a->W <= 0 || a->H <= 0) return set_error(WGSR_EINVAL, "image size must be positive (got %dx%d)", a->W, a->H);
  if (a->P == 0) return WGSR_OK;
  if (!a->means3D || !a->opacities || !a->bg || !a->viewmatrix || !a->projmatrix || !a->campos)
    return set_error(WGSR_EINVAL, "missing required tensor");
  if ((a->shs == nullptr) == (a->colors == nullptr))
    return set_error(WGSR_EINVAL, "Please provide excatly one of either SHs or precomputed colors!");
  const bool sr = a->scales && a->rotations;
  if (sr == (a->cov3D_precomp != nullptr))
    return set_error(WGSR_EINVAL,
                     "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
  if (a->shs && (a->M <= 0 || a->D < 0 || a->D > 3 || (a->D + 1) * (a->D + 1) > a->M))
    return set_error(WGSR_EINVAL, "invalid SH configuration (degree %d, %d coefficients)", a->D, a->M);
  const Grid g(*a);
  if (g.gx > 65535 || g.gy > 65535) return set_error(WGSR_EINVAL, "image too large");
  return WGSR_OK;
}

#define HIPCHK(expr)                                                                          \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess) return set_error(WGSR_EHIP, "%s: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

#define STAGE(a, s, expr)                   \
  do {                                      \
    HIPCHK(expr);                           \
    if ((a).debug) {                        \
      HIPCHK(hipStreamSynchronize(s));      \
      HIPCHK(hipGetLastError());            \
    }                                       \
  } while (0)

void* call_alloc(wgsr_alloc_fn fn, void* ctx, size_t bytes) { return fn ? fn(ctx, bytes) : nullptr; }

}  // namespace
}  // namespace wgsr

using namespace wgsr;

extern "C" {

const char* wgsr_last_error(void) { return g_err; }

void wgsr_profile_enable(int on) {
  g_prof.flush();
  // 1: every stage (each timed stage adds two event records to the stream);
  // otherwise on is the mask of stages to time, as (mask << 1) | 0 ... see wgsr.h
  g_prof.mask = on == 1 ? ((1u << WGSR_NUM_STAGES) - 1u) : (on > 1 ? ((uint32_t)on >> 1) : 0u);
}

int wgsr_profile_read(double* ms, int64_t* counts, int n, int reset) {
  g_prof.flush();
  const int m = n < WGSR_NUM_STAGES ? n : WGSR_NUM_STAGES;
  for (int i = 0; i < m; ++i) {
    if (ms) ms[i] = g_prof.ms[i];
    if (counts) counts[i] = g_prof.count[i];
  }
  if (reset)
    for (int i = 0; i < WGSR_NUM_STAGES; ++i) { g_prof.ms[i] = 0; g_prof.count[i] = 0; }
  return WGSR_NUM_STAGES;
}

const char* wgsr_profile_stage_name(int i) { return (i >= 0 && i < WGSR_NUM_STAGES) ? kStageNames[i] : ""; }
#ifndef WGSR_SRC_ID
#define WGSR_SRC_ID "unversioned"
#endif
// (src: digest of csrc/ + include/wgsr.h at build time, Makefile SRC_ID)
const char* wgsr_version(void) { return "wgsr 0.1 gfx950 src:" WGSR_SRC_ID; }
int64_t wgsr_depth_order_offset(void) { return g_depth_order_off; }

size_t wgsr_geometry_bytes(int P) { return GeomLayout((size_t)(P > 0 ? P : 0)).total; }
size_t wgsr_binning_bytes(int64_t N, int W, int H) {
  (void)W; (void)H;
  return BinLayout((size_t)(N > 0 ? N : 0)).total;
}
size_t wgsr_image_bytes(int W, int H) { return ImageLayout(W, H).total; }

int wgsr_rasterize_forward(const wgsr_raster_args* args, wgsr_alloc_fn geom_alloc, wgsr_alloc_fn binning_alloc,
                           wgsr_alloc_fn image_alloc, void* ctx, float* out_color, float* out_depth,
                           float* out_opacity, int32_t* radii, int32_t* n_touched, int64_t* num_rendered,
                           void* stream) {
  g_err[0] = 0;
  if (int e = validate(args)) return e;
  const wgsr_raster_args& a = *args;
  hipStream_t s = (hipStream_t)stream;
  *num_rendered = 0;
  const size_t HW = (size_t)a.W * a.H;
  if (a.P == 0) {
    // upstream returns zero images when there is nothing to rasterise
    call_alloc(geom_alloc, ctx, 0);
    call_alloc(binning_alloc, ctx, 0);
    call_alloc(image_alloc, ctx, 0);
    HIPCHK(hipMemsetAsync(out_color, 0, 3 * HW * sizeof(float), s));
    HIPCHK(hipMemsetAsync(out_depth, 0, HW * sizeof(float), s));
    HIPCHK(hipMemsetAsync(out_opacity, 0, HW * sizeof(float), s));
    return WGSR_OK;
  }
  const Grid grid(a);
  const GeomLayout GL((size_t)a.P);
  const ImageLayout IL(a.W, a.H);
  void* geom = call_alloc(geom_alloc, ctx, GL.total);
  if (!geom) return set_error(WGSR_EALLOC, "geometry buffer allocation failed");
  void* image = call_alloc(image_alloc, ctx, IL.total);
  if (!image) return set_error(WGSR_EALLOC, "image buffer allocation failed");

  // counter block (kCounterBytes): error flags and the partial sums of
  // upstream's num_rendered and of the exact list lengths, all produced by
  // k_preprocess
  DevCounters* dc = dev_counters(s);
  uint32_t* counter = dc ? dc->buf + (size_t)dc->parity * (kCounterBytes / 4) : at<uint32_t>(geom, GL.counter);
  if (!dc) HIPCHK(hipMemsetAsync(counter, 0, kCounterBytes, s));
  const int bshift = bin_shift(a);
  const Bins bins(grid.gx, grid.gy, bshift);
  // the depth sort's superblock sums are zeroed by k_preprocess's workgroups
  // (no memset launch), and so is the next forward's counter block
  bool bin_depth = depth_sort_bins(a, bshift);
  const bool full_depth = !bin_depth && depth_sort_full();
  size_t sup_off = 0;
  const size_t sup_words = bin_depth    ? 0
                           : full_depth ? sort_sup_words((size_t)a.P, 0, kDepthBits, &sup_off)
                                        : depth_sort_sup_words((size_t)a.P);
  if (!full_depth) sup_off = depth_sort_sup_offset_words((size_t)a.P);
  ZeroJob zj{};
  if (dc) {
    zj.p[zj.count] = reinterpret_cast<float*>(dc->buf + (size_t)(dc->parity ^ 1) * (kCounterBytes / 4));
    zj.n[zj.count++] = kCounterBytes / 4;
  }
  if (sup_words) {
    zj.p[zj.count] = reinterpret_cast<float*>(at<uint32_t>(geom, GL.hist) + sup_off);
    zj.n[zj.count++] = sup_words;
  }
  // ... and, with sort bins, the dual scan's superblock sums
  const bool scan_sup = bshift != 0;
  if (scan_sup) {
    zj.p[zj.count] = at<float>(geom, GL.bsup);
    zj.n[zj.count++] = 2 * kScanSupStride * packed_scan_supers((size_t)a.P);
  }
  // Once k_preprocess is queued it zeroes the thread's other counter block;
  // the next forward may only reuse that block after this call's host wait.
  // Any error return before that wait synchronises the stream instead.
  struct SyncOnError {
    hipStream_t s;
    bool armed = false;
    ~SyncOnError() { if (armed) (void)hipStreamSynchronize(s); }
  } sync_on_error{s};
  { StageTimer T(0, s);
  const hipError_t pe = launch_preprocess(a, geom, radii, n_touched, counter + 1,
                                          reinterpret_cast<unsigned long long*>(counter + 4), bshift, zj, s,
                                          at<uint32_t>(image, IL.meta));
  if (pe == hipSuccess && dc) dc->parity ^= 1;  // k_preprocess, which zeroes the other block, is queued
  sync_on_error.armed = true;
  STAGE(a, s, pe); }

  // The pair counts are known once k_preprocess is done: copy them to pinned
  // host memory behind it and let the depth sort + scan run while the host
  // waits for them, allocates the binning buffer and queues the rest.
  HostCounters& hc = host_counters();
  if (!hc.buf || !hc.ev) return set_error(WGSR_EHIP, "pinned counter buffer / event allocation failed");
  // (with the per-bin depth sort nothing would overlap the copy on the side
  // stream, whose start waits out an event round trip: copy in stream order)
  // per-bin default: the scan's first wave publishes the counts (PublishJob)
  const bool mailbox = bin_depth && bshift && hc.mbox;
  // (24-bit sequence numbers, never 0: the record's initial value)
  const uint32_t want = mailbox ? (hc.seq = (hc.seq % 0xFFFFFFu) + 1u) : 0u;
  PublishJob pub{};
  if (mailbox) {
    // (no event behind it: an event record makes the runtime end the kernel
    // with a system-scope release, ~6 us before the next kernel starts; the
    // wait below checks the stream itself instead)
    pub.counter = counter;
    pub.host = hc.mbox;
    pub.seq = want;
  } else if (hc.side && !bin_depth) {
    HIPCHK(hipEventRecord(hc.pre, s));
    HIPCHK(hipStreamWaitEvent(hc.side, hc.pre, 0));
    HIPCHK(hipMemcpyAsync(hc.buf, counter, kCounterBytes, hipMemcpyDeviceToHost, hc.side));
    HIPCHK(hipEventRecord(hc.ev, hc.side));
  } else {
    HIPCHK(hipMemcpyAsync(hc.buf, counter, kCounterBytes, hipMemcpyDeviceToHost, s));
    HIPCHK(hipEventRecord(hc.ev, s));
  }
  // depth order of the Gaussians (culled ones carry key 0xFFFFFFFF -> last)
  const uint32_t* depth_order = nullptr;  // null: index order (bin_depth)
  if (!bin_depth) { StageTimer T(1, s);
  if (full_depth) {
    bool in_alt = false;
    STAGE(a, s, radix_sort_pairs(at<uint32_t>(geom, GL.dkey), at<uint32_t>(geom, GL.dkey_alt),
                                 at<uint32_t>(geom, GL.dval), at<uint32_t>(geom, GL.dval_alt), true, (size_t)a.P, 0,
                                 kDepthBits, at<uint32_t>(geom, GL.hist), at<uint32_t>(geom, GL.totals), s, &in_alt,
                                 nullptr, nullptr, sup_words != 0));
    if (in_alt != kFullDepthInAlt) return set_error(WGSR_EHIP, "internal: depth sort parity");
    depth_order = at<uint32_t>(geom, kFullDepthInAlt ? GL.dval_alt : GL.dval);
  } else {
    STAGE(a, s, launch_depth_sort(at<uint32_t>(geom, GL.dkey), at<uint32_t>(geom, GL.dkey_alt),
                                  at<uint32_t>(geom, GL.dval), at<uint32_t>(geom, GL.dval_alt), (size_t)a.P,
                                  counter + kDepthRangeOffset / 4, counter + 2, at<uint32_t>(geom, GL.hist), s));
    depth_order = at<uint32_t>(geom, GL.dval_alt);
  } }
  // in depth order: duplicate-slot offsets of the exact tile lists (the
  // backward's record slots; Gaussian -> first slot), and with sort bins the
  // bin-pair offsets -- their down-sweep writes the pairs, after the binning
  // buffer exists
  auto queue_scan = [&](const PublishJob& pj) -> int {
    StageTimer T(2, s);
    if (bshift) {  // block sums of (list length, bins) in depth order; k_duplicate_bins finishes the scan
      STAGE(a, s, packed_scan_blocks(at<uint32_t>(geom, GL.tb), 1, depth_order, (size_t)a.P,
                                     at<uint32_t>(geom, GL.bsum), s, scan_sup ? at<uint2>(geom, GL.bsup) : nullptr,
                                     pj));
    } else {
      STAGE(a, s, exclusive_scan_gather(&at<ListRec>(geom, GL.lrec)->w.w, depth_order, (size_t)a.P,
                                        at<uint32_t>(geom, GL.offs), at<uint32_t>(geom, GL.slot_start),
                                        at<uint32_t>(geom, GL.bsum), at<uint32_t>(geom, GL.counter), s,
                                        sizeof(ListRec) / 4));
    }
    return WGSR_OK;
  };
  if (int e = queue_scan(pub)) return e;
  // the predicted binning buffer, allocated while the GPU works
  BinningGuess& bg = binning_guess();
  void* binning = nullptr;
  size_t binning_have = 0;
  if (bg.P == a.P && bg.W == a.W && bg.H == a.H && bg.bshift == bshift && bg.bytes > 0) {
    binning_have = bg.bytes + bg.bytes / 16;
    binning = call_alloc(binning_alloc, ctx, binning_have);
    if (!binning) binning_have = 0;
  }
  const uint32_t* host_counter = hc.buf;
  uint4 rec = make_uint4(0u, 0u, 0u, 0u);
  bool published_ok = true;
  if (mailbox) {
    // spin on the published word; every 1024 polls the stream is checked,
    // so a failed stream ends the wait (and a publish that never became
    // visible falls back to a copy)
    // (one aligned 16-byte load: the record is written by one 16-byte store)
    auto poll = [&]() {
      asm volatile("" ::: "memory");  // (a fresh load every poll: the GPU writes the record)
      const __m128i v = _mm_load_si128(reinterpret_cast<const __m128i*>(const_cast<const uint4*>(hc.mbox)));
      _mm_storeu_si128(reinterpret_cast<__m128i*>(&rec), v);
      return (rec.x >> 8) == want;
    };
    uint32_t polls = 0;
    while (!poll()) {
      _mm_pause();
      if ((++polls & 1023u) == 0) {
        const hipError_t q = hipStreamQuery(s);
        if (q == hipErrorNotReady) continue;
        HIPCHK(q);
        // the stream is done: the record may still be in flight to host
        // memory (a posted write) -- a few more polls before giving up on it
        bool seen = false;
        for (int k = 0; k < (1 << 16) && !(seen = poll()); ++k) _mm_pause();
        if (seen) break;
        hc.mbox = nullptr;  // (not visible on this system: copies from now on)
        break;
      }
    }
    if (hc.mbox && (rec.x & 0x80u)) published_ok = false;  // a count beyond 32 bits: the block itself
    if (!hc.mbox || !published_ok) {
      HIPCHK(hipMemcpyAsync(hc.buf, counter, kCounterBytes, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
    }
  } else {
    HIPCHK(hipEventSynchronize(hc.ev));
  }
  sync_on_error.armed = false;
  // upstream num_rendered, exact (Gaussian, tile) pairs (<= N_rect), (Gaussian, bin) pairs
  size_t N_rect = 0, N = 0, N_bin = 0;
  uint32_t host_flags = 0;
  const bool published = mailbox && hc.mbox && published_ok;
  if (published) {
    host_flags = rec.x & 0x7Fu;
    N_rect = rec.y;
    N = rec.z;
    N_bin = rec.w;
  } else {
    const uint64_t* partial = reinterpret_cast<const uint64_t*>(host_counter + 4);
    for (int i = 0; i < kRectPairLanes; ++i) {
      N_rect += partial[i];
      N += partial[kRectPairLanes + i];
      N_bin += partial[2 * kRectPairLanes + i];
    }
    host_flags = host_counter[1];
  }
  if (bin_depth && N_bin > bin_depth_max_avg() * (size_t)bins.n) {
    // bins too full for one LDS-resident sort each: the Gaussian-level depth
    // sort after all (queued now, with its scratch zeroed and the scan redone
    // in depth order)
    bin_depth = false;
    StageTimer T(1, s);
    HIPCHK(hipMemsetAsync(at<uint32_t>(geom, GL.hist) + depth_sort_sup_offset_words((size_t)a.P), 0,
                          4 * depth_sort_sup_words((size_t)a.P), s));
    STAGE(a, s, launch_depth_sort(at<uint32_t>(geom, GL.dkey), at<uint32_t>(geom, GL.dkey_alt),
                                  at<uint32_t>(geom, GL.dval), at<uint32_t>(geom, GL.dval_alt), (size_t)a.P,
                                  counter + kDepthRangeOffset / 4, counter + 2, at<uint32_t>(geom, GL.hist), s));
    depth_order = at<uint32_t>(geom, GL.dval_alt);
    if (scan_sup)
      HIPCHK(hipMemsetAsync(at<uint2>(geom, GL.bsup), 0,
                            sizeof(uint2) * kScanSupStride * packed_scan_supers((size_t)a.P), s));
    if (int e = queue_scan(PublishJob{})) return e;
  }
  if (!full_depth && !bin_depth) {
    // depths spanning more than the three passes' bits: one more stable pass
    // over the bits above them, then the scan again in the final order
    // (the published counts carry no key range: the bins-too-full switch
    // above reads the block, rarely)
    if (published) {
      HIPCHK(hipMemcpyAsync(hc.buf, counter, kCounterBytes, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
    }
    const uint32_t* rw = host_counter + kDepthRangeOffset / 4;
    uint32_t hi = 0, nlo = 0;
    for (int i = 0; i < kRectPairLanes; ++i) {
      hi = rw[i] > hi ? rw[i] : hi;
      nlo = rw[kRectPairLanes + i] > nlo ? rw[kRectPairLanes + i] : nlo;
    }
    const DepthKeyPlan pl = depth_key_plan(hi, ~nlo);
    if (pl.extra_bits > 0) {
      bool alt = false;
      StageTimer T(1, s);
      STAGE(a, s, radix_sort_pairs(at<uint32_t>(geom, GL.dkey_alt), at<uint32_t>(geom, GL.dkey),
                                   at<uint32_t>(geom, GL.dval_alt), at<uint32_t>(geom, GL.dval), false, (size_t)a.P,
                                   pl.extra_shift, pl.R, at<uint32_t>(geom, GL.hist), at<uint32_t>(geom, GL.totals),
                                   s, &alt));
      depth_order = at<uint32_t>(geom, alt ? GL.dval : GL.dval_alt);
      if (scan_sup)
        HIPCHK(hipMemsetAsync(at<uint2>(geom, GL.bsup), 0,
                              sizeof(uint2) * kScanSupStride * packed_scan_supers((size_t)a.P), s));
      if (int e = queue_scan(PublishJob{})) return e;
    }
  }
  g_depth_order_off = depth_order ? (int64_t)(reinterpret_cast<const uint8_t*>(depth_order) -
                                              static_cast<const uint8_t*>(geom))
                                  : (int64_t)-1;
  if (host_flags && a.prefiltered)
    return set_error(WGSR_EINVAL, "Error: a prefiltered Gaussian lies behind the near plane");
  if (N > N_rect) return set_error(WGSR_EHIP, "internal: exact tile lists exceed the rectangles");
  if (N_bin > N_rect) return set_error(WGSR_EHIP, "internal: bin pairs exceed the rectangles");

  // the binning layout is sized by upstream's num_rendered (returned to the
  // caller and handed back to the backward), so both sides agree on it; with
  // sort bins the per-tile lists follow it (2^2s entries per bin pair)
  const BinLayout BL(N_rect);
  const size_t lists_bytes = bshift ? align256(4 * ((size_t)N_bin << (2 * bshift))) : 0;
  // per-bin depth sort: scratch of the bins beyond one LDS tile (two uint2
  // ping-pong arrays; not the list region, which the same kernel now writes)
  const size_t bds_bytes = bin_depth ? align256(16 * (size_t)N_bin) : 0;
  const size_t binning_bytes = BL.total + lists_bytes + bds_bytes;
  bg.P = a.P; bg.W = a.W; bg.H = a.H; bg.bshift = bshift; bg.bytes = binning_bytes;
  // the exact size is allocated only without (or beyond) a prediction; a
  // predicted buffer that is large enough is used as it is (the layout only
  // needs binning_bytes of it), so a callback is never asked twice for a
  // buffer it has to keep
  if (binning_bytes > binning_have) {
    binning = call_alloc(binning_alloc, ctx, binning_bytes);
    if (!binning && binning_bytes) return set_error(WGSR_EALLOC, "binning buffer allocation failed");
  }
  uint32_t* lists = bshift ? at<uint32_t>(binning, BL.total) : at<uint32_t>(binning, BL.point_g);
  // (the per-bin depth sort gathers its keys from the Gaussians' depth keys)
  const uint32_t* gdep = bin_depth ? at<uint32_t>(geom, GeomLayout((size_t)a.P).dkey) : nullptr;
  void* bds_scratch = bin_depth ? static_cast<void*>(at<char>(binning, BL.total + lists_bytes)) : nullptr;
  uint2* ranges = at<uint2>(image, IL.ranges);
  // sorted pairs: (Gaussian, bin) pairs, or with bin shift 0 the exact
  // (Gaussian, tile) pairs themselves
  const size_t NL = bshift ? N_bin : N;
  if (NL > 0) {
    const int bits = bshift ? (num_bits((uint32_t)bins.n) > 0 ? num_bits((uint32_t)bins.n) : 1) : tile_sort_bits(grid);
    // the LSD sort alternates buffers every pass: start the payload in the
    // buffer that makes it end in point_g
    const bool odd = radix_passes(0, bits) % 2 == 1;
    uint32_t* vin = at<uint32_t>(binning, odd ? BL.slot_g : BL.point_g);
    uint32_t* valt = at<uint32_t>(binning, odd ? BL.point_g : BL.slot_g);
    // the bin sort's superblock sums are zeroed by k_duplicate_bins (no memset launch)
    size_t bs_off = 0;
    const size_t bs_words = bshift ? sort_sup_words(NL, 0, bits, &bs_off) : 0;
    ZeroJob zb{};
    if (bs_words) {
      zb.p[0] = reinterpret_cast<float*>(at<uint32_t>(binning, BL.hist) + bs_off);
      zb.n[0] = bs_words;
      zb.count = 1;
    }
    { StageTimer T(3, s);
    if (bshift) {
      // (the backward's record flags live on the exact slots: zeroed here too)
      STAGE(a, s, launch_duplicate_bins(a, geom, depth_order, bshift, at<uint8_t>(binning, BL.flag),
                                        at<uint32_t>(binning, BL.key), vin, scan_sup, zb,
                                        at<uint32_t>(image, IL.meta), s));
    } else {
      STAGE(a, s, launch_duplicate(a, geom, depth_order, (uint32_t)a.P, at<uint32_t>(binning, BL.key), vin,
                                   at<uint8_t>(binning, BL.flag), s));
    } }
    bool talt = false, bounds_done = false;
    // a one-pass bin sort also hands back each bin's [start, end): into the
    // tile_m region (16 B per tile; the forward render writes tile_m later)
    uint2* bin_bounds = (bshift && (size_t)8 << bits <= (size_t)16 * grid.nt) ? at<uint2>(image, IL.tile_m) : nullptr;
    { StageTimer T(4, s);
    STAGE(a, s, radix_sort_pairs(at<uint32_t>(binning, BL.key), at<uint32_t>(binning, BL.key_alt), vin, valt, false,
                                 NL, 0, bits, at<uint32_t>(binning, BL.hist), at<uint32_t>(binning, BL.totals), s,
                                 &talt, bin_bounds, &bounds_done, bs_words != 0)); }
    // the Gaussian ids are the payload; the backward recomputes each pair's
    // record slot from (Gaussian, tile) instead of carrying it through the sort
    if (talt != odd) return set_error(WGSR_EHIP, "internal: list sort parity");
    const uint32_t* sorted_keys = at<uint32_t>(binning, talt ? BL.key_alt : BL.key);
    const uint32_t* sorted_gid = at<uint32_t>(binning, BL.point_g);
    if (bin_depth) {
      // each bin by depth, into the spare key / payload buffers; scratch for
      // bins beyond one LDS tile: the list region (>= 16 NL bytes)
      // ... and emits the per-tile lists and ranges itself (no k_expand_bins)
      StageTimer T(4, s);
      uint32_t* okeys = at<uint32_t>(binning, talt ? BL.key : BL.key_alt);
      uint32_t* ogid = at<uint32_t>(binning, BL.slot_g);
      const bool emit = bds_emit(bshift);
      STAGE(a, s, launch_bin_depth_sort(a, sorted_keys, sorted_gid, (uint32_t)NL, bshift, at<uint2>(image, IL.tile_m),
                                        bounds_done, gdep, okeys, ogid, bds_scratch, s, emit ? lists : nullptr,
                                        ranges, at<uint32_t>(image, IL.tile_len), at<uint32_t>(image, IL.meta)));
      bounds_done = true;
      if (!emit) {
        sorted_keys = okeys;
        sorted_gid = ogid;
      }
    }
    StageTimer T(5, s);
    if (bin_depth && bds_emit(bshift)) {
      // (lists and ranges written by the per-bin depth sort)
    } else if (bshift) {
      STAGE(a, s, launch_expand_bins(a, sorted_keys, sorted_gid, (uint32_t)NL, bshift,
                                     at<uint2>(image, IL.tile_m), bounds_done, lists, ranges,
                                     at<uint32_t>(image, IL.tile_len), at<uint32_t>(image, IL.meta), s));
    } else {
      STAGE(a, s, launch_ranges(sorted_keys, (uint32_t)NL, grid.nt, ranges, at<uint32_t>(image, IL.tile_len),
                                at<uint32_t>(image, IL.meta), s));
    }
  } else {
    StageTimer T(5, s);  // every list is empty
    STAGE(a, s, launch_ranges(nullptr, 0u, grid.nt, ranges, at<uint32_t>(image, IL.tile_len),
                              at<uint32_t>(image, IL.meta), s));
  }
  const uint32_t* sorted_g = lists;
  { StageTimer T(6, s);
  STAGE(a, s, launch_render_fwd(a, ranges, sorted_g, geom,
                                out_color, out_depth, out_opacity, at<float>(image, IL.final_T),
                                at<uint32_t>(image, IL.n_contrib), n_touched, at<uint32_t>(image, IL.tile_m), s)); }
  *num_rendered = (int64_t)N_rect;
  return WGSR_OK;
}

int wgsr_check_tile_lists(const wgsr_raster_args* args, int64_t num_rendered, const void* binning, const void* image,
                          uint32_t* bad, void* stream) {
  g_err[0] = 0;
  if (int e = validate(args)) return e;
  if (!bad || !image || num_rendered < 0 || (num_rendered > 0 && !binning))
    return set_error(WGSR_EINVAL, "wgsr_check_tile_lists: missing buffers");
  if (args->P == 0 || num_rendered == 0) return WGSR_OK;
  HIPCHK(launch_check_tile_lists(*args, bin_shift(*args), (uint64_t)num_rendered, binning, image, bad,
                                 (hipStream_t)stream));
  return WGSR_OK;
}

size_t wgsr_binning_bytes_cap(const wgsr_raster_args* args, int64_t cap) {
  if (!args || cap < 0) return 0;
  const int bshift = bin_shift(*args);
  const size_t C = (size_t)cap;
  return BinLayout(C).total + align256(4 * (C << (2 * bshift))) + align256(16 * C);
}

// Capacity mode (wgsr.h): the forward above without its one host wait.  The
// buffers are sized for `cap` (Gaussian, tile) rectangle pairs -- upstream's
// num_rendered, which bounds the exact pairs and the bin pairs too -- and the
// device-side counts take the place of the host's: k_cap_counts turns the
// counter partials into counts[] and the overflow flag, the bin sort reads
// its key count from counts[4], and an overflow (N_rect > cap) leaves the
// render backward a zero fill (ImageLayout::meta[1]).  Only the default
// configuration: sort bins with the per-bin depth sort and the one-pass bin
// sort that hands back the bin bounds.  Every launch is stream-ordered
// device work with host-known sizes, so the call can be captured in a HIP
// graph (the next forward's counter block is zeroed by a memset here, not by
// the parity scheme of the host-synchronised forward).
int wgsr_rasterize_forward_cap(const wgsr_raster_args* args, int64_t cap, wgsr_alloc_fn geom_alloc,
                               wgsr_alloc_fn binning_alloc, wgsr_alloc_fn image_alloc, void* ctx, float* out_color,
                               float* out_depth, float* out_opacity, int32_t* radii, int32_t* n_touched,
                               uint32_t* counts, void* stream) {
  g_err[0] = 0;
  if (int e = validate(args)) return e;
  const wgsr_raster_args& a = *args;
  hipStream_t s = (hipStream_t)stream;
  if (cap <= 0 || cap >= ((int64_t)1 << 30)) return set_error(WGSR_EINVAL, "capacity %lld out of range", (long long)cap);
  if (!counts) return set_error(WGSR_EINVAL, "missing counts buffer");
  if (a.prefiltered) return set_error(WGSR_EINVAL, "capacity mode: prefiltered is not supported");
  const size_t HW = (size_t)a.W * a.H;
  if (a.P == 0) {
    call_alloc(geom_alloc, ctx, 0);
    call_alloc(binning_alloc, ctx, 0);
    call_alloc(image_alloc, ctx, 0);
    // (kernel nodes, not memset nodes: see launch_zero_u32)
    HIPCHK(launch_zero_u32(reinterpret_cast<uint32_t*>(out_color), 3 * HW, s));
    HIPCHK(launch_zero_u32(reinterpret_cast<uint32_t*>(out_depth), HW, s));
    HIPCHK(launch_zero_u32(reinterpret_cast<uint32_t*>(out_opacity), HW, s));
    HIPCHK(launch_zero_u32(counts, 5, s));
    return WGSR_OK;
  }
  const Grid grid(a);
  const int bshift = bin_shift(a);
  if (!bshift || !depth_sort_bins(a, bshift))
    return set_error(WGSR_EINVAL, "capacity mode needs sort bins with the per-bin depth sort");
  const Bins bins(grid.gx, grid.gy, bshift);
  const int bits = num_bits((uint32_t)bins.n) > 0 ? num_bits((uint32_t)bins.n) : 1;
  if (!((size_t)8 << bits <= (size_t)16 * grid.nt))
    return set_error(WGSR_EINVAL, "capacity mode: the bin bounds do not fit the tile_m region");
  const GeomLayout GL((size_t)a.P);
  const ImageLayout IL(a.W, a.H);
  void* geom = call_alloc(geom_alloc, ctx, GL.total);
  if (!geom) return set_error(WGSR_EALLOC, "geometry buffer allocation failed");
  void* image = call_alloc(image_alloc, ctx, IL.total);
  if (!image) return set_error(WGSR_EALLOC, "image buffer allocation failed");
  const size_t C = (size_t)cap;
  const BinLayout BL(C);
  const size_t lists_bytes = align256(4 * (C << (2 * bshift)));
  const size_t binning_bytes = BL.total + lists_bytes + align256(16 * C);
  void* binning = call_alloc(binning_alloc, ctx, binning_bytes);
  if (!binning) return set_error(WGSR_EALLOC, "binning buffer allocation failed");
  uint32_t* lists = at<uint32_t>(binning, BL.total);
  const uint32_t* gdep = at<uint32_t>(geom, GL.dkey);
  void* bds_scratch = at<char>(binning, BL.total + lists_bytes);
  uint32_t* counter = at<uint32_t>(geom, GL.counter);
  uint32_t* meta = at<uint32_t>(image, IL.meta);
  // the counter block zeroed by a kernel node (a captured memset node did not
  // reliably zero it: launch_zero_u32)
  HIPCHK(launch_zero_u32(counter, kCounterBytes / 4, s));
  ZeroJob zj{};
  const bool scan_sup = true;
  if (scan_sup) {
    zj.p[zj.count] = at<float>(geom, GL.bsup);
    zj.n[zj.count++] = 2 * kScanSupStride * packed_scan_supers((size_t)a.P);
  }
  { StageTimer T(0, s);
  STAGE(a, s, launch_preprocess(a, geom, radii, n_touched, counter + 1,
                                reinterpret_cast<unsigned long long*>(counter + 4), bshift, zj, s, meta)); }
  STAGE(a, s, launch_cap_counts(reinterpret_cast<const unsigned long long*>(counter + 4), (uint64_t)C, (uint64_t)C,
                                counts, meta, s));
  { StageTimer T(2, s);  // block sums of (list length, bins) in index order
  STAGE(a, s, packed_scan_blocks(at<uint32_t>(geom, GL.tb), 1, nullptr, (size_t)a.P, at<uint32_t>(geom, GL.bsum), s,
                                 scan_sup ? at<uint2>(geom, GL.bsup) : nullptr)); }
  const bool odd = radix_passes(0, bits) % 2 == 1;
  uint32_t* vin = at<uint32_t>(binning, odd ? BL.slot_g : BL.point_g);
  uint32_t* valt = at<uint32_t>(binning, odd ? BL.point_g : BL.slot_g);
  size_t bs_off = 0;
  const size_t bs_words = sort_sup_words(C, 0, bits, &bs_off);
  ZeroJob zb{};
  if (bs_words) {
    zb.p[0] = reinterpret_cast<float*>(at<uint32_t>(binning, BL.hist) + bs_off);
    zb.n[0] = bs_words;
    zb.count = 1;
  }
  { StageTimer T(3, s);  // (pairs past the capacity are not written; exact-slot flags likewise)
  STAGE(a, s, launch_duplicate_bins(a, geom, nullptr, bshift, at<uint8_t>(binning, BL.flag),
                                    at<uint32_t>(binning, BL.key), vin, scan_sup, zb, at<uint32_t>(image, IL.meta), s,
                                    (uint32_t)C, (uint32_t)C)); }
  bool talt = false, bounds_done = false;
  uint2* bin_bounds = at<uint2>(image, IL.tile_m);
  { StageTimer T(4, s);
  STAGE(a, s, radix_sort_pairs(at<uint32_t>(binning, BL.key), at<uint32_t>(binning, BL.key_alt), vin, valt, false, C,
                               0, bits, at<uint32_t>(binning, BL.hist), at<uint32_t>(binning, BL.totals), s, &talt,
                               bin_bounds, &bounds_done, bs_words != 0, counts + 4)); }
  if (talt != odd) return set_error(WGSR_EHIP, "internal: list sort parity");
  if (!bounds_done) return set_error(WGSR_EHIP, "internal: capacity mode without the sort's bin bounds");
  const uint32_t* sorted_keys = at<uint32_t>(binning, talt ? BL.key_alt : BL.key);
  const uint32_t* sorted_gid = at<uint32_t>(binning, BL.point_g);
  uint2* ranges = at<uint2>(image, IL.ranges);
  const bool emit = bds_emit(bshift);
  uint32_t* okeys = at<uint32_t>(binning, talt ? BL.key : BL.key_alt);
  uint32_t* ogid = at<uint32_t>(binning, BL.slot_g);
  { StageTimer T(4, s);
  STAGE(a, s, launch_bin_depth_sort(a, sorted_keys, sorted_gid, (uint32_t)C, bshift, bin_bounds, true, gdep, okeys,
                                    ogid, bds_scratch, s, emit ? lists : nullptr, ranges,
                                    at<uint32_t>(image, IL.tile_len), meta)); }
  if (!emit) { StageTimer T(5, s);
    STAGE(a, s, launch_expand_bins(a, okeys, ogid, (uint32_t)C, bshift, bin_bounds, true, lists, ranges,
                                   at<uint32_t>(image, IL.tile_len), meta, s));
  }
  g_depth_order_off = -1;
  { StageTimer T(6, s);
  STAGE(a, s, launch_render_fwd(a, ranges, lists, geom, out_color, out_depth, out_opacity, at<float>(image, IL.final_T),
                                at<uint32_t>(image, IL.n_contrib), n_touched, at<uint32_t>(image, IL.tile_m), s)); }
  return WGSR_OK;
}

}  // extern "C"

namespace wgsr {
namespace {
// Backward render of one view: per-pair partial records (scratch) + the
// "record written" flags in the binning buffer.  Shared by the full backward
// and the view-sharded records path.
int render_backward_pairs(const wgsr_raster_args& a, const void* geom, void* binning, void* image,
                          int64_t num_rendered, const float* dL_dcolor, const float* dL_ddepth,
                          wgsr_alloc_fn scratch_alloc, void* ctx, const ZeroJob& zero, hipStream_t s,
                          float4** partial_out, uint8_t** pflag_out) {
  if (!geom || !image || (num_rendered > 0 && !binning))
    return set_error(WGSR_EINVAL, "missing forward state buffers");
  const Grid grid(a);
  const ImageLayout IL(a.W, a.H);
  const size_t N = (size_t)num_rendered;
  // scratch: 48-byte partial record per pair.  The 1-byte "record written"
  // flag per pair lives in the binning buffer, zeroed by the forward's
  // k_duplicate (render_bwd sets it for the same pairs on every backward call
  // of that forward, so repeated backwards agree).
  const size_t rec_bytes = align256(48 * N);
  void* scratch = call_alloc(scratch_alloc, ctx, rec_bytes);
  if (!scratch && rec_bytes) return set_error(WGSR_EALLOC, "backward scratch allocation failed");
  float4* partial = N > 0 ? static_cast<float4*>(scratch) : nullptr;
  const BinLayout BL(N);
  uint8_t* pflag = N > 0 ? at<uint8_t>(binning, BL.flag) : nullptr;
  if (N > 0) {
    StageTimer T(7, s);
    uint32_t* order = at<uint32_t>(image, IL.order_bwd);
    STAGE(a, s, launch_tile_order(at<uint32_t>(image, IL.tile_m), grid.nt, order, s));
    // the tile lists: point_g, or with sort bins the region after the sized
    // layout -- the forward records which in the image buffer's meta word
    STAGE(a, s, launch_render_bwd(a, at<uint2>(image, IL.ranges), order, at<uint32_t>(image, IL.meta),
                                  at<uint32_t>(binning, BL.point_g), at<uint32_t>(binning, BL.total), geom,
                                  at<float>(image, IL.final_T),
                                  at<uint32_t>(image, IL.n_contrib), dL_dcolor, dL_ddepth, partial, pflag, zero,
                                  s));
  } else {
    // no render backward to carry the zero fill
    for (int j = 0; j < zero.count; ++j) HIPCHK(hipMemsetAsync(zero.p[j], 0, sizeof(float) * zero.n[j], s));
  }
  *partial_out = partial;
  *pflag_out = pflag;
  return WGSR_OK;
}
}  // namespace
}  // namespace wgsr

extern "C" {

int wgsr_rasterize_backward(const wgsr_raster_args* args, const int32_t* radii, const void* geom,
                            void* binning, void* image, int64_t num_rendered, const float* dL_dcolor,
                            const float* dL_ddepth, wgsr_alloc_fn scratch_alloc, void* ctx, float* dL_dmeans2D,
                            float* dL_dcolors, float* dL_dopacity, float* dL_dmeans3D, float* dL_dcov3D,
                            float* dL_dsh, float* dL_dscales, float* dL_drotations, float* dL_dtau, void* stream) {
  g_err[0] = 0;
  if (int e = validate(args)) return e;
  const wgsr_raster_args& a = *args;
  if (a.P == 0) return WGSR_OK;
  hipStream_t s = (hipStream_t)stream;
  float4* partial = nullptr;
  uint8_t* pflag = nullptr;
  // the render backward zero-fills the outputs and k_gauss_bwd_compact writes
  // only the rows of the Gaussians that received gradient
  ZeroJob zero{};
  {
    const uint64_t P = (uint64_t)a.P;
    auto add = [&](float* p, uint64_t n) {
      if (p && n) { zero.p[zero.count] = p; zero.n[zero.count] = n; ++zero.count; }
    };
    add(dL_dmeans2D, 3 * P); add(dL_dcolors, 3 * P); add(dL_dopacity, P); add(dL_dmeans3D, 3 * P);
    add(dL_dcov3D, 6 * P); add(a.shs ? dL_dsh : nullptr, 3 * (uint64_t)a.M * P); add(dL_dscales, 3 * P);
    add(dL_drotations, 4 * P); add(dL_dtau, 6 * P);
    for (int j = 0; j < zero.count; ++j)
      if (reinterpret_cast<uintptr_t>(zero.p[j]) & 3) return set_error(WGSR_EINVAL, "gradient outputs must be 4-byte aligned");
  }
  if (int e = render_backward_pairs(a, geom, binning, image, num_rendered, dL_dcolor, dL_ddepth, scratch_alloc, ctx,
                                    zero, s, &partial, &pflag))
    return e;
  StageTimer T(8, s);
  STAGE(a, s, launch_gauss_bwd(a, geom, partial, pflag, at<uint32_t>(image, ImageLayout(a.W, a.H).meta), dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D,
                               dL_dsh, dL_dscales, dL_drotations, dL_dtau, s));
  return WGSR_OK;
}

int wgsr_pack_view_camera(const wgsr_raster_args* args, float* camera_row, void* stream) {
  g_err[0] = 0;
  if (!args || !camera_row || !args->viewmatrix || !args->projmatrix || !args->projmatrix_raw || !args->campos)
    return set_error(WGSR_EINVAL, "wgsr_pack_view_camera: missing camera tensor");
  HIPCHK(launch_pack_camera(*args, camera_row, (hipStream_t)stream));
  return WGSR_OK;
}

int wgsr_rasterize_backward_records(const wgsr_raster_args* args, const int32_t* radii, const void* geom,
                                    void* binning, void* image, int64_t num_rendered, const float* dL_dcolor,
                                    const float* dL_ddepth, wgsr_alloc_fn scratch_alloc, void* ctx, int P_pad,
                                    float* records, void* stream) {
  g_err[0] = 0;
  if (int e = validate(args)) return e;
  const wgsr_raster_args& a = *args;
  if (P_pad < a.P) return set_error(WGSR_EINVAL, "P_pad (%d) < P (%d)", P_pad, a.P);
  if (P_pad > 0 && !records) return set_error(WGSR_EINVAL, "missing records buffer");
  hipStream_t s = (hipStream_t)stream;
  float4* partial = nullptr;
  uint8_t* pflag = nullptr;
  if (a.P > 0) {
    if (int e = render_backward_pairs(a, geom, binning, image, num_rendered, dL_dcolor, dL_ddepth, scratch_alloc,
                                      ctx, ZeroJob{}, s, &partial, &pflag))
      return e;
  }
  StageTimer T(8, s);
  STAGE(a, s, launch_view_records(a, radii, geom, partial, pflag, P_pad, records, s));
  return WGSR_OK;
}

int wgsr_gauss_backward_views_blocks(int lo, int hi) { return gauss_bwd_views_blocks(lo, hi); }

int wgsr_gauss_backward_views(const wgsr_raster_args* params, int lo, int hi, int n_views, const float* cameras,
                              const float* records, int64_t record_view_stride, float* dL_dmeans3D, float* dL_dsh,
                              float* dL_dopacity, float* dL_dscales, float* dL_drotations, float* tau_partials,
                              float* stats, void* stream) {
  g_err[0] = 0;
  if (!params) return set_error(WGSR_EINVAL, "null args");
  const wgsr_raster_args& a = *params;
  if (lo < 0 || hi < lo || hi > a.P) return set_error(WGSR_EINVAL, "shard [%d, %d) outside [0, %d)", lo, hi, a.P);
  if (n_views < 0) return set_error(WGSR_EINVAL, "negative view count");
  if (hi == lo || n_views == 0) {
    if (hi > lo) return set_error(WGSR_EINVAL, "a non-empty shard needs at least one view");
    return WGSR_OK;
  }
  if (!a.means3D || !a.scales || !a.rotations)
    return set_error(WGSR_EINVAL, "the view-sharded backward needs means3D, scales and rotations "
                                  "(cov3D_precomp is not supported)");
  if (a.shs && (a.M <= 0 || a.M > 16 || a.D < 0 || a.D > 3 || (a.D + 1) * (a.D + 1) > a.M))
    return set_error(WGSR_EINVAL, "invalid SH configuration (degree %d, %d coefficients)", a.D, a.M);
  if (!cameras || !records) return set_error(WGSR_EINVAL, "missing camera table or records");
  if (record_view_stride < (int64_t)(hi - lo) * WGSR_VIEW_RECORD_FLOATS || record_view_stride % 4)
    return set_error(WGSR_EINVAL, "record_view_stride must be a multiple of 4 and >= %d",
                     (hi - lo) * WGSR_VIEW_RECORD_FLOATS);
  if (!dL_dmeans3D || !dL_dopacity || !dL_dscales || !dL_drotations || (a.shs && !dL_dsh))
    return set_error(WGSR_EINVAL, "missing gradient output");
  hipStream_t s = (hipStream_t)stream;
  StageTimer T(8, s);
  HIPCHK(launch_gauss_bwd_views(a, lo, hi, n_views, cameras, records, record_view_stride, dL_dmeans3D, dL_dsh,
                                dL_dopacity, dL_dscales, dL_drotations, tau_partials, stats, s));
  if (a.debug) {
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipGetLastError());
  }
  return WGSR_OK;
}

int wgsr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                      uint8_t* present, void* stream) {
  g_err[0] = 0;
  if (P < 0) return set_error(WGSR_EINVAL, "negative point count");
  HIPCHK(launch_mark_visible(P, means3D, viewmatrix, projmatrix, present, (hipStream_t)stream));
  return WGSR_OK;
}

int wgsr_dist_cuda2(int P, const float* points, float* out, wgsr_alloc_fn scratch_alloc, void* ctx, void* stream) {
  g_err[0] = 0;
  if (P < 0) return set_error(WGSR_EINVAL, "negative point count");
  if (P == 0) return WGSR_OK;
  void* scratch = call_alloc(scratch_alloc, ctx, knn_scratch_bytes(P));
  if (!scratch) return set_error(WGSR_EALLOC, "distCUDA2 scratch allocation failed");
  StageTimer T(9, (hipStream_t)stream);
  HIPCHK(launch_dist_cuda2(P, points, out, scratch, (hipStream_t)stream));
  return WGSR_OK;
}

}  // extern "C"
