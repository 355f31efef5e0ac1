// Host-side launchers shared between the translation units of libwgsr.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wgsr.h"

namespace wgsr {

// Stable LSD radix sort on bits [begin_bit, end_bit) (8-bit digits, onesweep).
// Input in keys/vals (vals ignored if vals_iota: value = input position); the
// result lands in keys_alt/vals_alt when *result_in_alt, else in keys/vals.
// Scratch: status >= sort_status_bytes(n), totals >= kSortTotalsBytes.
// number of passes radix_sort_pairs makes over [begin_bit, end_bit) (the
// result alternates buffers each pass).  digit_bounds: when the sort runs as
// one wide pass over bits [0, end_bit), each digit's [start, end) in the
// sorted output is written there (*bounds_done = true).
int radix_passes(int begin_bit, int end_bit);
hipError_t radix_sort_pairs(uint32_t* keys, uint32_t* keys_alt, uint32_t* vals, uint32_t* vals_alt, bool vals_iota,
                            size_t n, int begin_bit, int end_bit, uint32_t* status, uint32_t* totals,
                            hipStream_t stream, bool* result_in_alt,
                            uint2* digit_bounds = nullptr, bool* bounds_done = nullptr, bool sup_zeroed = false,
                            const uint32_t* ndev = nullptr);
// (ndev: capacity mode -- n is the capacity the grid is sized for, *ndev the
// live key count, read on the device; reduce-then-scan / wide schedules only)
// words of `status` a reduce-then-scan sort accumulates superblock sums in
// (zero before the sort; 0 = none), at *offset_words
size_t sort_sup_words(size_t n, int begin_bit, int end_bit, size_t* offset_words);

// Depth sort (DepthKeyPlan): three stable passes over key'' of the depth keys
// in `keys` (values = input positions); range = the counter block's range
// words (kDepthRangeOffset), range2 = two words for their reduction, scratch = depth_sort_status_bytes(n) bytes whose
// superblock sums (depth_sort_sup_offset_words / depth_sort_sup_words) are
// zero.  Result: rank -> position in vals_alt; keys_alt holds key'' when the
// plan leaves extra_bits (the caller's fix-up pass sorts those), else
// garbage.  keys and vals are clobbered.
hipError_t launch_depth_sort(uint32_t* keys, uint32_t* keys_alt, uint32_t* vals, uint32_t* vals_alt, size_t n,
                             const uint32_t* range, uint32_t* range2, uint32_t* scratch, hipStream_t s);

// out[i] = sum_{j<i} vals[idx ? idx[j] : j]  (i in [0, n]; out has n + 1
// entries), optional scatter_out[idx[i]] = out[i]; *total_out = out[n].
hipError_t exclusive_scan_gather(const uint32_t* vals, const uint32_t* idx, size_t n, uint32_t* out,
                                 uint32_t* scatter_out, uint32_t* bsum, uint32_t* total_out, hipStream_t stream,
                                 uint32_t stride = 1);

// First two steps of a scan of packed (lo 16 | hi 16) values gathered as
// packed[idx[i]]: bsum[b] = exclusive prefix (lo sums, hi sums) of block b of
// kScanTile elements, bsum[blocks] = totals.  bsum: 8 x (blocks + 1) bytes.
// With bsup (zeroed, packed_scan_supers(n) uint2): bsum keeps the raw block
// sums and bsup[s] the sums of blocks [16 s, 16 s + 16); no prefix pass.
// The down-sweep is the caller's (k_scan_bins_down emits pairs).
// packed[idx[i] * stride]: (lo 16 | hi 16 bits) pairs gathered through idx
hipError_t packed_scan_blocks(const uint32_t* packed, uint32_t stride, const uint32_t* idx, size_t n, void* bsum,
                              hipStream_t stream,
                              void* bsup = nullptr, const PublishJob& pub = PublishJob{});

int num_bits(uint32_t n);  // bits needed to represent values in [0, n)

// thread-local error message plumbing for the C ABI
int set_error(int code, const char* fmt, ...);

struct RasterGrid {
  int gx, gy, ntiles;
};

// forward stages (raster_fwd.hip)
// rect_pairs[0..kRectPairLanes) += upstream's num_rendered contributions (rect
// areas); rect_pairs[kRectPairLanes..2 kRectPairLanes) += exact list lengths
// rect_pairs[2 kRectPairLanes..3 kRectPairLanes) += bins touched (bshift > 0;
// geometry tb[g] = exact list length | bins touched << 16)
hipError_t launch_preprocess(const wgsr_raster_args& a, void* geom, int32_t* radii, int32_t* n_touched,
                             uint32_t* err_flag, unsigned long long* rect_pairs, int bshift, const ZeroJob& zero, hipStream_t s, uint32_t* meta);
// capacity-mode forward: counter partials -> counts [N_rect, N_exact, N_bin,
// overflow, clamped N_bin] and the overflow flag into meta[1]
hipError_t launch_cap_counts(const unsigned long long* partial, uint64_t cap_rect, uint64_t cap_bin, uint32_t* counts,
                             uint32_t* meta, hipStream_t s);
// Sort bins: after packed_scan_blocks, the scan's down-sweep (slot_start[g],
// the slot flags zeroed) fused with the (bin | exact tile mask << 16,
// Gaussian) pair expansion.  Sets ImageLayout::meta[2] when the slots follow
// the Gaussian index order (depth_order null), which k_gauss_bwd_compact
// reads: then Gaussian g's slots are [slot_start[g], slot_start[g + 1]).
hipError_t launch_duplicate_bins(const wgsr_raster_args& a, void* geom, const uint32_t* depth_order, int bshift,
                                 uint8_t* pflag, uint32_t* keys, uint32_t* vals, bool bsup, const ZeroJob& zero,
                                 uint32_t* meta, hipStream_t s, uint32_t cap_slots = 0xFFFFFFFFu,
                                 uint32_t cap_pairs = 0xFFFFFFFFu);
hipError_t launch_duplicate(const wgsr_raster_args& a, const void* geom, const uint32_t* sorted_g, uint32_t P,
                            uint32_t* keys, uint32_t* slot_g, uint8_t* pflag, hipStream_t s);
// per-bin depth sort (pairs duplicated in index order): every bin's entries
// stably by depth key (gdepth: the Gaussians' depth keys, gathered through
// each bin's Gaussian ids)
// (bounds written first unless bounds_done); scratch: >= 2 NB uint2 (bins
// beyond one LDS tile).  With lists: the per-tile exact lists, ranges,
// tile_len and meta emitted straight from each sorted bin (what
// launch_expand_bins would make of it); else the sorted bins -> okeys / ogid.
// stable argsort of n <= argsort_small_max() keys in one workgroup (perm: positions)
uint32_t argsort_small_max();
hipError_t launch_argsort_small(const uint32_t* keys, uint32_t n, uint32_t* perm, hipStream_t s);
hipError_t launch_bin_depth_sort(const wgsr_raster_args& a, const uint32_t* sorted_keys, const uint32_t* sorted_g,
                                 uint32_t NB, int bshift, uint2* bounds, bool bounds_done, const uint32_t* gdepth,
                                 uint32_t* okeys, uint32_t* ogid, void* scratch, hipStream_t s,
                                 uint32_t* lists = nullptr, uint2* ranges = nullptr, uint32_t* tile_len = nullptr,
                                 uint32_t* meta = nullptr);
// per-tile exact lists out of the bin-sorted pairs: ranges / tile_len per
// tile, the lists in bin-sized regions of `lists` (2^2s x NB entries)
hipError_t launch_expand_bins(const wgsr_raster_args& a, const uint32_t* sorted_keys, const uint32_t* sorted_g,
                              uint32_t NB, int bshift, uint2* bounds, bool bounds_done, uint32_t* lists, uint2* ranges,
                              uint32_t* tile_len, uint32_t* meta, hipStream_t s);
// tile ranges of the exact (Gaussian, tile) pair sort
hipError_t launch_ranges(const uint32_t* sorted_keys, uint32_t N, int ntiles, uint2* ranges, uint32_t* len,
                         uint32_t* meta, hipStream_t s);
// the backward's launch order (tiles by deepest contributor, per XCD chunk)
hipError_t launch_tile_order(const uint32_t* work_quads, int ntiles, uint32_t* order, hipStream_t s);
hipError_t launch_render_fwd(const wgsr_raster_args& a, const uint2* ranges, const uint32_t* point_g,
                             const void* geom, float* out_color, float* out_depth,
                             float* out_opacity, float* final_T, uint32_t* n_contrib, int32_t* n_touched,
                             uint32_t* tile_m4, hipStream_t s);
// p[0..n) = 0 by a kernel (graph-capturable without a memset node)
hipError_t launch_zero_u32(uint32_t* p, size_t n, hipStream_t s);
// wgsr_check_tile_lists' kernel (lists region sizes from num_rendered and the bin shift)
hipError_t launch_check_tile_lists(const wgsr_raster_args& a, int bshift, uint64_t num_rendered, const void* binning,
                                   const void* image, uint32_t* bad, hipStream_t s);
hipError_t launch_mark_visible(int P, const float* means3D, const float* view, const float* proj, uint8_t* present,
                               hipStream_t s);

// backward stages (raster_bwd.hip)
// the tile lists: lists_bins when the forward's ImageLayout::meta word says so, else lists_exact
hipError_t launch_render_bwd(const wgsr_raster_args& a, const uint2* ranges, const uint32_t* order,
                             const uint32_t* meta, const uint32_t* lists_exact, const uint32_t* lists_bins,
                             const void* geom, const float* final_T,
                             const uint32_t* n_contrib, const float* dL_dcolor, const float* dL_ddepth,
                             float4* partial, uint8_t* pflag, const ZeroJob& zero, hipStream_t s);
// Per-Gaussian backward (k_gauss_bwd_compact): the rows of the Gaussians the
// render backward marked in gflag; the render backward zero-filled the outputs.
hipError_t launch_gauss_bwd(const wgsr_raster_args& a, const void* geom, const float4* partial, const uint8_t* pflag,
                            const uint32_t* meta, float* dL_dmeans2D, float* dL_dcolors, float* dL_dopacity,
                            float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscales, float* dL_drot,
                            float* dL_dtau, hipStream_t s);
// view-sharded backward (raster_bwd.hip, wgsr/dp.py)
hipError_t launch_view_records(const wgsr_raster_args& a, const int32_t* radii, const void* geom, const float4* partial,
                               const uint8_t* pflag, int P_pad, float* records, hipStream_t s);
hipError_t launch_pack_camera(const wgsr_raster_args& a, float* row, hipStream_t s);
int gauss_bwd_views_blocks(int lo, int hi);
hipError_t launch_gauss_bwd_views(const wgsr_raster_args& a, int lo, int hi, int nv, const float* cams,
                                  const float* records, int64_t rec_stride_floats, float* dL_dmeans3D, float* dL_dsh,
                                  float* dL_dopacity, float* dL_dscales, float* dL_drot, float* tau_blk, float* stats,
                                  hipStream_t s);

// distCUDA2 (knn.hip)
size_t knn_scratch_bytes(int P);
hipError_t launch_dist_cuda2(int P, const float* points, float* out, void* scratch, hipStream_t s);

}  // namespace wgsr
