"""ctypes binding of libwgsr.so (include/wgsr.h).

The library is the MI355X (gfx950) implementation of the two native
extensions WildGS-SLAM loads on its mapping path; this module is the only
place Python touches it.  There is deliberately no fallback: if the shared
library is missing or fails to load, every entry point raises.

Device memory comes from the torch caching allocator through the C ABI's
allocation callbacks (``wgsr_alloc_fn``), and launches go on torch's current
HIP stream, so the kernels compose with the rest of a PyTorch-ROCm program.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_PKG_ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
LIB_PATH = os.environ.get("WGSR_LIB", os.path.join(_PKG_ROOT, "lib", "libwgsr.so"))

ALLOC_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)
_fp = ctypes.c_void_p  # device pointers travel as raw addresses


class RasterArgs(ctypes.Structure):
    """Mirror of ``wgsr_raster_args``."""

    _fields_ = [
        ("P", ctypes.c_int), ("D", ctypes.c_int), ("M", ctypes.c_int),
        ("W", ctypes.c_int), ("H", ctypes.c_int),
        ("bg", _fp), ("means3D", _fp), ("colors", _fp), ("opacities", _fp),
        ("scales", _fp), ("rotations", _fp), ("cov3D_precomp", _fp), ("shs", _fp),
        ("viewmatrix", _fp), ("projmatrix", _fp), ("projmatrix_raw", _fp), ("campos", _fp),
        ("scale_modifier", ctypes.c_float), ("tan_fovx", ctypes.c_float),
        ("tan_fovy", ctypes.c_float), ("prefiltered", ctypes.c_int), ("debug", ctypes.c_int),
    ]


class AdamTensor(ctypes.Structure):
    """Mirror of ``wgsr_adam_tensor``."""

    _fields_ = [("param", _fp), ("grad", _fp), ("exp_avg", _fp), ("exp_avg_sq", _fp),
                ("numel", ctypes.c_int64), ("step_size", ctypes.c_float),
                ("bias_correction2_sqrt", ctypes.c_float), ("split_period", ctypes.c_int64),
                ("split_len", ctypes.c_int64), ("step_size_tail", ctypes.c_float)]


class GatherJob(ctypes.Structure):
    """Mirror of ``wgsr_gather_job``."""

    _fields_ = [("src", _fp), ("dst", _fp), ("row_words", ctypes.c_int64), ("src_stride_words", ctypes.c_int64),
                ("idx_offset", ctypes.c_int32), ("nrows", ctypes.c_int32)]


GATHER_MAX_JOBS = 8


class RowTensor(ctypes.Structure):
    """Mirror of ``wgsr_row_tensor``."""

    _fields_ = [("src", _fp), ("dst", _fp), ("row_bytes", ctypes.c_int64)]


class PlyColumnSet(ctypes.Structure):
    """Mirror of ``wgsr_ply_column_set``."""

    _fields_ = [("data", _fp), ("cols", ctypes.c_int), ("record_col", ctypes.POINTER(ctypes.c_int))]


class UncerParams(ctypes.Structure):
    """Mirror of ``wgsr_uncer_params``."""

    _fields_ = [("H", ctypes.c_int), ("W", ctypes.c_int), ("h", ctypes.c_int), ("w", ctypes.c_int),
                ("rgb_threshold", ctypes.c_float), ("data_rate", ctypes.c_float),
                ("ssim_weight", ctypes.c_float), ("opacity_th", ctypes.c_float),
                ("uncer_depth_mult", ctypes.c_float), ("initialization", ctypes.c_int),
                ("pre_exposed", ctypes.c_int)]


PLY_MAX_TENSORS = 8
PLY_MAX_COLS = 128
ADAM_MAX_TENSORS = 16
class GaussianBank(ctypes.Structure):
    """Mirror of ``wgsr_gaussian_bank`` (one bank of the densification SoA)."""

    _fields_ = [("xyz", _fp), ("features", _fp), ("opacity", _fp), ("scaling", _fp), ("rotation", _fp),
                ("exp_avg", _fp * 5), ("exp_avg_sq", _fp * 5), ("kf_id", _fp), ("n_obs", _fp)]


class DeformFrame(ctypes.Structure):
    """Mirror of ``wgsr_deform_frame`` (one keyframe of a map deformation)."""

    _fields_ = [("kf_id", ctypes.c_int32), ("method", ctypes.c_int32), ("T", ctypes.c_float * 16),
                ("q", ctypes.c_float * 4), ("w2c_old", ctypes.c_float * 16), ("c2w_old", ctypes.c_float * 16),
                ("K", ctypes.c_float * 9), ("H", ctypes.c_int32), ("W", ctypes.c_int32), ("depth", _fp),
                ("depth_old", _fp)]


COMPACT_MAX_TENSORS = 32

_lib = None
_lock = threading.Lock()


class LibraryMissing(RuntimeError):
    pass


def load():
    """Load libwgsr.so (after torch, so the HIP runtime is torch's)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise LibraryMissing(
                f"libwgsr.so not found at {LIB_PATH}; build it with "
                f"`make -C wildgs-slam-blackwell_amd` (or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        c_int, c_i64, c_sz = ctypes.c_int, ctypes.c_int64, ctypes.c_size_t
        P_ARGS = ctypes.POINTER(RasterArgs)
        L.wgsr_rasterize_forward.restype = c_int
        L.wgsr_rasterize_forward.argtypes = [P_ARGS, ALLOC_FN, ALLOC_FN, ALLOC_FN, ctypes.c_void_p,
                                             _fp, _fp, _fp, _fp, _fp, ctypes.POINTER(c_i64), _fp]
        L.wgsr_rasterize_backward.restype = c_int
        L.wgsr_rasterize_backward.argtypes = [P_ARGS, _fp, _fp, _fp, _fp, c_i64, _fp, _fp, ALLOC_FN,
                                              ctypes.c_void_p] + [_fp] * 9 + [_fp]
        L.wgsr_pack_view_camera.restype = c_int
        L.wgsr_pack_view_camera.argtypes = [P_ARGS, _fp, _fp]
        L.wgsr_rasterize_backward_records.restype = c_int
        L.wgsr_rasterize_backward_records.argtypes = [P_ARGS, _fp, _fp, _fp, _fp, c_i64, _fp, _fp, ALLOC_FN,
                                                      ctypes.c_void_p, c_int, _fp, _fp]
        L.wgsr_gauss_backward_views_blocks.restype = c_int
        L.wgsr_gauss_backward_views_blocks.argtypes = [c_int, c_int]
        L.wgsr_gauss_backward_views.restype = c_int
        L.wgsr_gauss_backward_views.argtypes = [P_ARGS, c_int, c_int, c_int, _fp, _fp, c_i64] + [_fp] * 7 + [_fp]
        L.wgsr_map_blocks.restype = c_int
        L.wgsr_map_blocks.argtypes = [c_i64]
        L.wgsr_gaussian_activate.restype = c_int
        L.wgsr_gaussian_activate.argtypes = [c_int] + [_fp] * 7 + [_fp]
        L.wgsr_gaussian_activate_backward_stats.restype = c_int
        L.wgsr_gaussian_activate_backward_stats.argtypes = ([c_int] + [_fp] * 6 + [ctypes.c_float] + [_fp] * 9
                                                            + [_fp])
        L.wgsr_gaussian_activate_backward.restype = c_int
        L.wgsr_gaussian_activate_backward.argtypes = [c_int] + [_fp] * 6 + [ctypes.c_float] + [_fp] * 3 + [_fp]
        L.wgsr_mapping_loss_forward.restype = c_int
        L.wgsr_mapping_loss_forward.argtypes = [c_int, c_int] + [_fp] * 6 + [ctypes.c_float, _fp, _fp, _fp]
        L.wgsr_mapping_loss_backward.restype = c_int
        L.wgsr_mapping_loss_backward.argtypes = ([c_int, c_int] + [_fp] * 6 + [ctypes.c_float] * 3 +
                                                 [_fp] * 4 + [_fp])
        U = ctypes.POINTER(UncerParams)
        L.wgsr_uncer_blocks.restype = c_int
        L.wgsr_uncer_blocks.argtypes = [c_i64]
        L.wgsr_uncer_loss_forward.restype = c_int
        L.wgsr_uncer_loss_forward.argtypes = [U] + [_fp] * 10 + [_fp]
        L.wgsr_uncer_small_maps.restype = c_int
        L.wgsr_uncer_small_maps.argtypes = [U] + [_fp] * 10 + [_fp]
        L.wgsr_uncer_loss_small.restype = c_int
        L.wgsr_uncer_loss_small.argtypes = [U] + [_fp] * 4 + [ctypes.c_float] + [_fp] * 3 + [_fp]
        L.wgsr_uncer_loss_combine.restype = c_int
        L.wgsr_uncer_loss_combine.argtypes = ([U] + [_fp] * 4 + [c_int] + [ctypes.c_float] * 4 + [c_int] +
                                              [_fp] * 3 + [_fp])
        L.wgsr_uncer_loss_backward.restype = c_int
        L.wgsr_uncer_loss_backward.argtypes = [U] + [_fp] * 9 + [ctypes.c_float] * 2 + [_fp] * 5 + [_fp]
        L.wgsr_track_blocks.restype = c_int
        L.wgsr_track_blocks.argtypes = [c_i64]
        L.wgsr_tracking_loss.restype = c_int
        L.wgsr_tracking_loss.argtypes = [c_int, c_int] + [_fp] * 7 + [ctypes.c_float] + [_fp] * 3 + [_fp]
        L.wgsr_pose_state_floats.restype = c_int
        L.wgsr_pose_state_floats.argtypes = []
        L.wgsr_pose_step.restype = c_int
        L.wgsr_pose_step.argtypes = ([_fp] * 3 + [c_int, _fp] + [ctypes.c_float] * 6 + [c_int, ctypes.c_float, _fp,
                                                                                          c_int, _fp])
        L.wgsr_densify_blocks.restype = c_i64
        L.wgsr_densify_blocks.argtypes = [c_i64]
        L.wgsr_densify_select.restype = c_int
        L.wgsr_densify_select.argtypes = ([c_i64] + [_fp] * 5 + [ctypes.c_float] * 4 + [c_int, ctypes.c_float]
                                          + [_fp, _fp, _fp])
        L.wgsr_densify_emit.restype = c_int
        L.wgsr_densify_emit.argtypes = [c_i64, c_int, _fp, _fp, _fp, ctypes.POINTER(GaussianBank),
                                        ctypes.POINTER(GaussianBank), _fp]
        L.wgsr_reset_opacity.restype = c_int
        L.wgsr_reset_opacity.argtypes = [c_i64, _fp, _fp, ctypes.c_float, _fp, _fp, _fp]
        L.wgsr_deform_points.restype = c_int
        L.wgsr_deform_points.argtypes = [c_i64, ctypes.POINTER(GaussianBank), _fp, c_int, _fp, c_int, _fp, _fp]
        L.wgsr_sparse_grad_row_floats.restype = c_int
        L.wgsr_sparse_grad_row_floats.argtypes = [c_int]
        L.wgsr_sparse_mask_words.restype = c_i64
        L.wgsr_sparse_mask_words.argtypes = [c_i64]
        L.wgsr_sparse_pack_records.restype = c_int
        L.wgsr_sparse_pack_records.argtypes = [_fp, c_i64, c_i64, _fp, _fp, _fp, _fp]
        L.wgsr_sparse_summary_block_words.restype = c_i64
        L.wgsr_sparse_summary_block_words.argtypes = [c_int, c_i64]
        L.wgsr_sparse_exchange_summary.restype = c_int
        L.wgsr_sparse_exchange_summary.argtypes = [_fp, c_int, c_int, c_i64, _fp, _fp, _fp, _fp]
        L.wgsr_sparse_unpack_records.restype = c_int
        L.wgsr_sparse_unpack_records.argtypes = [_fp, _fp, c_int, c_i64, c_int, _fp, _fp, _fp]
        L.wgsr_sparse_fill_radius.restype = c_int
        L.wgsr_sparse_fill_radius.argtypes = [_fp, c_i64, _fp, _fp]
        L.wgsr_sparse_pack_grads.restype = c_int
        L.wgsr_sparse_pack_grads.argtypes = [c_i64, c_i64, c_int] + [_fp] * 8 + [_fp]
        L.wgsr_sparse_unpack_grads.restype = c_int
        L.wgsr_sparse_unpack_grads.argtypes = ([_fp, c_i64, _fp, c_int, c_int, c_i64, c_i64, c_i64, c_int] + [_fp] * 5
                                               + [c_int, _fp])
        L.wgsr_grad_mask.restype = c_int
        L.wgsr_grad_mask.argtypes = [c_int, c_int, _fp, ctypes.c_float, _fp, _fp]
        L.wgsr_mlp_scratch_bytes.restype = c_sz
        L.wgsr_mlp_scratch_bytes.argtypes = [c_int, c_int]
        L.wgsr_mlp_grad_floats.restype = c_int
        L.wgsr_mlp_grad_floats.argtypes = [c_int]
        L.wgsr_mlp_forward.restype = c_int
        L.wgsr_mlp_forward.argtypes = [c_int, c_int] + [_fp] * 7 + [ctypes.c_float, ctypes.c_uint32] + [_fp] * 4 + [_fp]
        L.wgsr_mlp_forward_dev_seed.restype = c_int
        L.wgsr_mlp_forward_dev_seed.argtypes = [c_int, c_int] + [_fp] * 7 + [ctypes.c_float, _fp] + [_fp] * 4 + [_fp]
        L.wgsr_random_keys.restype = c_int
        L.wgsr_random_keys.argtypes = [c_i64, ctypes.c_uint32, _fp, _fp, _fp]
        L.wgsr_random_perm_max.restype = c_i64
        L.wgsr_random_perm_max.argtypes = []
        L.wgsr_random_perm.restype = c_int
        L.wgsr_random_perm.argtypes = [c_i64, ctypes.c_uint32, _fp, _fp, _fp, _fp]
        L.wgsr_random_perm_prefix_max_n.restype = c_i64
        L.wgsr_random_perm_prefix_max_n.argtypes = []
        L.wgsr_random_perm_prefix_max_k.restype = c_i64
        L.wgsr_random_perm_prefix_max_k.argtypes = []
        L.wgsr_random_perm_prefix.restype = c_int
        L.wgsr_random_perm_prefix.argtypes = [c_i64, c_i64, ctypes.c_uint32, _fp, _fp, _fp]
        L.wgsr_mlp_forward_seg2.restype = c_int
        L.wgsr_mlp_forward_seg2.argtypes = [c_int, c_int, c_int] + [_fp] * 8 + [ctypes.c_float] + [_fp] * 7
        L.wgsr_mlp_backward_seg2.restype = c_int
        L.wgsr_mlp_backward_seg2.argtypes = ([c_int, c_int, c_int] + [_fp] * 4 + [ctypes.c_float] + [_fp] * 5
                                             + [ctypes.c_float, ctypes.c_float, c_int, _fp, _fp, _fp])
        L.wgsr_ssim_forward_partials.restype = c_int
        L.wgsr_ssim_forward_partials.argtypes = [_fp, _fp, c_i64, c_int, c_int, c_int, _fp, _fp, _fp]
        L.wgsr_ssim_tiles.restype = c_int
        L.wgsr_ssim_tiles.argtypes = [c_int, c_int]
        L.wgsr_uncer_loss_combine_ssim.restype = c_int
        L.wgsr_uncer_loss_combine_ssim.argtypes = ([U] + [_fp] * 5 + [c_int] + [ctypes.c_float] * 4
                                                   + [_fp] * 3 + [_fp])
        L.wgsr_adam_step_dev2.restype = c_int
        L.wgsr_adam_step_dev2.argtypes = ([ctypes.POINTER(AdamTensor), c_int, c_int] + [ctypes.c_double] * 4
                                          + [_fp] + [ctypes.c_double] * 2 + [_fp, _fp, _fp])
        L.wgsr_mlp_backward_acc.restype = c_int
        L.wgsr_mlp_backward_acc.argtypes = ([c_int, c_int] + [_fp] * 3 + [ctypes.c_float] + [_fp] * 4
                                            + [ctypes.c_float, c_int, _fp, _fp, _fp])
        L.wgsr_gather_rows.restype = c_int
        L.wgsr_gather_rows.argtypes = [ctypes.POINTER(GatherJob), c_int, _fp, _fp]
        L.wgsr_exposure_step.restype = c_int
        L.wgsr_exposure_step.argtypes = [_fp] * 3 + [c_int] + [_fp] * 3 + [ctypes.c_double] * 3 + [_fp] * 4
        L.wgsr_mlp_backward.restype = c_int
        L.wgsr_mlp_backward.argtypes = [c_int, c_int] + [_fp] * 3 + [ctypes.c_float] + [_fp] * 6 + [_fp]
        L.wgsr_dino_reg.restype = c_int
        L.wgsr_dino_reg.argtypes = ([_fp, _fp, c_int, c_int, c_int, ctypes.c_float, ctypes.c_float] + [_fp] * 5
                                    + [_fp])
        L.wgsr_densification_stats.restype = c_int
        L.wgsr_densification_stats.argtypes = [c_int] + [_fp] * 5 + [_fp]
        L.wgsr_mark_visible.restype = c_int
        L.wgsr_mark_visible.argtypes = [c_int, _fp, _fp, _fp, _fp, _fp]
        L.wgsr_dist_cuda2.restype = c_int
        L.wgsr_dist_cuda2.argtypes = [c_int, _fp, _fp, ALLOC_FN, ctypes.c_void_p, _fp]
        for name in ("wgsr_geometry_bytes",):
            getattr(L, name).restype = c_sz
            getattr(L, name).argtypes = [c_int]
        L.wgsr_binning_bytes.restype = c_sz
        L.wgsr_binning_bytes.argtypes = [c_i64, c_int, c_int]
        L.wgsr_image_bytes.restype = c_sz
        L.wgsr_image_bytes.argtypes = [c_int, c_int]
        L.wgsr_adam_step.restype = c_int
        L.wgsr_adam_step.argtypes = [ctypes.POINTER(AdamTensor), c_int, ctypes.c_double, ctypes.c_double,
                                     ctypes.c_double, _fp]
        L.wgsr_adam_step_dev.restype = c_int
        L.wgsr_adam_step_dev.argtypes = [ctypes.POINTER(AdamTensor), c_int, ctypes.c_double, ctypes.c_double,
                                         ctypes.c_double, ctypes.c_double, _fp, _fp, _fp]
        L.wgsr_rasterize_forward_cap.restype = c_int
        L.wgsr_rasterize_forward_cap.argtypes = [P_ARGS, c_i64, ALLOC_FN, ALLOC_FN, ALLOC_FN, ctypes.c_void_p,
                                                 _fp, _fp, _fp, _fp, _fp, _fp, _fp]
        L.wgsr_binning_bytes_cap.restype = c_sz
        L.wgsr_binning_bytes_cap.argtypes = [P_ARGS, c_i64]
        L.wgsr_check_tile_lists.restype = c_int
        L.wgsr_check_tile_lists.argtypes = [P_ARGS, c_i64, _fp, _fp, _fp, _fp]
        L.wgsr_compact_rows.restype = c_int
        L.wgsr_compact_rows.argtypes = [_fp, c_i64, ctypes.POINTER(RowTensor), c_int, ALLOC_FN,
                                        ctypes.c_void_p, _fp]
        L.wgsr_ssim_scratch_bytes.restype = ctypes.c_size_t
        L.wgsr_ssim_scratch_bytes.argtypes = [c_i64, c_int, c_int]
        L.wgsr_ssim_forward.restype = c_int
        L.wgsr_ssim_forward.argtypes = [_fp, _fp, c_i64, c_int, c_int, c_int, _fp, _fp, _fp, ALLOC_FN,
                                        ctypes.c_void_p, _fp]
        L.wgsr_ssim_backward.restype = c_int
        L.wgsr_ssim_backward.argtypes = [_fp, _fp, c_i64, c_int, c_int, c_int, _fp, _fp, _fp, _fp]
        L.wgsr_ssim_components.restype = c_int
        L.wgsr_ssim_components.argtypes = [_fp, _fp, c_i64, c_int, c_int, c_int, c_int, _fp, _fp, _fp, _fp]
        L.wgsr_ply_pack.restype = c_int
        L.wgsr_ply_pack.argtypes = [ctypes.POINTER(PlyColumnSet), c_int, c_i64, c_int, _fp, _fp]
        L.wgsr_ply_unpack.restype = c_int
        L.wgsr_ply_unpack.argtypes = [_fp, c_i64, c_int, ctypes.POINTER(PlyColumnSet), c_int, _fp]
        L.wgsr_last_error.restype = ctypes.c_char_p
        L.wgsr_last_error.argtypes = []
        L.wgsr_version.restype = ctypes.c_char_p
        L.wgsr_version.argtypes = []
        L.wgsr_depth_order_offset.restype = ctypes.c_int64
        L.wgsr_depth_order_offset.argtypes = []
        L.wgsr_profile_enable.restype = None
        L.wgsr_profile_enable.argtypes = [c_int]
        L.wgsr_profile_read.restype = c_int
        L.wgsr_profile_read.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(c_i64), c_int, c_int]
        L.wgsr_profile_stage_name.restype = ctypes.c_char_p
        L.wgsr_profile_stage_name.argtypes = [c_int]
        _lib = L
    return _lib


EXPORTED_SYMBOLS = (
    "wgsr_rasterize_forward", "wgsr_rasterize_backward", "wgsr_mark_visible", "wgsr_dist_cuda2",
    "wgsr_geometry_bytes", "wgsr_binning_bytes", "wgsr_image_bytes", "wgsr_last_error",
    "wgsr_version", "wgsr_depth_order_offset", "wgsr_profile_enable", "wgsr_profile_read", "wgsr_profile_stage_name",
    "wgsr_adam_step", "wgsr_adam_step_dev", "wgsr_compact_rows",
    "wgsr_rasterize_forward_cap", "wgsr_binning_bytes_cap", "wgsr_check_tile_lists", "wgsr_mlp_forward_dev_seed", "wgsr_random_keys",
    "wgsr_random_perm_max", "wgsr_random_perm", "wgsr_random_perm_prefix_max_n", "wgsr_random_perm_prefix_max_k",
    "wgsr_random_perm_prefix", "wgsr_mlp_forward_seg2", "wgsr_mlp_backward_seg2",
    "wgsr_gaussian_activate_backward_stats", "wgsr_ssim_forward_partials", "wgsr_ssim_tiles",
    "wgsr_uncer_loss_combine_ssim", "wgsr_adam_step_dev2", "wgsr_mlp_backward_acc", "wgsr_gather_rows", "wgsr_exposure_step",
    "wgsr_ssim_scratch_bytes", "wgsr_ssim_forward", "wgsr_ssim_backward", "wgsr_ssim_components",
    "wgsr_ply_pack", "wgsr_ply_unpack",
    "wgsr_pack_view_camera", "wgsr_rasterize_backward_records", "wgsr_gauss_backward_views_blocks",
    "wgsr_gauss_backward_views",
    "wgsr_map_blocks", "wgsr_gaussian_activate", "wgsr_gaussian_activate_backward",
    "wgsr_mapping_loss_forward", "wgsr_mapping_loss_backward", "wgsr_densification_stats",
    "wgsr_uncer_blocks", "wgsr_uncer_loss_forward", "wgsr_uncer_small_maps", "wgsr_uncer_loss_small",
    "wgsr_uncer_loss_backward", "wgsr_uncer_loss_combine", "wgsr_track_blocks", "wgsr_tracking_loss", "wgsr_grad_mask",
    "wgsr_pose_state_floats", "wgsr_pose_step",
    "wgsr_mlp_scratch_bytes", "wgsr_mlp_grad_floats", "wgsr_mlp_forward", "wgsr_mlp_backward", "wgsr_dino_reg",
    "wgsr_densify_blocks", "wgsr_densify_select", "wgsr_densify_emit", "wgsr_reset_opacity", "wgsr_deform_points",
    "wgsr_sparse_grad_row_floats", "wgsr_sparse_mask_words", "wgsr_sparse_pack_records",
    "wgsr_sparse_summary_block_words", "wgsr_sparse_exchange_summary", "wgsr_sparse_unpack_records",
    "wgsr_sparse_fill_radius", "wgsr_sparse_pack_grads", "wgsr_sparse_unpack_grads",
)

VIEW_RECORD_FLOATS = 12   # WGSR_VIEW_RECORD_FLOATS
VIEW_CAMERA_FLOATS = 64   # WGSR_VIEW_CAMERA_FLOATS


class StageProfile:
    """Per-stage device time (HIP events on the launch stream) inside a block.

    stages: names of the stages to time (None: all).  Each timed stage adds
    two event records per launch to the stream, which the GPU serialises, so
    a timed loop should time only what it reports."""

    def __init__(self, stages=None):
        self.only = stages

    def __enter__(self):
        L = load()
        L.wgsr_profile_read(None, None, 0, 1)
        if self.only is None:
            L.wgsr_profile_enable(1)
        else:
            names = [L.wgsr_profile_stage_name(i).decode() for i in range(16)]
            mask = 0
            for st in self.only:
                mask |= 1 << names.index(st)
            L.wgsr_profile_enable(mask << 1)
        return self

    def __exit__(self, *exc):
        L = load()
        n = 16
        ms = (ctypes.c_double * n)()
        cnt = (ctypes.c_int64 * n)()
        k = L.wgsr_profile_read(ms, cnt, n, 1)
        L.wgsr_profile_enable(0)
        self.stages = {L.wgsr_profile_stage_name(i).decode(): (ms[i], int(cnt[i])) for i in range(k)}
        return False


def check(code: int):
    if code != 0:
        msg = load().wgsr_last_error().decode(errors="replace")
        raise RuntimeError(f"wgsr error {code}: {msg}")


# ---------------------------------------------------------------------------
# Allocation callbacks: each call records a torch uint8 tensor in the active
# request's slot so Python owns (and later frees) every byte.
# ---------------------------------------------------------------------------
_tls = threading.local()


class AllocRequest:
    def __init__(self, device: torch.device):
        self.device = device
        self.buffers = {}

    def __enter__(self):
        self._prev = getattr(_tls, "req", None)
        _tls.req = self
        return self

    def __exit__(self, *exc):
        _tls.req = self._prev
        return False


def _make_alloc(slot: str):
    # (a second call for the same buffer within one library call -- the
    # forward's predicted binning buffer was too small for the exact size --
    # replaces the first allocation; the library uses the pointer of the last
    # call and wrote nothing through the first)
    def _alloc(_ctx, nbytes):
        req = _tls.req
        n = int(nbytes)
        base = req.buffers.get(slot + "_base")
        if base is None or base.numel() < max(n, 1):
            base = torch.empty(max(n, 1), dtype=torch.uint8, device=req.device)
        req.buffers[slot] = base[:n]
        req.buffers[slot + "_base"] = base
        return base.data_ptr()
    return ALLOC_FN(_alloc)


ALLOC_GEOM = _make_alloc("geom")
ALLOC_BINNING = _make_alloc("binning")
ALLOC_IMAGE = _make_alloc("image")
ALLOC_SCRATCH = _make_alloc("scratch")


def ptr(t):
    """Device address of a tensor, or None for an absent (empty) one."""
    if t is None or t.numel() == 0:
        return None
    return t.data_ptr()


def stream_handle(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream
