"""Loader for liborbslam2_amd.so (the HIP kernels + C-ABI, include/orbslam2_amd.h).

There is deliberately no CPU fallback: if the library is missing or cannot be loaded this module
raises, and every op in the package fails loudly.
"""
import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("ORBSLAM2_AMD_LIB", PKG / "liborbslam2_amd.so"))


class OrbxParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scaleFactor", C.c_float), ("nlevels", C.c_int32),
                ("iniThFAST", C.c_int32), ("minThFAST", C.c_int32)]


class TriFrame(C.Structure):
    _fields_ = [("n", C.c_int32), ("kp_xy", C.c_void_p), ("octave", C.c_void_p), ("uright", C.c_void_p),
                ("has_mappoint", C.c_void_p), ("desc", C.c_void_p), ("n_nodes", C.c_int32),
                ("node_id", C.c_void_p), ("node_off", C.c_void_p), ("indices", C.c_void_p)]


class TriBatch(C.Structure):
    """orbm_tri_batch (include/orbslam2_amd.h)."""
    _fields_ = [("n_pairs", C.c_int32), ("cap1", C.c_int32), ("cap2", C.c_int32),
                ("kps1", C.c_void_p), ("desc1", C.c_void_p), ("counts1", C.c_void_p), ("uright1", C.c_void_p),
                ("has_mappoint1", C.c_void_p), ("kps2", C.c_void_p), ("desc2", C.c_void_p), ("counts2", C.c_void_p),
                ("uright2", C.c_void_p), ("has_mappoint2", C.c_void_p), ("frame1", C.c_void_p),
                ("frame2", C.c_void_p), ("F12", C.c_void_p), ("ep2", C.c_void_p),
                ("fv_node1", C.c_void_p), ("fv_off1", C.c_void_p), ("fv_idx1", C.c_void_p),
                ("fv_n_nodes1", C.c_void_p), ("fv_node2", C.c_void_p), ("fv_off2", C.c_void_p),
                ("fv_idx2", C.c_void_p), ("fv_n_nodes2", C.c_void_p), ("fv_cap1", C.c_int32),
                ("fv_cap2", C.c_int32), ("n_levels", C.c_int32), ("scale_factors2", C.c_void_p),
                ("sigma2", C.c_void_p), ("only_stereo", C.c_int32)]


class BowBatch(C.Structure):
    """orbm_bow_batch (include/orbslam2_amd.h)."""
    _fields_ = [("n_pairs", C.c_int32), ("cap1", C.c_int32), ("cap2", C.c_int32),
                ("kps1", C.c_void_p), ("desc1", C.c_void_p), ("mp_valid1", C.c_void_p), ("frame1", C.c_void_p),
                ("kps2", C.c_void_p), ("desc2", C.c_void_p), ("counts2", C.c_void_p),
                ("fv_node1", C.c_void_p), ("fv_off1", C.c_void_p), ("fv_idx1", C.c_void_p),
                ("fv_n_nodes1", C.c_void_p), ("fv_node2", C.c_void_p), ("fv_off2", C.c_void_p),
                ("fv_idx2", C.c_void_p), ("fv_n_nodes2", C.c_void_p), ("fv_cap1", C.c_int32),
                ("fv_cap2", C.c_int32), ("nnratio", C.c_float), ("check_orientation", C.c_int32),
                ("counts1", C.c_void_p), ("mp_valid2", C.c_void_p), ("frame2", C.c_void_p)]


class StereoView(C.Structure):
    _fields_ = [("n", C.c_int32), ("kps", C.c_void_p), ("desc", C.c_void_p), ("n_levels", C.c_int32),
                ("level", C.c_void_p), ("level_rows", C.c_void_p), ("level_cols", C.c_void_p),
                ("level_step", C.c_void_p)]


class BAProblem(C.Structure):
    _fields_ = [("n_poses", C.c_int32), ("pose_R", C.c_void_p), ("pose_t", C.c_void_p),
                ("pose_fixed", C.c_void_p), ("n_points", C.c_int32), ("points", C.c_void_p),
                ("n_edges", C.c_int32), ("edge_point", C.c_void_p), ("edge_pose", C.c_void_p),
                ("edge_obs", C.c_void_p), ("edge_inv_sigma2", C.c_void_p), ("edge_cam", C.c_void_p)]


class BAResult(C.Structure):
    _fields_ = [("pose_R", C.c_void_p), ("pose_t", C.c_void_p), ("pose_q", C.c_void_p),
                ("points", C.c_void_p), ("edge_outlier", C.c_void_p), ("edge_chi2", C.c_void_p),
                ("iterations", C.c_int32 * 2), ("chi2", C.c_double * 2), ("ran", C.c_int32)]


class ProjBatch(C.Structure):
    _fields_ = [("n_frames", C.c_int32), ("total_kp", C.c_int32), ("total_mp", C.c_int32),
                ("kp_begin", C.c_void_p), ("kp_xy", C.c_void_p), ("kp_octave", C.c_void_p), ("kp_uright", C.c_void_p),
                ("kp_desc", C.c_void_p), ("kp_claimed", C.c_void_p), ("bounds", C.c_void_p),
                ("mp_begin", C.c_void_p), ("mp_valid", C.c_void_p), ("mp_proj", C.c_void_p),
                ("mp_view_cos", C.c_void_p), ("mp_level", C.c_void_p), ("mp_desc", C.c_void_p),
                ("mp_has_obs", C.c_void_p), ("n_levels", C.c_int32), ("scale_factors", C.c_void_p),
                ("th", C.c_float), ("nnratio", C.c_float)]


class MotionBatch(C.Structure):
    """orbm_motion_batch (include/orbslam2_amd.h)."""
    _fields_ = [("n_frames", C.c_int32), ("total_kp", C.c_int32), ("total_mp", C.c_int32),
                ("kp_begin", C.c_void_p), ("kp_xy", C.c_void_p), ("kp_octave", C.c_void_p), ("kp_uright", C.c_void_p),
                ("kp_desc", C.c_void_p), ("kp_angle", C.c_void_p), ("kp_claimed", C.c_void_p), ("bounds", C.c_void_p),
                ("mp_begin", C.c_void_p), ("mp_valid", C.c_void_p), ("mp_proj", C.c_void_p), ("mp_octave", C.c_void_p),
                ("mp_desc", C.c_void_p), ("mp_has_obs", C.c_void_p), ("mp_angle", C.c_void_p), ("motion", C.c_void_p),
                ("n_levels", C.c_int32), ("scale_factors", C.c_void_p), ("th", C.c_float),
                ("check_orientation", C.c_int32)]


class RelocBatch(C.Structure):
    """orbm_reloc_batch (include/orbslam2_amd.h)."""
    _fields_ = [("n_frames", C.c_int32), ("total_kp", C.c_int32), ("total_mp", C.c_int32),
                ("kp_begin", C.c_void_p), ("kp_xy", C.c_void_p), ("kp_octave", C.c_void_p), ("kp_desc", C.c_void_p),
                ("kp_angle", C.c_void_p), ("kp_claimed", C.c_void_p), ("bounds", C.c_void_p), ("pose", C.c_void_p),
                ("camera", C.c_void_p), ("mp_begin", C.c_void_p), ("mp_valid", C.c_void_p), ("mp_xw", C.c_void_p),
                ("mp_max_min", C.c_void_p), ("mp_desc", C.c_void_p), ("mp_angle", C.c_void_p), ("n_levels", C.c_int32),
                ("scale_factors", C.c_void_p), ("log_scale_factor", C.c_float), ("th", C.c_float),
                ("orb_dist", C.c_int32), ("check_orientation", C.c_int32)]


class InitBatch(C.Structure):
    """orbm_init_batch (include/orbslam2_amd.h)."""
    _fields_ = [("n_pairs", C.c_int32), ("total_kp", C.c_int32), ("total_q", C.c_int32),
                ("kp_begin", C.c_void_p), ("kp_xy", C.c_void_p), ("kp_octave", C.c_void_p), ("kp_desc", C.c_void_p),
                ("kp_angle", C.c_void_p), ("bounds", C.c_void_p), ("q_begin", C.c_void_p), ("q_octave", C.c_void_p),
                ("q_desc", C.c_void_p), ("q_angle", C.c_void_p), ("prev_matched", C.c_void_p), ("window", C.c_int32),
                ("nnratio", C.c_float), ("check_orientation", C.c_int32)]


class PoseBatch(C.Structure):
    _fields_ = [("n_frames", C.c_int32), ("edge_begin", C.c_void_p), ("pose_R", C.c_void_p), ("pose_t", C.c_void_p),
                ("cam", C.c_void_p), ("xw", C.c_void_p), ("obs", C.c_void_p), ("inv_sigma2", C.c_void_p)]


class PoseResult(C.Structure):
    _fields_ = [("pose_R", C.c_void_p), ("pose_t", C.c_void_p), ("n_inliers", C.c_void_p), ("outlier", C.c_void_p)]


# cv::KeyPoint layout (28 bytes)
KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])

VP = C.c_void_p
I32 = C.c_int32
SZ = C.c_size_t

# name -> (restype, argtypes); every symbol declared in include/orbslam2_amd.h
SIGNATURES = {
    "orbx_create": (C.c_int, [C.POINTER(OrbxParams), C.c_int, C.POINTER(VP)]),
    "orbx_destroy": (C.c_int, [VP]),
    "orbx_scale_tables": (C.c_int, [VP, VP, VP, VP, VP, VP]),
    "orbx_max_keypoints": (C.c_int, [VP, C.c_int, C.c_int, C.POINTER(I32)]),
    "orbx_set_opencv_compat": (C.c_int, [VP, C.c_int, C.c_int]),
    "orbx_get_opencv_compat": (C.c_int, [VP, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "orbx_extract": (C.c_int, [VP, VP, C.c_int, C.c_int, SZ, VP, VP, C.c_int, C.POINTER(C.c_int)]),
    "orbx_pyramid_level": (C.c_int, [VP, C.c_int, VP, SZ, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "orbx_extract_batch_device": (C.c_int, [VP, VP, C.c_int, C.c_int, C.c_int, SZ, SZ, VP, VP, VP, C.c_int, VP]),
    "orbx_batch_status": (C.c_int, [VP, VP, C.POINTER(C.c_uint32)]),
    "orbx_fault_word_device": (C.c_int, [VP, C.POINTER(VP)]),
    "orbx_pyramid_device": (C.c_int, [VP, C.c_int, C.c_int, C.POINTER(VP), C.POINTER(C.c_int),
                                      C.POINTER(C.c_int), C.POINTER(SZ)]),
    "orbm_descriptor_distance": (C.c_int, [VP, VP]),
    "orbm_hamming_top2_device": (C.c_int, [VP, C.c_int, VP, C.c_int, VP, VP, VP, VP]),
    "orbm_bf_match_batch_device": (C.c_int, [VP, VP, C.c_int, VP, VP, C.c_int, VP, C.c_int, C.c_float, C.c_int,
                                             VP, VP, VP, VP, VP]),
    "orbm_bf_match": (C.c_int, [VP, C.c_int, VP, C.c_int, C.c_float, C.c_int, VP, VP, VP, VP]),
    "orbm_check_orientation": (C.c_int, [VP, C.c_int, VP, C.c_int, VP, C.POINTER(I32)]),
    "orbm_check_orientation_batch_device": (C.c_int, [VP, C.c_int, C.c_int, VP, VP, C.c_int, C.c_int, VP, C.c_int,
                                                      VP, C.c_int, VP, VP]),
    "orbm_search_for_triangulation": (C.c_int, [C.POINTER(TriFrame), C.POINTER(TriFrame), VP, VP, VP, VP,
                                                C.c_int, C.c_int, VP, C.POINTER(I32)]),
    "orbm_search_for_triangulation_batch_device": (C.c_int, [C.POINTER(TriBatch), VP, VP, VP]),
    "orbm_search_by_bow_batch_device": (C.c_int, [C.POINTER(BowBatch), VP, VP, VP]),
    "orbm_search_by_bow_kf_batch_device": (C.c_int, [C.POINTER(BowBatch), VP, VP, VP]),
    "orbm_compute_stereo_matches": (C.c_int, [C.POINTER(StereoView), C.POINTER(StereoView), VP, VP, C.c_float,
                                              C.c_float, VP, VP]),
    "orbx_stereo_matches_batch_device": (C.c_int, [VP, VP, C.c_int, VP, VP, VP, VP, VP, VP, C.c_int, C.c_float,
                                                   C.c_float, VP, VP, VP]),
    "orbx_stereo_matches_last": (C.c_int, [VP, VP, C.c_float, C.c_float, VP, VP, C.c_int]),
    "orbm_search_by_projection": (C.c_int, [C.POINTER(ProjBatch), VP, VP, C.c_int]),
    "orbm_search_by_projection_device": (C.c_int, [C.POINTER(ProjBatch), VP, VP, VP]),
    "orbm_search_by_projection_motion_device": (C.c_int, [C.POINTER(MotionBatch), VP, VP, VP]),
    "orbm_search_for_initialization": (C.c_int, [C.POINTER(InitBatch), VP, VP, C.c_int]),
    "orbm_search_by_projection_reloc": (C.c_int, [C.POINTER(RelocBatch), VP, VP, C.c_int]),
    "orbm_search_by_projection_reloc_device": (C.c_int, [C.POINTER(RelocBatch), VP, VP, VP]),
    "orbm_search_for_initialization_device": (C.c_int, [C.POINTER(InitBatch), VP, VP, VP]),
    "orbv_load_text": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(VP)]),
    "orbv_create": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, VP, VP, VP, VP, C.c_int, C.POINTER(VP)]),
    "orbv_destroy": (C.c_int, [VP]),
    "orbv_info": (C.c_int, [VP, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int),
                            C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "orbv_transform": (C.c_int, [VP, VP, C.c_int, C.c_int, VP, VP, C.POINTER(C.c_int), VP, VP, VP,
                                 C.POINTER(C.c_int)]),
    "orbv_transform_batch_device": (C.c_int, [VP, VP, VP, C.c_int, C.c_int, C.c_int, VP, VP, VP, VP, VP, VP, VP, VP]),
    "orbba_local_ba": (C.c_int, [C.POINTER(BAProblem), C.POINTER(BAResult), VP, C.c_int]),
    "orbba_pose_optimization": (C.c_int, [C.POINTER(PoseBatch), C.POINTER(PoseResult), C.c_int]),
    "orbba_pose_optimization_device": (C.c_int, [C.POINTER(PoseBatch), C.POINTER(PoseResult), VP]),
    "orbx_pack_descriptors": (C.c_int, [VP, C.c_int, VP, VP, C.c_int, VP, C.c_int, VP]),
    "orbx_profile_enable": (C.c_int, [VP, C.c_int]),
    "orbx_profile_read": (C.c_int, [VP, VP, VP]),
    "orbx_debug_level_candidates": (C.c_int, [VP, C.c_int, C.c_int, VP, C.c_int, C.POINTER(C.c_int)]),
    "orbx_debug_qt_sort": (C.c_int, [VP, C.c_int, VP]),
    "orbba_debug_po_wave": (C.c_int, [VP, VP, VP]),
    "orbx_debug_level_selected": (C.c_int, [VP, C.c_int, C.c_int, VP, C.c_int, C.POINTER(C.c_int)]),
    "orb_last_error": (C.c_char_p, []),
    "orb_device_count": (C.c_int, []),
}

_lib = None


class OrbError(RuntimeError):
    pass


def lib():
    """Load the native library (raises if absent: no fallback path exists)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise OrbError(f"{LIB_PATH} not found — build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        l = C.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            # an A/B build named by ORBSLAM2_AMD_LIB may predate newer entry points: those stay
            # unbound (calling one fails); the in-tree library must export every symbol
            if os.environ.get("ORBSLAM2_AMD_LIB") and not hasattr(l, name):
                continue
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        _lib = l
    return _lib


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib().orb_last_error().decode(errors="replace")
        raise OrbError(f"{what} failed with status {rc}: {msg}")
    return rc


def ptr(a: np.ndarray):
    # The buffer protocol is the cheapest address (~1 us; a.ctypes.data_as(VP) builds numpy's ctypes
    # helper, ~3 us, per array per call); read-only or empty arrays take the helper.
    try:
        return VP(C.addressof(C.c_char.from_buffer(a)))
    except (TypeError, ValueError, BufferError):
        return VP(a.ctypes.data)


def tptr(t):
    """Device pointer of a torch tensor."""
    return VP(t.data_ptr())


def stream_ptr(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return VP(s.cuda_stream)
