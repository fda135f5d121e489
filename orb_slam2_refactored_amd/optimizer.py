"""Optimizer::LocalBundleAdjustment / PoseOptimization mirrors (include/Optimizer.h:47-49) over the
gfx950 C-ABI.

The reference's graph gathering (local KFs by covisibility, local MPs, fixed KFs; Optimizer.cc:493-537)
operates on ORB-SLAM's pointer graph; callers flatten that into a `problem` dict (see
include/orbslam2_amd.h, orbba_problem) and get back optimised poses / points / outlier flags, which
they write back exactly like :677-735.
"""
import ctypes as C

import numpy as np

from ._lib import BAProblem, BAResult, PoseBatch, PoseResult, check, lib, ptr, stream_ptr, tptr


def _need(arrays: dict, counts: dict, what: str):
    """Refuse arrays with fewer elements than the C-ABI reads from them (it has no bound of its own)."""
    for name, want in counts.items():
        a = arrays[name]
        n = a.size if isinstance(a, np.ndarray) else int(a.numel()) if hasattr(a, "numel") else int(np.size(a))
        if n < want:
            raise ValueError(f"{what}: {name} has {n} elements, needs {want}")


def LocalBundleAdjustment(problem: dict, stop_flag=None, device: int = 0) -> dict:
    keep = []

    def k(a, dt):
        a = np.ascontiguousarray(a, dt)
        keep.append(a)
        return ptr(a)

    P0, N0, E0 = len(problem["pose_R"]), len(problem["points"]), len(problem["edge_point"])
    _need(problem, {"pose_R": 9 * P0, "pose_t": 3 * P0, "pose_fixed": P0, "points": 3 * N0, "edge_pose": E0,
                    "edge_obs": 3 * E0, "edge_inv_sigma2": E0, "edge_cam": 5 * E0}, "LocalBundleAdjustment")
    pr = BAProblem(len(problem["pose_R"]), k(problem["pose_R"], np.float64), k(problem["pose_t"], np.float64),
                   k(problem["pose_fixed"], np.uint8), len(problem["points"]), k(problem["points"], np.float64),
                   len(problem["edge_point"]), k(problem["edge_point"], np.int32), k(problem["edge_pose"], np.int32),
                   k(problem["edge_obs"], np.float64), k(problem["edge_inv_sigma2"], np.float64),
                   k(problem["edge_cam"], np.float64))
    P, N, E = pr.n_poses, pr.n_points, pr.n_edges
    # (np.empty: orbba_local_ba writes every element of each, also when it optimises nothing)
    out = dict(pose_R=np.empty((P, 9)), pose_t=np.empty((P, 3)), pose_q=np.empty((P, 4)), points=np.empty((N, 3)),
               edge_outlier=np.empty(E, np.uint8), edge_chi2=np.empty(E))
    res = BAResult(ptr(out["pose_R"]), ptr(out["pose_t"]), ptr(out["pose_q"]), ptr(out["points"]),
                   ptr(out["edge_outlier"]), ptr(out["edge_chi2"]))
    sf = None
    if stop_flag is not None:
        flag = stop_flag if isinstance(stop_flag, C.c_int32) else C.c_int32(int(stop_flag))
        keep.append(flag)
        sf = C.cast(C.pointer(flag), C.c_void_p)
    check(lib().orbba_local_ba(C.byref(pr), C.byref(res), sf, device), "orbba_local_ba")
    out["iterations"] = tuple(res.iterations)
    out["chi2"] = tuple(res.chi2)
    out["ran"] = bool(res.ran)   # False: stop flag set on entry, nothing to write back (Optimizer.cc:633-634)
    return out


def _pose_arrays(batch: dict):
    keep = []

    def k(a, dt):
        a = np.ascontiguousarray(a, dt)
        keep.append(a)
        return ptr(a)

    n = len(batch["edge_begin"]) - 1
    E = int(batch["edge_begin"][-1]) if n >= 0 and len(batch["edge_begin"]) else 0
    _need(batch, {"pose_R": 9 * n, "pose_t": 3 * n, "cam": 5 * n, "xw": 3 * E, "obs": 3 * E, "inv_sigma2": E},
          "PoseOptimization")
    pb = PoseBatch(n, k(batch["edge_begin"], np.int32), k(batch["pose_R"], np.float64), k(batch["pose_t"], np.float64),
                   k(batch["cam"], np.float64), k(batch["xw"], np.float64), k(batch["obs"], np.float64),
                   k(batch["inv_sigma2"], np.float64))
    return pb, keep


def PoseOptimization(batch: dict, device: int = 0) -> dict:
    """int Optimizer::PoseOptimization(Frame*) (include/Optimizer.h:49, src/Optimizer.cc:345-489) over a
    batch of frames.  `batch` holds, per frame f, the edges [edge_begin[f], edge_begin[f+1]) of the
    keypoints that have a map point, in keypoint order: xw (E,3) map point positions, obs (E,3)
    = (u, v, ur) with ur < 0 for monocular, inv_sigma2 (E,), plus pose_R (F,9) / pose_t (F,3) = frame->pose
    and cam (F,5) = fx, fy, cx, cy, bf.  Returns pose_R / pose_t (the frame->SetPose argument),
    n_inliers (the return value) and outlier (E,) = frame->outlier."""
    pb, keep = _pose_arrays(batch)
    n, E = pb.n_frames, int(batch["edge_begin"][-1]) if len(batch["edge_begin"]) else 0
    out = dict(pose_R=np.zeros((n, 9)), pose_t=np.zeros((n, 3)), n_inliers=np.zeros(n, np.int32),
               outlier=np.zeros(E, np.uint8))
    res = PoseResult(ptr(out["pose_R"]), ptr(out["pose_t"]), ptr(out["n_inliers"]), ptr(out["outlier"]))
    check(lib().orbba_pose_optimization(C.byref(pb), C.byref(res), device), "orbba_pose_optimization")
    return out


def pose_optimization_device(batch: dict, out: dict | None = None, stream=None) -> dict:
    """Device form: `batch` values are torch tensors on the GPU (int32 edge_begin, float64 others);
    enqueues one launch on `stream` (default: torch's current stream) and returns the output tensors."""
    import torch
    eb = batch["edge_begin"]
    n = eb.numel() - 1
    E = batch["inv_sigma2"].numel()
    _need(batch, {"pose_R": 9 * n, "pose_t": 3 * n, "cam": 5 * n, "xw": 3 * E, "obs": 3 * E},
          "pose_optimization_device")
    for name in ("pose_R", "pose_t", "cam", "xw", "obs", "inv_sigma2"):
        t = batch[name]
        if t.dtype != torch.float64 or not t.is_contiguous():
            raise ValueError(f"pose_optimization_device: {name} must be a contiguous float64 tensor")
    if eb.dtype != torch.int32 or not eb.is_contiguous():
        raise ValueError("pose_optimization_device: edge_begin must be a contiguous int32 tensor")
    dev = eb.device
    if out is None:
        out = dict(pose_R=torch.empty((n, 9), dtype=torch.float64, device=dev),
                   pose_t=torch.empty((n, 3), dtype=torch.float64, device=dev),
                   n_inliers=torch.empty(n, dtype=torch.int32, device=dev),
                   outlier=torch.empty(max(E, 1), dtype=torch.uint8, device=dev))
    pb = PoseBatch(n, tptr(eb), tptr(batch["pose_R"]), tptr(batch["pose_t"]), tptr(batch["cam"]), tptr(batch["xw"]),
                   tptr(batch["obs"]), tptr(batch["inv_sigma2"]))
    res = PoseResult(tptr(out["pose_R"]), tptr(out["pose_t"]), tptr(out["n_inliers"]), tptr(out["outlier"]))
    check(lib().orbba_pose_optimization_device(C.byref(pb), C.byref(res), stream_ptr(stream)),
          "orbba_pose_optimization_device")
    return out
