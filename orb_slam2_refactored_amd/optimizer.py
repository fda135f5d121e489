"""Optimizer::LocalBundleAdjustment mirror (include/Optimizer.h:47) over the gfx950 C-ABI.

The reference's graph gathering (local KFs by covisibility, local MPs, fixed KFs; Optimizer.cc:493-537)
operates on ORB-SLAM's pointer graph; callers flatten that into a `problem` dict (see
include/orbslam2_amd.h, orbba_problem) and get back optimised poses / points / outlier flags, which
they write back exactly like :677-735.
"""
import ctypes as C

import numpy as np

from ._lib import BAProblem, BAResult, check, lib, ptr


def LocalBundleAdjustment(problem: dict, stop_flag=None, device: int = 0) -> dict:
    keep = []

    def k(a, dt):
        a = np.ascontiguousarray(a, dt)
        keep.append(a)
        return ptr(a)

    pr = BAProblem(len(problem["pose_R"]), k(problem["pose_R"], np.float64), k(problem["pose_t"], np.float64),
                   k(problem["pose_fixed"], np.uint8), len(problem["points"]), k(problem["points"], np.float64),
                   len(problem["edge_point"]), k(problem["edge_point"], np.int32), k(problem["edge_pose"], np.int32),
                   k(problem["edge_obs"], np.float64), k(problem["edge_inv_sigma2"], np.float64),
                   k(problem["edge_cam"], np.float64))
    P, N, E = pr.n_poses, pr.n_points, pr.n_edges
    out = dict(pose_R=np.zeros((P, 9)), pose_t=np.zeros((P, 3)), pose_q=np.zeros((P, 4)), points=np.zeros((N, 3)),
               edge_outlier=np.zeros(E, np.uint8), edge_chi2=np.zeros(E))
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
    return out
