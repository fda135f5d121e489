"""ctypes binding of the CPU oracle (oracle/orb_oracle.cpp).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module.
"""
import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
ORACLE_DIR = ROOT / "oracle"
ORACLE_SO = ORACLE_DIR / "_build" / "liborb_oracle.so"


class OrbxParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scaleFactor", C.c_float), ("nlevels", C.c_int32),
                ("iniThFAST", C.c_int32), ("minThFAST", C.c_int32)]


class Keypoint(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("size", C.c_float), ("angle", C.c_float),
                ("response", C.c_float), ("octave", C.c_int32), ("class_id", C.c_int32)]


KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])


class TriFrame(C.Structure):
    _fields_ = [("n", C.c_int32), ("kp_xy", C.c_void_p), ("octave", C.c_void_p), ("uright", C.c_void_p),
                ("has_mappoint", C.c_void_p), ("desc", C.c_void_p), ("n_nodes", C.c_int32),
                ("node_id", C.c_void_p), ("node_off", C.c_void_p), ("indices", C.c_void_p)]


class BAProblem(C.Structure):
    _fields_ = [("n_poses", C.c_int32), ("pose_R", C.c_void_p), ("pose_t", C.c_void_p),
                ("pose_fixed", C.c_void_p), ("n_points", C.c_int32), ("points", C.c_void_p),
                ("n_edges", C.c_int32), ("edge_point", C.c_void_p), ("edge_pose", C.c_void_p),
                ("edge_obs", C.c_void_p), ("edge_inv_sigma2", C.c_void_p), ("edge_cam", C.c_void_p)]


class BAResult(C.Structure):
    _fields_ = [("pose_R", C.c_void_p), ("pose_t", C.c_void_p), ("pose_q", C.c_void_p),
                ("points", C.c_void_p), ("edge_outlier", C.c_void_p), ("edge_chi2", C.c_void_p),
                ("iterations", C.c_int32 * 2), ("chi2", C.c_double * 2), ("ran", C.c_int32)]


def build():
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not ORACLE_SO.exists() and (ORACLE_DIR / "orb_oracle.cpp").exists():
            build()
        _lib = C.CDLL(str(ORACLE_SO))
        _lib.oracle_fast_atan2.restype = C.c_float
        _lib.oracle_fast_atan2.argtypes = [C.c_float, C.c_float]
    return _lib


def set_compat(trig=None, resize_simd=None):
    """The oracle's OpenCV-build switches (process-wide; oracle_set_compat): trig "double" / "float",
    resize_simd V.  None keeps a switch.  Returns the previous (trig, resize_simd)."""
    t = -1 if trig is None else {"double": 0, "float": 1}[trig] if isinstance(trig, str) else int(trig)
    v = -1 if resize_simd is None else int(resize_simd)
    prev = lib().oracle_set_compat(t, v)
    return ("double", "float")[prev & 0xff], prev >> 8


class compat:
    """Context manager: oracle switches set for the block, restored after."""
    def __init__(self, trig=None, resize_simd=None):
        self.args = (trig, resize_simd)

    def __enter__(self):
        self.prev = set_compat(*self.args)
        return self

    def __exit__(self, *exc):
        set_compat(*self.prev)


def resize_tail_x(w, resize_simd):
    return lib().oracle_resize_tail_x(int(w), int(resize_simd))


def ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def params(nfeatures=2000, scale=1.2, nlevels=8, ini=20, mn=7):
    return OrbxParams(nfeatures, scale, nlevels, ini, mn)


def scale_tables(p):
    L = p.nlevels
    s, i, s2, is2 = (np.zeros(L, np.float32) for _ in range(4))
    q = np.zeros(L, np.int32)
    um = np.zeros(16, np.int32)
    lib().oracle_scale_tables(C.byref(p), ptr(s), ptr(i), ptr(s2), ptr(is2), ptr(q), ptr(um))
    return dict(scale=s, inv_scale=i, sigma2=s2, inv_sigma2=is2, quota=q, umax=um)


def gaussian_taps():
    t = np.zeros(7, np.int32)
    lib().oracle_gaussian_taps(ptr(t))
    return t


def pyramid(p, img):
    img = np.ascontiguousarray(img)
    L = p.nlevels
    offs = np.zeros(L, np.int64)
    w = np.zeros(L, np.int32)
    h = np.zeros(L, np.int32)
    lib().oracle_pyramid(C.byref(p), ptr(img), img.shape[0], img.shape[1], C.c_size_t(img.shape[1]), None,
                         ptr(offs), ptr(w), ptr(h))
    total = int((w.astype(np.int64) * h).sum())
    out = np.zeros(total, np.uint8)
    lib().oracle_pyramid(C.byref(p), ptr(img), img.shape[0], img.shape[1], C.c_size_t(img.shape[1]), ptr(out),
                         ptr(offs), ptr(w), ptr(h))
    return [out[offs[l]:offs[l] + w[l] * h[l]].reshape(h[l], w[l]) for l in range(L)]


def _kp_out(fn, *args, cap=1 << 20):
    xs, ys, rs = (np.zeros(cap, np.float32) for _ in range(3))
    n = fn(*args, ptr(xs), ptr(ys), ptr(rs), cap)
    assert n <= cap
    return np.stack([xs[:n], ys[:n], rs[:n]], axis=1)


def detect_fast(level_img, ini=20, mn=7):
    im = np.ascontiguousarray(level_img)
    return _kp_out(lib().oracle_detect_fast, ptr(im), im.shape[0], im.shape[1], C.c_size_t(im.shape[1]), ini, mn)


def fast_raw(img, th):
    im = np.ascontiguousarray(img)
    return _kp_out(lib().oracle_fast_raw, ptr(im), im.shape[0], im.shape[1], C.c_size_t(im.shape[1]), th)


def quadtree(kps, rows, cols, nfeat):
    kps = np.ascontiguousarray(kps, np.float32)
    xs, ys, rs = (np.ascontiguousarray(kps[:, i]) for i in range(3))
    cap = max(len(kps), 1) + 8
    ox, oy, orr = (np.zeros(cap, np.float32) for _ in range(3))
    n = lib().oracle_quadtree(ptr(xs), ptr(ys), ptr(rs), len(kps), rows, cols, nfeat, ptr(ox), ptr(oy), ptr(orr), cap)
    return np.stack([ox[:n], oy[:n], orr[:n]], axis=1)


def gaussian_blur(img):
    im = np.ascontiguousarray(img)
    out = np.zeros_like(im)
    lib().oracle_gaussian_blur(ptr(im), im.shape[0], im.shape[1], C.c_size_t(im.shape[1]), ptr(out))
    return out


def extract(p, img, cap=8192):
    img = np.ascontiguousarray(img)
    kps = np.zeros(cap, KP_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n = C.c_int32(0)
    per = np.zeros(p.nlevels, np.int32)
    rc = lib().oracle_extract(C.byref(p), ptr(img), img.shape[0], img.shape[1], C.c_size_t(img.shape[1]), ptr(kps),
                              ptr(desc), cap, C.byref(n), ptr(per))
    assert rc == 0, rc
    return kps[:n.value].copy(), desc[:n.value].copy(), per


def bf_match(A, B, nnratio=0.6, th_low=50):
    A = np.ascontiguousarray(A, np.uint8)
    B = np.ascontiguousarray(B, np.uint8)
    nA = len(A)
    bi, bd, sd, m = (np.zeros(nA, np.int32) for _ in range(4))
    lib().oracle_bf_match(ptr(A), nA, ptr(B), len(B), C.c_float(nnratio), th_low, ptr(bi), ptr(bd), ptr(sd), ptr(m))
    return bi, bd, sd, m


def check_orientation(angA, angB, match):
    """CheckOrientation (ORBmatcher.cc:249-309) on a query-indexed match (SearchForInitialization
    convention): returns (match after the filter, nmatches)."""
    angA = np.ascontiguousarray(angA, np.float32)
    angB = np.ascontiguousarray(angB, np.float32)
    m = np.array(match, np.int32, copy=True)
    n = lib().oracle_check_orientation(ptr(angA), len(m), ptr(angB), ptr(m))
    assert n >= 0, "bin out of range"
    return m, n


def descriptor_distance(a, b):
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return lib().oracle_descriptor_distance(ptr(a), ptr(b))


class _Keep:
    """Holds numpy arrays alive while a ctypes struct points into them."""

    def __init__(self):
        self.arrs = []

    def __call__(self, a, dtype):
        a = np.ascontiguousarray(a, dtype)
        self.arrs.append(a)
        return ptr(a)


def tri_frame(keep, xy, octave, uright, has_mp, desc, node_ids, node_off, indices):
    return TriFrame(len(xy), keep(xy, np.float32), keep(octave, np.int32), keep(uright, np.float32),
                    keep(has_mp, np.uint8), keep(desc, np.uint8), len(node_ids), keep(node_ids, np.uint32),
                    keep(node_off, np.int32), keep(indices, np.int32))


def search_for_triangulation(f1, f2, F12, ep2, scale2, sigma2, only_stereo=False):
    keep = _Keep()
    out = np.zeros(f1.n, np.int32)
    n = lib().oracle_search_for_triangulation(C.byref(f1), C.byref(f2), keep(F12, np.float32), keep(ep2, np.float32),
                                              keep(scale2, np.float32), keep(sigma2, np.float32), int(only_stereo),
                                              ptr(out))
    return out, n


def search_by_bow(kf, fr, ang_kf, ang_fr, nnratio=0.6, check_ori=True):
    """SearchByBoW(KeyFrame*, Frame&) (ORBmatcher.cc:452-516): kf / fr are tri_frame structs (kf's
    has_mappoint = MapPoint valid).  Returns (match [fr.n] = idx1 or -1, nmatches)."""
    keep = _Keep()
    out = np.zeros(max(fr.n, 1), np.int32)
    n = lib().oracle_search_by_bow(C.byref(kf), C.byref(fr), C.c_float(nnratio), int(check_ori),
                                   keep(ang_kf, np.float32), keep(ang_fr, np.float32), ptr(out))
    assert n >= 0, "bin out of range"
    return out[:fr.n], n


def search_by_bow_kf(kf1, kf2, ang1, ang2, nnratio=0.6, check_ori=True):
    """SearchByBoW(KeyFrame*, KeyFrame*) (ORBmatcher.cc:696-766): has_mappoint = MapPoint valid on
    both sides.  Returns (match12 [kf1.n] = idx2 or -1, nmatches)."""
    keep = _Keep()
    out = np.zeros(max(kf1.n, 1), np.int32)
    n = lib().oracle_search_by_bow_kf(C.byref(kf1), C.byref(kf2), C.c_float(nnratio), int(check_ori),
                                      keep(ang1, np.float32), keep(ang2, np.float32), ptr(out))
    assert n >= 0, "bin out of range"
    return out[:kf1.n], n


def ba_problem(keep, prob):
    return BAProblem(len(prob["pose_R"]), keep(prob["pose_R"], np.float64), keep(prob["pose_t"], np.float64),
                     keep(prob["pose_fixed"], np.uint8), len(prob["points"]), keep(prob["points"], np.float64),
                     len(prob["edge_point"]), keep(prob["edge_point"], np.int32), keep(prob["edge_pose"], np.int32),
                     keep(prob["edge_obs"], np.float64), keep(prob["edge_inv_sigma2"], np.float64),
                     keep(prob["edge_cam"], np.float64))


def local_ba(prob, stop=None, stop_after=-1):
    keep = _Keep()
    pr = ba_problem(keep, prob)
    P, N, E = pr.n_poses, pr.n_points, pr.n_edges
    out = dict(pose_R=np.zeros((P, 9)), pose_t=np.zeros((P, 3)), pose_q=np.zeros((P, 4)),
               points=np.zeros((N, 3)), edge_outlier=np.zeros(E, np.uint8), edge_chi2=np.zeros(E))
    res = BAResult(ptr(out["pose_R"]), ptr(out["pose_t"]), ptr(out["pose_q"]), ptr(out["points"]),
                   ptr(out["edge_outlier"]), ptr(out["edge_chi2"]))
    sf = None
    if stop is not None:
        sf = C.byref(C.c_int32(int(stop)))
    lib().oracle_local_ba_stop_after(C.byref(pr), C.byref(res), sf, int(stop_after))
    out["iterations"] = tuple(res.iterations)
    out["chi2"] = tuple(res.chi2)
    return out


class ProjBatch(C.Structure):
    _fields_ = [("n_frames", C.c_int32), ("total_kp", C.c_int32), ("total_mp", C.c_int32),
                ("kp_begin", C.c_void_p), ("kp_xy", C.c_void_p), ("kp_octave", C.c_void_p), ("kp_uright", C.c_void_p),
                ("kp_desc", C.c_void_p), ("kp_claimed", C.c_void_p), ("bounds", C.c_void_p),
                ("mp_begin", C.c_void_p), ("mp_valid", C.c_void_p), ("mp_proj", C.c_void_p),
                ("mp_view_cos", C.c_void_p), ("mp_level", C.c_void_p), ("mp_desc", C.c_void_p),
                ("mp_has_obs", C.c_void_p), ("n_levels", C.c_int32), ("scale_factors", C.c_void_p),
                ("th", C.c_float), ("nnratio", C.c_float)]


def proj_batch(keep, b):
    F = len(b["kp_begin"]) - 1
    claimed = b.get("kp_claimed")
    return ProjBatch(F, int(b["kp_begin"][-1]), int(b["mp_begin"][-1]), keep(b["kp_begin"], np.int32),
                     keep(b["kp_xy"], np.float32), keep(b["kp_octave"], np.int32), keep(b["kp_uright"], np.float32),
                     keep(b["kp_desc"], np.uint8), keep(claimed, np.uint8) if claimed is not None else None,
                     keep(b["bounds"], np.float32), keep(b["mp_begin"], np.int32), keep(b["mp_valid"], np.uint8),
                     keep(b["mp_proj"], np.float32), keep(b["mp_view_cos"], np.float32), keep(b["mp_level"], np.int32),
                     keep(b["mp_desc"], np.uint8), keep(b["mp_has_obs"], np.uint8), len(b["scale_factors"]),
                     keep(b["scale_factors"], np.float32), float(b["th"]), float(b["nnratio"]))


class MotionBatch(C.Structure):
    _fields_ = [("n_frames", C.c_int32), ("total_kp", C.c_int32), ("total_mp", C.c_int32),
                ("kp_begin", C.c_void_p), ("kp_xy", C.c_void_p), ("kp_octave", C.c_void_p), ("kp_uright", C.c_void_p),
                ("kp_desc", C.c_void_p), ("kp_angle", C.c_void_p), ("kp_claimed", C.c_void_p), ("bounds", C.c_void_p),
                ("mp_begin", C.c_void_p), ("mp_valid", C.c_void_p), ("mp_proj", C.c_void_p), ("mp_octave", C.c_void_p),
                ("mp_desc", C.c_void_p), ("mp_has_obs", C.c_void_p), ("mp_angle", C.c_void_p), ("motion", C.c_void_p),
                ("n_levels", C.c_int32), ("scale_factors", C.c_void_p), ("th", C.c_float),
                ("check_orientation", C.c_int32)]


_MOTION_KEYS = [("kp_begin", np.int32), ("kp_xy", np.float32), ("kp_octave", np.int32), ("kp_uright", np.float32),
                ("kp_desc", np.uint8), ("kp_angle", np.float32), ("kp_claimed", np.uint8), ("bounds", np.float32),
                ("mp_begin", np.int32), ("mp_valid", np.uint8), ("mp_proj", np.float32), ("mp_octave", np.int32),
                ("mp_desc", np.uint8), ("mp_has_obs", np.uint8), ("mp_angle", np.float32), ("motion", np.int32)]


def search_by_projection_motion(b):
    """SearchByProjection(Frame& currFrame, const Frame& lastFrame, th, mono) per frame
    (ORBmatcher.cc:1279-1362).  b: dict of numpy arrays (orbm_motion_batch fields)."""
    keep = _Keep()
    F = len(b["kp_begin"]) - 1
    ptrs = [keep(b[k], dt) if b.get(k) is not None else None for k, dt in _MOTION_KEYS]
    mb = MotionBatch(F, int(b["kp_begin"][-1]), int(b["mp_begin"][-1]), *ptrs, len(b["scale_factors"]),
                     keep(b["scale_factors"], np.float32), float(b["th"]), int(b["check_orientation"]))
    kp_match = np.zeros(max(mb.total_kp, 1), np.int32)
    n = np.zeros(F, np.int32)
    assert lib().oracle_search_by_projection_motion(C.byref(mb), ptr(kp_match), ptr(n)) == 0
    return kp_match[:mb.total_kp], n


def search_by_projection(b):
    """ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th) per frame (ORBmatcher.cc:315-382)."""
    keep = _Keep()
    pb = proj_batch(keep, b)
    kp_match = np.zeros(pb.total_kp, np.int32)
    n = np.zeros(pb.n_frames, np.int32)
    lib().oracle_search_by_projection(C.byref(pb), ptr(kp_match), ptr(n))
    return kp_match, n


def features_grid(xy, octave, bounds):
    """FeaturesGrid::AssignFeatures (Frame.cc:71-100) as CSR (cell = cx * 48 + cy)."""
    xy = np.ascontiguousarray(xy, np.float32)
    octave = np.ascontiguousarray(octave, np.int32)
    bounds = np.ascontiguousarray(bounds, np.float32)
    cs = np.zeros(64 * 48 + 1, np.int32)
    idx = np.zeros(max(len(xy), 1), np.int32)
    k = lib().oracle_features_grid(ptr(xy), ptr(octave), len(xy), ptr(bounds), ptr(cs), ptr(idx))
    return cs, idx[:k]


def features_in_area(xy, octave, bounds, nlevels, x, y, r, min_level=-1, max_level=-1):
    xy = np.ascontiguousarray(xy, np.float32)
    octave = np.ascontiguousarray(octave, np.int32)
    bounds = np.ascontiguousarray(bounds, np.float32)
    out = np.zeros(max(len(xy), 1), np.int32)
    n = lib().oracle_features_in_area(ptr(xy), ptr(octave), len(xy), ptr(bounds), nlevels, C.c_float(x), C.c_float(y),
                                      C.c_float(r), min_level, max_level, ptr(out), len(out))
    return out[:n]


class PoseBatch(C.Structure):
    _fields_ = [("n_frames", C.c_int32), ("edge_begin", C.c_void_p), ("pose_R", C.c_void_p), ("pose_t", C.c_void_p),
                ("cam", C.c_void_p), ("xw", C.c_void_p), ("obs", C.c_void_p), ("inv_sigma2", C.c_void_p)]


class PoseResult(C.Structure):
    _fields_ = [("pose_R", C.c_void_p), ("pose_t", C.c_void_p), ("n_inliers", C.c_void_p), ("outlier", C.c_void_p)]


def pose_optimization(batch):
    """Optimizer::PoseOptimization (src/Optimizer.cc:345-489) per frame of a make_pose_batch dict."""
    keep = _Keep()
    n = len(batch["edge_begin"]) - 1
    E = int(batch["edge_begin"][-1])
    pb = PoseBatch(n, keep(batch["edge_begin"], np.int32), keep(batch["pose_R"], np.float64),
                   keep(batch["pose_t"], np.float64), keep(batch["cam"], np.float64), keep(batch["xw"], np.float64),
                   keep(batch["obs"], np.float64), keep(batch["inv_sigma2"], np.float64))
    out = dict(pose_R=np.zeros((n, 9)), pose_t=np.zeros((n, 3)), n_inliers=np.zeros(n, np.int32),
               outlier=np.zeros(E, np.uint8))
    res = PoseResult(ptr(out["pose_R"]), ptr(out["pose_t"]), ptr(out["n_inliers"]), ptr(out["outlier"]))
    lib().oracle_pose_optimization(C.byref(pb), C.byref(res))
    return out


def std_sort_perm(sizes):
    sizes = np.ascontiguousarray(sizes, np.int32)
    perm = np.zeros(len(sizes), np.int32)
    lib().oracle_std_sort_sizes(ptr(sizes), len(sizes), ptr(perm))
    return perm


class StereoView(C.Structure):
    _fields_ = [("n", C.c_int32), ("kps", C.c_void_p), ("desc", C.c_void_p), ("n_levels", C.c_int32),
                ("level", C.c_void_p), ("level_rows", C.c_void_p), ("level_cols", C.c_void_p),
                ("level_step", C.c_void_p)]


def _stereo_view(keep, kps, desc, pyramid):
    kps = np.ascontiguousarray(kps)
    desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    levels = [np.ascontiguousarray(im, np.uint8) for im in pyramid]
    ptrs = (C.c_void_p * len(levels))(*[im.ctypes.data for im in levels])
    rows = np.array([im.shape[0] for im in levels], np.int32)
    cols = np.array([im.shape[1] for im in levels], np.int32)
    step = np.array([im.strides[0] for im in levels], np.int32)
    keep.arrs += [kps, desc, levels, ptrs, rows, cols, step]
    return StereoView(len(kps), kps.ctypes.data, desc.ctypes.data, len(levels), C.cast(ptrs, C.c_void_p),
                      rows.ctypes.data, cols.ctypes.data, step.ctypes.data)


def compute_stereo_matches(kpsL, descL, pyrL, kpsR, descR, pyrR, scale, inv_scale, bf, baseline):
    """ComputeStereoMatches oracle (src/ORBmatcher.cc:72-247) -> (uright, depth)."""
    keep = _Keep()
    vl = _stereo_view(keep, kpsL, descL, pyrL)
    vr = _stereo_view(keep, kpsR, descR, pyrR)
    ur = np.zeros(vl.n, np.float32)
    dp = np.zeros(vl.n, np.float32)
    lib().oracle_compute_stereo_matches(C.byref(vl), C.byref(vr), keep(scale, np.float32), keep(inv_scale, np.float32),
                                        C.c_float(bf), C.c_float(baseline), ptr(ur), ptr(dp))
    return ur, dp


class Vocabulary:
    """DBoW2 restatement handle (oracle/orb_oracle.cpp Vocabulary)."""

    def __init__(self, voc=None, path=None):
        L = lib()
        L.oracle_voc_load_text.restype = C.c_void_p
        L.oracle_voc_create.restype = C.c_void_p
        L.oracle_voc_destroy.argtypes = [C.c_void_p]
        if path is not None:
            self.h = L.oracle_voc_load_text(str(path).encode())
            assert self.h, "oracle failed to load the vocabulary"
        else:
            self._keep = [np.ascontiguousarray(voc["parent"], np.int32), np.ascontiguousarray(voc["is_leaf"], np.uint8),
                          np.ascontiguousarray(voc["desc"], np.uint8), np.ascontiguousarray(voc["weight"], np.float64)]
            self.h = L.oracle_voc_create(voc["k"], voc["L"], voc["scoring"], voc["weighting"], len(voc["parent"]),
                                         *[ptr(a) for a in self._keep])

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_voc_destroy(C.c_void_p(self.h))

    def info(self):
        o = np.zeros(6, np.int32)
        lib().oracle_voc_info(C.c_void_p(self.h), ptr(o))
        return dict(zip(("k", "L", "n_nodes", "n_words", "scoring", "weighting"), o.tolist()))

    def words(self, desc, levelsup=4):
        d = np.ascontiguousarray(desc, np.uint8)
        n = len(d)
        w, wt, nid = np.zeros(n, np.uint32), np.zeros(n), np.zeros(n, np.uint32)
        lib().oracle_voc_words(C.c_void_p(self.h), ptr(d), n, levelsup, ptr(w), ptr(wt), ptr(nid))
        return w, wt, nid

    def transform(self, desc, levelsup=4):
        d = np.ascontiguousarray(desc, np.uint8)
        n = len(d)
        cap = max(n, 1)
        bw, bv = np.zeros(cap, np.uint32), np.zeros(cap)
        fn, fo, fi = np.zeros(cap, np.uint32), np.zeros(cap + 1, np.int32), np.zeros(cap, np.int32)
        nw, nn = np.zeros(1, np.int32), np.zeros(1, np.int32)
        lib().oracle_voc_transform(C.c_void_p(self.h), ptr(d), n, levelsup, ptr(bw), ptr(bv), ptr(nw), ptr(fn),
                                   ptr(fo), ptr(fi), ptr(nn))
        a, b = int(nw[0]), int(nn[0])
        return (bw[:a], bv[:a]), (fn[:b], fo[:b + 1], fi[:fo[b]])


class InitBatch(C.Structure):
    _fields_ = [("n_pairs", C.c_int32), ("total_kp", C.c_int32), ("total_q", C.c_int32),
                ("kp_begin", C.c_void_p), ("kp_xy", C.c_void_p), ("kp_octave", C.c_void_p), ("kp_desc", C.c_void_p),
                ("kp_angle", C.c_void_p), ("bounds", C.c_void_p), ("q_begin", C.c_void_p), ("q_octave", C.c_void_p),
                ("q_desc", C.c_void_p), ("q_angle", C.c_void_p), ("prev_matched", C.c_void_p), ("window", C.c_int32),
                ("nnratio", C.c_float), ("check_orientation", C.c_int32)]


_INIT_KEYS = [("kp_begin", np.int32), ("kp_xy", np.float32), ("kp_octave", np.int32), ("kp_desc", np.uint8),
              ("kp_angle", np.float32), ("bounds", np.float32), ("q_begin", np.int32), ("q_octave", np.int32),
              ("q_desc", np.uint8), ("q_angle", np.float32)]


def search_for_initialization(b):
    """ORBmatcher::SearchForInitialization per pair (ORBmatcher.cc:614-694).  b: dict of numpy arrays
    (orbm_init_batch fields).  Returns (matches12, n_matches, prev_matched after the call); b is not
    modified."""
    keep = _Keep()
    P = len(b["kp_begin"]) - 1
    prev = np.ascontiguousarray(b["prev_matched"], np.float32).copy()
    ptrs = [keep(b[k], dt) for k, dt in _INIT_KEYS]
    ib = InitBatch(P, int(b["kp_begin"][-1]), int(b["q_begin"][-1]), *ptrs, ptr(prev), int(b["window"]),
                   float(b["nnratio"]), int(bool(b["check_orientation"])))
    m12 = np.zeros(max(ib.total_q, 1), np.int32)
    n = np.zeros(max(P, 1), np.int32)
    assert lib().oracle_search_for_initialization(C.byref(ib), ptr(m12), ptr(n)) == 0
    return m12[:ib.total_q], n[:P], prev


class RelocBatch(C.Structure):
    _fields_ = [("n_frames", C.c_int32), ("total_kp", C.c_int32), ("total_mp", C.c_int32),
                ("kp_begin", C.c_void_p), ("kp_xy", C.c_void_p), ("kp_octave", C.c_void_p), ("kp_desc", C.c_void_p),
                ("kp_angle", C.c_void_p), ("kp_claimed", C.c_void_p), ("bounds", C.c_void_p), ("pose", C.c_void_p),
                ("camera", C.c_void_p), ("mp_begin", C.c_void_p), ("mp_valid", C.c_void_p), ("mp_xw", C.c_void_p),
                ("mp_max_min", C.c_void_p), ("mp_desc", C.c_void_p), ("mp_angle", C.c_void_p), ("n_levels", C.c_int32),
                ("scale_factors", C.c_void_p), ("log_scale_factor", C.c_float), ("th", C.c_float),
                ("orb_dist", C.c_int32), ("check_orientation", C.c_int32)]


_RELOC_KEYS = [("kp_begin", np.int32), ("kp_xy", np.float32), ("kp_octave", np.int32), ("kp_desc", np.uint8),
               ("kp_angle", np.float32), ("kp_claimed", np.uint8), ("bounds", np.float32), ("pose", np.float32),
               ("camera", np.float32), ("mp_begin", np.int32), ("mp_valid", np.uint8), ("mp_xw", np.float32),
               ("mp_max_min", np.float32), ("mp_desc", np.uint8), ("mp_angle", np.float32)]


def search_by_projection_reloc(b):
    """SearchByProjection(Frame&, KeyFrame*, alreadyFound, th, ORBdist) per frame (ORBmatcher.cc:1364-1445)."""
    keep = _Keep()
    F = len(b["kp_begin"]) - 1
    ptrs = [keep(b[k], dt) if b.get(k) is not None else None for k, dt in _RELOC_KEYS]
    rb = RelocBatch(F, int(b["kp_begin"][-1]), int(b["mp_begin"][-1]), *ptrs, len(b["scale_factors"]),
                    keep(b["scale_factors"], np.float32), float(b["log_scale_factor"]), float(b["th"]),
                    int(b["orb_dist"]), int(bool(b["check_orientation"])))
    km = np.zeros(max(rb.total_kp, 1), np.int32)
    n = np.zeros(max(F, 1), np.int32)
    assert lib().oracle_search_by_projection_reloc(C.byref(rb), ptr(km), ptr(n)) == 0
    return km[:rb.total_kp], n[:F]
