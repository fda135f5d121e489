"""ORBmatcher mirror for the Hamming hot loops (include/ORBmatcher.h, src/ORBmatcher.cc)."""
import ctypes as C

import numpy as np

from ._lib import TriFrame, check, lib, ptr, stream_ptr, tptr

TH_HIGH = 100   # src/ORBmatcher.cc:41
TH_LOW = 50     # src/ORBmatcher.cc:42
HISTO_LENGTH = 30


class ORBmatcher:
    def __init__(self, nnratio: float = 0.6, checkOri: bool = True):
        self.fNNRatio_ = float(nnratio)
        self.checkOrientation_ = bool(checkOri)

    @staticmethod
    def DescriptorDistance(a, b) -> int:
        """static int DescriptorDistance(const cv::Mat&, const cv::Mat&) (src/ORBmatcher.cc:1449-1457)."""
        a = np.ascontiguousarray(a, np.uint8).reshape(32)
        b = np.ascontiguousarray(b, np.uint8).reshape(32)
        return lib().orbm_descriptor_distance(ptr(a), ptr(b))

    def MatchBruteForce(self, descA, descB, th_low: int = TH_LOW, keypointsA=None, keypointsB=None):
        """Best / second-best search of every row of A over all rows of B with the reference loop
        semantics (src/ORBmatcher.cc:477-507).  Returns (best_idx, best, second, match).

        With checkOri (the constructor's default, as ORBmatcher(nnratio, checkOri=true)) the
        rotation-histogram filter CheckOrientation (:249-309) is applied to `match` as
        SearchForInitialization does (:676-686); it needs the keypoint angles, so keypointsA /
        keypointsB (KP_DTYPE arrays or float angle arrays) are then required."""
        A = np.ascontiguousarray(descA, np.uint8).reshape(-1, 32)
        B = np.ascontiguousarray(descB, np.uint8).reshape(-1, 32)
        nA = len(A)
        bi, bd, sd, m = (np.zeros(nA, np.int32) for _ in range(4))
        if self.checkOrientation_ and (keypointsA is None or keypointsB is None):
            raise ValueError("ORBmatcher(checkOri=True): MatchBruteForce needs keypointsA / keypointsB "
                             "(CheckOrientation reads their angles)")
        check(lib().orbm_bf_match(ptr(A), nA, ptr(B), len(B), C.c_float(self.fNNRatio_), th_low, ptr(bi), ptr(bd),
                                  ptr(sd), ptr(m)), "orbm_bf_match")
        if self.checkOrientation_:
            angA, angB = _angles(keypointsA), _angles(keypointsB)
            if len(angA) != nA or len(angB) != len(B):
                raise ValueError("keypoints and descriptors differ in length")
            n = C.c_int32(0)
            check(lib().orbm_check_orientation(ptr(angA), nA, ptr(angB), len(angB), ptr(m), C.byref(n)),
                  "orbm_check_orientation")
        return bi, bd, sd, m

    def match_batch_device(self, descA, nA, descB, nB, th_low: int = TH_LOW, out=None, stream=None, pair_b=None,
                           kpsA=None, kpsB=None, nmatches=None):
        """Batched pairs on the GPU: descA [P, capA, 32], nA [P] int32, descB [Q, capB, 32], nB [Q];
        pair p uses B frame pair_b[p] (int32 [P] tensor) or p when pair_b is None.
        Returns int32 tensor [4, P, capA] = (best_idx, best, second, match).  With checkOri,
        CheckOrientation runs on `match` (kpsA [P, capA, 7] / kpsB [Q, capB, 7], the
        extract_batch_device keypoint slots, are then required; nmatches [P] int32 receives the
        kept counts when given)."""
        import torch
        P, capA = descA.shape[0], descA.shape[1]
        if self.checkOrientation_ and (kpsA is None or kpsB is None):
            raise ValueError("ORBmatcher(checkOri=True): match_batch_device needs kpsA / kpsB")
        if out is None:
            out = torch.empty((4, P, capA), dtype=torch.int32, device=descA.device)
        pb = tptr(pair_b) if pair_b is not None else None
        check(lib().orbm_bf_match_batch_device(tptr(descA), tptr(nA), capA, tptr(descB), tptr(nB), descB.shape[1], pb,
                                               P, C.c_float(self.fNNRatio_), th_low, tptr(out[0]), tptr(out[1]),
                                               tptr(out[2]), tptr(out[3]), stream_ptr(stream)),
              "orbm_bf_match_batch_device")
        if self.checkOrientation_:
            for t, cap in ((kpsA, capA), (kpsB, descB.shape[1])):
                if t.dim() != 3 or t.shape[1] != cap or t.shape[2] != 7 or not t.is_contiguous():
                    raise ValueError("keypoint slots must be contiguous [frames, cap, 7] like the descriptors")
            angA = C.c_void_p(kpsA.data_ptr() + 12)   # &kps[0].angle (orbx_keypoint: x y size angle ...)
            angB = C.c_void_p(kpsB.data_ptr() + 12)
            check(lib().orbm_check_orientation_batch_device(angA, 7, capA, tptr(nA), angB, 7, descB.shape[1], pb, P,
                                                            tptr(out[3]), capA,
                                                            tptr(nmatches) if nmatches is not None else None,
                                                            stream_ptr(stream)),
                  "orbm_check_orientation_batch_device")
        return out

    def SearchForTriangulation(self, kf1, kf2, F12, onlyStereo: bool = False):
        """int SearchForTriangulation(kf1, kf2, F12, matchIds, onlyStereo) (src/ORBmatcher.cc:768-866).

        kf1/kf2: dicts with keys xy [N,2] f32, octave [N], uright [N], has_mappoint [N] bool,
        desc [N,32] u8, fv = (node_ids ascending, offsets, indices) (DBoW2 FeatureVector as CSR),
        scale_factors [L], sigma2 [L] (kf2's pyramid), ep2 = projection of kf1's centre in kf2
        (computed by the caller, :772-773).  Returns the (idx1, idx2) pairs sorted by idx1."""
        keep = []

        def k(a, dt):
            a = np.ascontiguousarray(a, dt)
            keep.append(a)
            return ptr(a)

        def frame(kf):
            ids, off, idx = kf["fv"]
            return TriFrame(len(kf["xy"]), k(kf["xy"], np.float32), k(kf["octave"], np.int32),
                            k(kf["uright"], np.float32), k(kf["has_mappoint"], np.uint8), k(kf["desc"], np.uint8),
                            len(ids), k(ids, np.uint32), k(off, np.int32), k(idx, np.int32))

        f1, f2 = frame(kf1), frame(kf2)
        n1 = f1.n
        out = np.zeros(max(n1, 1), np.int32)
        nm = C.c_int32(0)
        L = len(kf2["scale_factors"])
        check(lib().orbm_search_for_triangulation(C.byref(f1), C.byref(f2), k(F12, np.float32), k(kf2["ep2"], np.float32),
                                                  k(kf2["scale_factors"], np.float32), k(kf2["sigma2"], np.float32),
                                                  L, int(onlyStereo), ptr(out), C.byref(nm)),
              "orbm_search_for_triangulation")
        out = out[:n1]
        idx1 = np.nonzero(out >= 0)[0]
        return [(int(i), int(out[i])) for i in idx1], out


def _check_fv(fv, n_frames: int, name: str):
    """A FeatureVector batch (node [F, fv_cap], off [F, fv_cap + 1], idx [F, fv_cap], n_nodes [F]) as
    ORBVocabulary.transform_batch_device returns it: contiguous int32 tensors of consistent shapes
    covering at least n_frames frames (the kernels read fv_cap from node's width)."""
    import torch
    if not isinstance(fv, (tuple, list)) or len(fv) != 4:
        raise ValueError(f"{name} must be (node, off, idx, n_nodes)")
    node, off, idx, nn = fv
    for t in fv:
        if not isinstance(t, torch.Tensor) or t.dtype != torch.int32 or not t.is_contiguous():
            raise ValueError(f"{name}: every FeatureVector tensor must be a contiguous int32 tensor")
    if node.dim() != 2:
        raise ValueError(f"{name}: node must be [F, fv_cap]")
    F, cap = int(node.shape[0]), int(node.shape[1])
    if tuple(off.shape) != (F, cap + 1) or tuple(idx.shape) != (F, cap) or tuple(nn.shape) != (F,):
        raise ValueError(f"{name}: off / idx / n_nodes must be [F, fv_cap + 1] / [F, fv_cap] / [F]")
    if F < n_frames:
        raise ValueError(f"{name}: {F} frames, {n_frames} needed")


def _check_frames(t, P: int, name: str):
    """An optional per-pair frame index tensor: contiguous int32 [P] (values must index the slot set)."""
    import torch
    if t is None:
        return
    if not isinstance(t, torch.Tensor) or t.dtype != torch.int32 or not t.is_contiguous() or t.dim() != 1 or \
            int(t.shape[0]) < P:
        raise ValueError(f"{name} must be a contiguous int32 [P] tensor")


def search_for_triangulation_batch_device(kps1, desc1, counts1, kps2, desc2, counts2, F12, ep2, scale_factors2,
                                          sigma2, frame1=None, frame2=None, uright1=None, uright2=None,
                                          has_mappoint1=None, has_mappoint2=None, fv1=None, fv2=None,
                                          only_stereo=False, out=None, stream=None):
    """Batched SearchForTriangulation (src/ORBmatcher.cc:768-866) on extract_batch_device slots.

    kps*/desc*/counts*: [F, cap, 7] int32 / [F, cap, 32] uint8 / [F] int32 tensors; pair p matches
    frame frame1[p] of set 1 against frame2[p] of set 2 (int32 [P] tensors, default p); F12 [P, 9]
    and ep2 [P, 2] float32 device tensors (the caller's ComputeF12 and epipole); scale_factors2 /
    sigma2 host arrays (kf2's pyramid); uright* float32 [F, cap] / has_mappoint* uint8 [F, cap] or
    None; fv1 / fv2 = (node, off, idx, n_nodes) from ORBVocabulary.transform_batch_device, or None
    for a single node holding every keypoint.  Returns (match12 [P, cap1] int32, nmatches [P])."""
    import torch
    from ._lib import TriBatch
    P = int(F12.shape[0])
    cap1, cap2 = int(kps1.shape[1]), int(kps2.shape[1])
    for k, d, cap in ((kps1, desc1, cap1), (kps2, desc2, cap2)):
        if k.dim() != 3 or k.shape[2] != 7 or d.shape[:2] != k.shape[:2] or d.shape[2] != 32 or \
                not k.is_contiguous() or not d.is_contiguous():
            raise ValueError("keypoint / descriptor slots must be contiguous [F, cap, 7] / [F, cap, 32]")
    if ep2.shape[0] != P or F12.shape[-1] != 9 or ep2.shape[-1] != 2:
        raise ValueError("F12 must be [P, 9] and ep2 [P, 2]")
    _check_frames(frame1, P, "frame1")
    _check_frames(frame2, P, "frame2")
    if fv1 is not None:
        _check_fv(fv1, int(kps1.shape[0]), "fv1")
    if fv2 is not None:
        _check_fv(fv2, int(kps2.shape[0]), "fv2")
    if out is None:
        out = (torch.empty((P, cap1), dtype=torch.int32, device=kps1.device),
               torch.empty((P,), dtype=torch.int32, device=kps1.device))
    sf = np.ascontiguousarray(scale_factors2, np.float32)
    s2 = np.ascontiguousarray(sigma2, np.float32)
    opt = lambda t: tptr(t) if t is not None else None   # noqa: E731
    f1 = fv1 if fv1 is not None else (None,) * 4
    f2 = fv2 if fv2 is not None else (None,) * 4
    b = TriBatch(P, cap1, cap2, tptr(kps1), tptr(desc1), tptr(counts1), opt(uright1), opt(has_mappoint1),
                 tptr(kps2), tptr(desc2), tptr(counts2), opt(uright2), opt(has_mappoint2), opt(frame1), opt(frame2),
                 tptr(F12), tptr(ep2), *[opt(t) for t in f1], *[opt(t) for t in f2],
                 int(f1[0].shape[1]) if fv1 is not None else 0, int(f2[0].shape[1]) if fv2 is not None else 0,
                 len(sf), ptr(sf), ptr(s2), int(only_stereo))
    check(lib().orbm_search_for_triangulation_batch_device(C.byref(b), tptr(out[0]), tptr(out[1]),
                                                           stream_ptr(stream)),
          "orbm_search_for_triangulation_batch_device")
    return out


def search_by_bow_batch_device(kps1, desc1, fv1, kps2, desc2, counts2, fv2, frame1=None, mp_valid1=None,
                               nnratio: float = 0.6, checkOri: bool = True, out=None, stream=None):
    """Batched SearchByBoW(KeyFrame*, Frame&, matches) (src/ORBmatcher.cc:452-516) on extract_batch_device
    slots: pair p matches keyframe frame1[p] of set 1 (int32 [P] tensor, default p) against frame p of
    set 2.  kps*/desc* [F, cap, 7] / [F, cap, 32]; counts2 [P]; fv1 / fv2 = (node, off, idx, n_nodes)
    from ORBVocabulary.transform_batch_device; mp_valid1 uint8 [F1, cap1] (MapPoint non-null and not
    bad; None = all valid).  checkOri applies CheckOrientation (:512-513).  Returns (match [P, cap2]
    int32 = keyframe feature idx1 or -1 per frame feature, nmatches [P])."""
    import torch
    from ._lib import BowBatch
    P = int(counts2.shape[0])
    cap1, cap2 = int(desc1.shape[1]), int(desc2.shape[1])
    for k, d in ((kps1, desc1), (kps2, desc2)):
        if k.dim() != 3 or k.shape[2] != 7 or d.shape[:2] != k.shape[:2] or d.shape[2] != 32 or \
                not k.is_contiguous() or not d.is_contiguous():
            raise ValueError("keypoint / descriptor slots must be contiguous [F, cap, 7] / [F, cap, 32]")
    if desc2.shape[0] < P:
        raise ValueError("set 2 needs one frame per pair")
    _check_frames(frame1, P, "frame1")
    _check_fv(fv1, int(desc1.shape[0]), "fv1")
    _check_fv(fv2, P, "fv2")
    if out is None:
        out = (torch.empty((P, cap2), dtype=torch.int32, device=desc2.device),
               torch.empty((P,), dtype=torch.int32, device=desc2.device))
    opt = lambda t: tptr(t) if t is not None else None   # noqa: E731
    b = BowBatch(P, cap1, cap2, tptr(kps1), tptr(desc1), opt(mp_valid1), opt(frame1), tptr(kps2), tptr(desc2),
                 tptr(counts2), *[tptr(t) for t in fv1], *[tptr(t) for t in fv2], int(fv1[0].shape[1]),
                 int(fv2[0].shape[1]), float(nnratio), int(bool(checkOri)), None, None, None)
    check(lib().orbm_search_by_bow_batch_device(C.byref(b), tptr(out[0]), tptr(out[1]), stream_ptr(stream)),
          "orbm_search_by_bow_batch_device")
    return out


def search_by_bow_kf_batch_device(kps1, desc1, counts1, fv1, kps2, desc2, counts2, fv2, n_pairs=None, frame1=None,
                                  frame2=None, mp_valid1=None, mp_valid2=None, nnratio: float = 0.6,
                                  checkOri: bool = True, out=None, stream=None):
    """Batched SearchByBoW(KeyFrame* kf1, KeyFrame* kf2, matches12) (src/ORBmatcher.cc:696-766): pair p =
    (kf1 frame1[p] of set 1, kf2 frame2[p] of set 2; default p).  mp_valid* uint8 [F, cap] (None = all
    valid).  Returns (match12 [P, cap1] int32 = idx2 or -1 per kf1 feature, nmatches [P])."""
    import torch
    from ._lib import BowBatch
    P = int(n_pairs if n_pairs is not None else (frame1.shape[0] if frame1 is not None else desc1.shape[0]))
    cap1, cap2 = int(desc1.shape[1]), int(desc2.shape[1])
    for k, d in ((kps1, desc1), (kps2, desc2)):
        if k.dim() != 3 or k.shape[2] != 7 or d.shape[:2] != k.shape[:2] or d.shape[2] != 32 or \
                not k.is_contiguous() or not d.is_contiguous():
            raise ValueError("keypoint / descriptor slots must be contiguous [F, cap, 7] / [F, cap, 32]")
    _check_frames(frame1, P, "frame1")
    _check_frames(frame2, P, "frame2")
    if frame1 is None and desc1.shape[0] < P or frame2 is None and desc2.shape[0] < P:
        raise ValueError("without frame1 / frame2 each set needs one frame per pair")
    _check_fv(fv1, int(desc1.shape[0]), "fv1")
    _check_fv(fv2, int(desc2.shape[0]), "fv2")
    if out is None:
        out = (torch.empty((P, cap1), dtype=torch.int32, device=desc1.device),
               torch.empty((P,), dtype=torch.int32, device=desc1.device))
    opt = lambda t: tptr(t) if t is not None else None   # noqa: E731
    b = BowBatch(P, cap1, cap2, tptr(kps1), tptr(desc1), opt(mp_valid1), opt(frame1), tptr(kps2), tptr(desc2),
                 tptr(counts2), *[tptr(t) for t in fv1], *[tptr(t) for t in fv2], int(fv1[0].shape[1]),
                 int(fv2[0].shape[1]), float(nnratio), int(bool(checkOri)), tptr(counts1), opt(mp_valid2),
                 opt(frame2))
    check(lib().orbm_search_by_bow_kf_batch_device(C.byref(b), tptr(out[0]), tptr(out[1]), stream_ptr(stream)),
          "orbm_search_by_bow_kf_batch_device")
    return out


def _angles(kps):
    """float32 angles from a KP_DTYPE keypoint array, an [N, 7] slot array or a plain angle array."""
    from ._lib import KP_DTYPE
    a = np.asarray(kps)
    if a.dtype == KP_DTYPE:
        return np.ascontiguousarray(a["angle"], np.float32)
    if a.ndim == 2 and a.shape[1] == 7:
        return np.ascontiguousarray(np.ascontiguousarray(a).view(np.float32)[:, 3])
    return np.ascontiguousarray(a, np.float32).reshape(-1)


def _stereo_view(kps, desc, pyramid):
    from ._lib import KP_DTYPE, StereoView
    kps = np.ascontiguousarray(kps)
    if kps.dtype != KP_DTYPE:
        kps = kps.view(KP_DTYPE).reshape(-1)
    desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    levels = [np.ascontiguousarray(im, np.uint8) for im in pyramid]
    ptrs = (C.c_void_p * len(levels))(*[im.ctypes.data for im in levels])
    rows = np.array([im.shape[0] for im in levels], np.int32)
    cols = np.array([im.shape[1] for im in levels], np.int32)
    step = np.array([im.strides[0] for im in levels], np.int32)
    v = StereoView(len(kps), kps.ctypes.data, desc.ctypes.data, len(levels), C.cast(ptrs, C.c_void_p),
                   rows.ctypes.data, cols.ctypes.data, step.ctypes.data)
    return v, (kps, desc, levels, ptrs, rows, cols, step)


def ComputeStereoMatches(keypointsL, descriptorsL, pyramidL, keypointsR, descriptorsR, pyramidR, scaleFactors,
                         invScaleFactors, bf: float, baseline: float):
    """ComputeStereoMatches (src/ORBmatcher.cc:72-247): keypoints as KP_DTYPE arrays (level-0
    coordinates), descriptors [N,32] u8, pyramids = lists of unblurred level images
    (ORBextractor.GetImagePyramid()).  Returns (uright, depth), float32 [N_left], -1 = no match."""
    vl, keep_l = _stereo_view(keypointsL, descriptorsL, pyramidL)
    vr, keep_r = _stereo_view(keypointsR, descriptorsR, pyramidR)
    n = vl.n
    ur = np.full(n, -1, np.float32)
    dp = np.full(n, -1, np.float32)
    s = np.ascontiguousarray(scaleFactors, np.float32)
    inv = np.ascontiguousarray(invScaleFactors, np.float32)
    check(lib().orbm_compute_stereo_matches(C.byref(vl), C.byref(vr), ptr(s), ptr(inv), C.c_float(bf),
                                            C.c_float(baseline), ptr(ur), ptr(dp)), "orbm_compute_stereo_matches")
    return ur, dp


def ComputeStereoMatchesLast(extractor_l, extractor_r, n_left: int, bf: float, baseline: float):
    """ComputeStereoMatches at the reference's call shape (System.cc:449-461: Extract L and R, then
    ComputeStereoMatches on mvKeys / mvKeysRight and both mvImagePyramid): on the two extractors' last
    single-frame Extract, whose keypoints, descriptors and pyramids are still on the device.  n_left =
    the left Extract's keypoint count.  Returns (uright, depth), float32 [n_left], -1 = no match."""
    ur = np.full(n_left, -1, np.float32)
    dp = np.full(n_left, -1, np.float32)
    check(lib().orbx_stereo_matches_last(extractor_l._h, extractor_r._h, C.c_float(bf), C.c_float(baseline), ptr(ur),
                                         ptr(dp), int(n_left)), "orbx_stereo_matches_last")
    return ur, dp


def stereo_matches_batch_device(extractor_l, extractor_r, outs_l, outs_r, bf: float, baseline: float, out=None,
                                stream=None):
    """Batched ComputeStereoMatches on the frames of two extractors' last batches.  outs_l / outs_r are
    the (kps, desc, counts) tensors those extract_batch_device calls returned.  Returns float32
    tensors (uright, depth) of shape [F, cap]."""
    import torch
    kl, dl, cl = outs_l
    kr, dr, cr = outs_r
    F, cap = kl.shape[0], kl.shape[1]
    if out is None:
        out = (torch.empty((F, cap), dtype=torch.float32, device=kl.device),
               torch.empty((F, cap), dtype=torch.float32, device=kl.device))
    check(lib().orbx_stereo_matches_batch_device(extractor_l._h, extractor_r._h, F, tptr(kl), tptr(dl), tptr(cl),
                                                 tptr(kr), tptr(dr), tptr(cr), cap, C.c_float(bf),
                                                 C.c_float(baseline), tptr(out[0]), tptr(out[1]), stream_ptr(stream)),
          "orbx_stereo_matches_batch_device")
    return out


def _proj_struct(b: dict, conv, total_kp: int, total_mp: int):
    """orbm_proj_batch from a make_proj_batch-style dict; `conv(array, dtype)` returns a pointer."""
    from ._lib import ProjBatch
    F = len(b["kp_begin"]) - 1
    claimed = b.get("kp_claimed")
    sf = np.ascontiguousarray(b["scale_factors"], np.float32)
    return ProjBatch(F, total_kp, total_mp, conv(b["kp_begin"], np.int32),
                     conv(b["kp_xy"], np.float32), conv(b["kp_octave"], np.int32), conv(b["kp_uright"], np.float32),
                     conv(b["kp_desc"], np.uint8), conv(claimed, np.uint8) if claimed is not None else None,
                     conv(b["bounds"], np.float32), conv(b["mp_begin"], np.int32), conv(b["mp_valid"], np.uint8),
                     conv(b["mp_proj"], np.float32), conv(b["mp_view_cos"], np.float32), conv(b["mp_level"], np.int32),
                     conv(b["mp_desc"], np.uint8), conv(b["mp_has_obs"], np.uint8), len(sf), ptr(sf),
                     float(b["th"]), float(b["nnratio"])), sf


def SearchByProjection(batch: dict, device: int = 0):
    """int ORBmatcher::SearchByProjection(Frame& frame, const std::vector<MapPoint*>& mappoints, float th)
    (include/ORBmatcher.h:58, src/ORBmatcher.cc:315-382) with the frame's FeaturesGrid, batched over frames.
    Returns (kp_match, n_matches): kp_match[k] = frame-relative index of the map point assigned to
    keypoint k by this call (frame.mappoints[bestIdx] = mappoint), -1 if none; n_matches per frame."""
    keep = []

    def conv(a, dt):
        a = np.ascontiguousarray(a, dt)
        keep.append(a)
        return ptr(a)

    pb, sf = _proj_struct(batch, conv, int(batch["kp_begin"][-1]), int(batch["mp_begin"][-1]))
    kp_match = np.zeros(max(pb.total_kp, 1), np.int32)
    n = np.zeros(max(pb.n_frames, 1), np.int32)
    check(lib().orbm_search_by_projection(C.byref(pb), ptr(kp_match), ptr(n), device), "orbm_search_by_projection")
    return kp_match[:pb.total_kp], n[:pb.n_frames]


def search_by_projection_device(batch: dict, kp_match=None, n_matches=None, stream=None):
    """Device form: array values of `batch` are torch tensors on the GPU (scale_factors / th / nnratio
    stay host values); one enqueue of the grid, score and walk kernels on `stream`."""
    import torch
    from ._lib import stream_ptr, tptr
    eb = batch["kp_begin"]
    F = eb.numel() - 1
    K = int(batch["kp_xy"].shape[0])
    dev = eb.device
    if kp_match is None:
        kp_match = torch.empty(max(K, 1), dtype=torch.int32, device=dev)
    if n_matches is None:
        n_matches = torch.empty(max(F, 1), dtype=torch.int32, device=dev)

    def conv(t, dt):
        return tptr(t)

    pb, sf = _proj_struct(batch, conv, K, int(batch["mp_proj"].shape[0]))
    check(lib().orbm_search_by_projection_device(C.byref(pb), tptr(kp_match), tptr(n_matches), stream_ptr(stream)),
          "orbm_search_by_projection_device")
    return kp_match, n_matches


_MOTION_KEYS = ("kp_begin", "kp_xy", "kp_octave", "kp_uright", "kp_desc", "kp_angle", "kp_claimed", "bounds",
                "mp_begin", "mp_valid", "mp_proj", "mp_octave", "mp_desc", "mp_has_obs", "mp_angle", "motion")
_MOTION_DT = (np.int32, np.float32, np.int32, np.float32, np.uint8, np.float32, np.uint8, np.float32,
              np.int32, np.uint8, np.float32, np.int32, np.uint8, np.uint8, np.float32, np.int32)

# Element counts the C-ABI batches read per array: (row count symbol, elements per row).  F = frames or
# pairs, F1 = F + 1, K / M / Q = total keypoints / map points / F1-keypoints.  The kernels index by
# these counts with no bound of their own, so a shorter array would be read out of bounds.
_BATCH_ROWS = {
    "kp_begin": ("F1", 1), "q_begin": ("F1", 1), "mp_begin": ("F1", 1),
    "kp_xy": ("K", 2), "kp_octave": ("K", 1), "kp_uright": ("K", 1), "kp_desc": ("K", 32), "kp_angle": ("K", 1),
    "kp_claimed": ("K", 1), "bounds": ("F", 4), "pose": ("F", 12), "camera": ("F", 4), "motion": ("F", 1),
    "mp_valid": ("M", 1), "mp_proj": ("M", 3), "mp_octave": ("M", 1), "mp_desc": ("M", 32), "mp_has_obs": ("M", 1),
    "mp_angle": ("M", 1), "mp_xw": ("M", 3), "mp_max_min": ("M", 2),
    "q_octave": ("Q", 1), "q_desc": ("Q", 32), "q_angle": ("Q", 1), "prev_matched": ("Q", 2),
}


def _check_batch_rows(batch: dict, keys, dims: dict, what: str):
    for k in keys:
        a = batch.get(k)
        if a is None:
            continue
        sym, per = _BATCH_ROWS[k]
        want = dims[sym] * per
        n = int(a.numel()) if hasattr(a, "numel") else int(np.size(a))
        if n < want:
            raise ValueError(f"{what}: {k} has {n} elements, needs {want} ({sym} = {dims[sym]} rows x {per})")


def _check_device_dtypes(batch: dict, keys_dtypes, what: str):
    import torch
    for k, dt in keys_dtypes:
        t = batch.get(k)
        if t is not None and (not t.is_contiguous() or t.dtype != getattr(torch, np.dtype(dt).name)):
            raise ValueError(f"{what}: {k} must be a contiguous {np.dtype(dt).name} tensor")


def search_by_projection_motion_device(batch: dict, kp_match=None, n_matches=None, stream=None):
    """SearchByProjection(Frame& currFrame, const Frame& lastFrame, float th, bool monocular)
    (src/ORBmatcher.cc:1279-1362, TrackWithMotionModel) batched over frames: `batch` holds GPU tensors
    for the orbm_motion_batch arrays (kp_claimed / motion may be None) and host values for
    scale_factors, th and check_orientation.  Returns (kp_match [total_kp], n_matches [F])."""
    import torch
    from ._lib import MotionBatch
    eb = batch["kp_begin"]
    F = eb.numel() - 1
    K = int(batch["kp_xy"].shape[0])
    M = int(batch["mp_proj"].shape[0])
    _check_device_dtypes(batch, zip(_MOTION_KEYS, _MOTION_DT), "search_by_projection_motion_device")
    _check_batch_rows(batch, _MOTION_KEYS, {"F": F, "F1": F + 1, "K": K, "M": M}, "search_by_projection_motion_device")
    if kp_match is None:
        kp_match = torch.empty(max(K, 1), dtype=torch.int32, device=eb.device)
    if n_matches is None:
        n_matches = torch.empty(max(F, 1), dtype=torch.int32, device=eb.device)
    sf = np.ascontiguousarray(batch["scale_factors"], np.float32)
    ptrs = [tptr(batch[k]) if batch.get(k) is not None else None for k in _MOTION_KEYS]
    mb = MotionBatch(F, K, M, *ptrs, len(sf), ptr(sf), float(batch["th"]), int(bool(batch["check_orientation"])))
    check(lib().orbm_search_by_projection_motion_device(C.byref(mb), tptr(kp_match), tptr(n_matches),
                                                        stream_ptr(stream)),
          "orbm_search_by_projection_motion_device")
    return kp_match, n_matches


_INIT_KEYS = (("kp_begin", np.int32), ("kp_xy", np.float32), ("kp_octave", np.int32), ("kp_desc", np.uint8),
              ("kp_angle", np.float32), ("bounds", np.float32), ("q_begin", np.int32), ("q_octave", np.int32),
              ("q_desc", np.uint8), ("q_angle", np.float32), ("prev_matched", np.float32))


def SearchForInitialization(batch: dict, device: int = 0):
    """ORBmatcher::SearchForInitialization(F1, F2, prevMatched, matches12, windowSize)
    (src/ORBmatcher.cc:614-694) batched over pairs, host arrays (orbm_init_batch fields: F2 keypoints
    kp_* with kp_begin, F1 keypoints q_* with q_begin, prev_matched [total_q, 2] float32 updated in
    place, window, nnratio, check_orientation).  Returns (matches12 [total_q] = F2-relative idx2 or
    -1, n_matches [P])."""
    from ._lib import InitBatch
    arrs = {k: np.ascontiguousarray(batch[k], dt) for k, dt in _INIT_KEYS if batch.get(k) is not None}
    if arrs["prev_matched"] is not batch["prev_matched"]:
        raise ValueError("prev_matched must be a contiguous float32 array (updated in place)")
    P = len(arrs["kp_begin"]) - 1
    K, Q = int(arrs["kp_begin"][-1]), int(arrs["q_begin"][-1])
    _check_batch_rows(arrs, arrs.keys(), {"F": P, "F1": P + 1, "K": K, "Q": Q}, "SearchForInitialization")
    m12 = np.empty(max(Q, 1), np.int32)
    nm = np.empty(max(P, 1), np.int32)
    ib = InitBatch(P, K, Q, *[ptr(arrs[k]) if k in arrs else None for k, _ in _INIT_KEYS], int(batch["window"]),
                   float(batch["nnratio"]), int(bool(batch["check_orientation"])))
    check(lib().orbm_search_for_initialization(C.byref(ib), ptr(m12), ptr(nm), int(device)),
          "orbm_search_for_initialization")
    return m12[:Q], nm[:P]


def search_for_initialization_device(batch: dict, matches12=None, n_matches=None, stream=None):
    """Device form of SearchForInitialization: `batch` holds GPU tensors for the orbm_init_batch arrays
    (prev_matched float32 [total_q, 2] is updated in place) and host values for window, nnratio and
    check_orientation.  Returns (matches12 [total_q], n_matches [P]); n_matches[p] = -1 when a frame of
    the pair has more than ORBM_PROJ_MAX_KP keypoints."""
    import torch
    from ._lib import InitBatch
    kb, qb = batch["kp_begin"], batch["q_begin"]
    P = kb.numel() - 1
    if qb.numel() != P + 1:
        raise ValueError("kp_begin and q_begin must both have n_pairs + 1 entries")
    _check_device_dtypes(batch, _INIT_KEYS, "search_for_initialization_device")
    K, Q = int(batch["kp_xy"].shape[0]), int(batch["q_octave"].shape[0])
    _check_batch_rows(batch, [k for k, _ in _INIT_KEYS], {"F": P, "F1": P + 1, "K": K, "Q": Q},
                      "search_for_initialization_device")
    if matches12 is None:
        matches12 = torch.empty(max(Q, 1), dtype=torch.int32, device=kb.device)
    if n_matches is None:
        n_matches = torch.empty(max(P, 1), dtype=torch.int32, device=kb.device)
    ib = InitBatch(P, K, Q, *[tptr(batch[k]) if batch.get(k) is not None else None for k, _ in _INIT_KEYS],
                   int(batch["window"]), float(batch["nnratio"]), int(bool(batch["check_orientation"])))
    check(lib().orbm_search_for_initialization_device(C.byref(ib), tptr(matches12), tptr(n_matches), stream_ptr(stream)),
          "orbm_search_for_initialization_device")
    return matches12, n_matches


_RELOC_KEYS = (("kp_begin", np.int32), ("kp_xy", np.float32), ("kp_octave", np.int32), ("kp_desc", np.uint8),
               ("kp_angle", np.float32), ("kp_claimed", np.uint8), ("bounds", np.float32), ("pose", np.float32),
               ("camera", np.float32), ("mp_begin", np.int32), ("mp_valid", np.uint8), ("mp_xw", np.float32),
               ("mp_max_min", np.float32), ("mp_desc", np.uint8), ("mp_angle", np.float32))


def _reloc_struct(batch, conv, K, M):
    from ._lib import RelocBatch
    sf = np.ascontiguousarray(batch["scale_factors"], np.float32)
    F = len(batch["kp_begin"]) - 1
    rb = RelocBatch(F, K, M, *[conv(batch[k], dt) if batch.get(k) is not None else None for k, dt in _RELOC_KEYS],
                    len(sf), ptr(sf), float(batch["log_scale_factor"]), float(batch["th"]), int(batch["orb_dist"]),
                    int(bool(batch["check_orientation"])))
    return rb, sf


def SearchByProjectionReloc(batch: dict, device: int = 0):
    """ORBmatcher::SearchByProjection(Frame& frame, KeyFrame* keyframe, alreadyFound, th, ORBdist)
    (src/ORBmatcher.cc:1364-1445, Tracking::Relocalization) batched over (frame, keyframe) pairs, host
    arrays (orbm_reloc_batch fields; kp_claimed may be None).  Returns (kp_match [total_kp] = keyframe
    idx1 assigned to each frame keypoint or -1, n_matches [F])."""
    keep = []

    def conv(a, dt):
        a = np.ascontiguousarray(a, dt)
        keep.append(a)
        return ptr(a)
    F = len(batch["kp_begin"]) - 1
    K, M = int(batch["kp_begin"][-1]), int(batch["mp_begin"][-1])
    _check_batch_rows(batch, [k for k, _ in _RELOC_KEYS], {"F": F, "F1": F + 1, "K": K, "M": M},
                      "SearchByProjectionReloc")
    rb, _sf = _reloc_struct(batch, conv, K, M)
    km = np.empty(max(K, 1), np.int32)
    nm = np.empty(max(F, 1), np.int32)
    check(lib().orbm_search_by_projection_reloc(C.byref(rb), ptr(km), ptr(nm), int(device)),
          "orbm_search_by_projection_reloc")
    return km[:K], nm[:F]


def search_by_projection_reloc_device(batch: dict, kp_match=None, n_matches=None, stream=None):
    """Device form of SearchByProjectionReloc: GPU tensors for the orbm_reloc_batch arrays, host values for
    scale_factors, log_scale_factor, th, orb_dist and check_orientation."""
    import torch
    kb = batch["kp_begin"]
    F = kb.numel() - 1
    K, M = int(batch["kp_xy"].shape[0]), int(batch["mp_xw"].shape[0])
    _check_device_dtypes(batch, _RELOC_KEYS, "search_by_projection_reloc_device")
    _check_batch_rows(batch, [k for k, _ in _RELOC_KEYS], {"F": F, "F1": F + 1, "K": K, "M": M},
                      "search_by_projection_reloc_device")
    if kp_match is None:
        kp_match = torch.empty(max(K, 1), dtype=torch.int32, device=kb.device)
    if n_matches is None:
        n_matches = torch.empty(max(F, 1), dtype=torch.int32, device=kb.device)
    rb, _sf = _reloc_struct(batch, lambda t, dt: tptr(t), K, M)
    check(lib().orbm_search_by_projection_reloc_device(C.byref(rb), tptr(kp_match), tptr(n_matches),
                                                       stream_ptr(stream)),
          "orbm_search_by_projection_reloc_device")
    return kp_match, n_matches
