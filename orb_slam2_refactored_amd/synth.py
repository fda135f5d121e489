"""Seeded synthetic inputs.  No datasets are available offline.

G(seed, W, H): background 128, 300 filled axis-aligned rectangles with uniform random
corners and uniform gray level 0..255 painted in order, plus i.i.d. integer noise U{-6..6},
clipped to u8.  Rectangle corners give FAST corners at every pyramid level.
"""
import numpy as np


def synth_image(seed: int, width: int, height: int, n_rects: int = 300) -> np.ndarray:
    rng = np.random.default_rng(seed)
    img = np.full((height, width), 128, np.int16)
    xs = np.sort(rng.integers(0, width, size=(n_rects, 2)), axis=1)
    ys = np.sort(rng.integers(0, height, size=(n_rects, 2)), axis=1)
    gray = rng.integers(0, 256, size=n_rects)
    for (x0, x1), (y0, y1), g in zip(xs, ys, gray):
        img[y0:y1 + 1, x0:x1 + 1] = g
    img += rng.integers(-6, 7, size=(height, width)).astype(np.int16)
    return np.clip(img, 0, 255).astype(np.uint8)


def shifted_pair(seed: int, width: int, height: int, dx: int = 3, dy: int = 2):
    """C2 pair: A = G(seed), B = A shifted by (dx, dy) with edge replicate + fresh noise."""
    a = synth_image(seed, width, height)
    base = np.pad(a.astype(np.int16), ((dy, 0), (dx, 0)), mode="edge")[:height, :width]
    rng = np.random.default_rng(seed + 1000)
    b = np.clip(base + rng.integers(-3, 4, size=(height, width)), 0, 255).astype(np.uint8)
    return a, b


def pan_sequence(seed: int, width: int, height: int, n: int, dx: int = 3, dy: int = 2) -> np.ndarray:
    """A camera-pan sequence for the C2 / C5 "frame i matched to i-1" workload: frame 0 = G(seed) and
    frame k = G(seed) shifted by k*(dx, dy) with edge replicate plus fresh noise U{-3..3} (frame k and
    k-1 are the shifted pair of SURVEY.md §8d C2; the noise does not accumulate along the chain).
    Returns [n, H, W] uint8."""
    out = np.empty((n, height, width), np.uint8)
    a = synth_image(seed, width, height).astype(np.int16)
    out[0] = a
    rng = np.random.default_rng(seed + 1000)
    for k in range(1, n):
        base = np.pad(a, ((k * dy, 0), (k * dx, 0)), mode="edge")[:height, :width]
        out[k] = np.clip(base + rng.integers(-3, 4, size=(height, width)), 0, 255).astype(np.uint8)
    return out


def textured_image(seed: int, width: int, height: int) -> np.ndarray:
    """Texture-rich frame (FAST fires almost everywhere, thousands of candidates per level):
    low-frequency value noise (1/8 resolution, bilinear) at +-40 grey levels plus per-pixel
    Gaussian noise sigma 12, around 128."""
    rng = np.random.default_rng(seed)
    gh, gw = height // 8 + 2, width // 8 + 2
    g = rng.normal(0, 40, (gh, gw))
    ys = np.arange(height) / 8.0
    xs = np.arange(width) / 8.0
    y0, x0 = ys.astype(int), xs.astype(int)
    fy, fx = (ys - y0)[:, None], (xs - x0)[None, :]
    low = (g[y0][:, x0] * (1 - fy) * (1 - fx) + g[y0 + 1][:, x0] * fy * (1 - fx) +
           g[y0][:, x0 + 1] * (1 - fy) * fx + g[y0 + 1][:, x0 + 1] * fy * fx)
    img = 128 + low + rng.normal(0, 12, (height, width))
    return np.ascontiguousarray(np.clip(np.rint(img), 0, 255).astype(np.uint8))


# KITTI 00-02 intrinsics (Examples/Stereo/KITTI00-02.yaml:8-25)
KITTI = dict(fx=718.856, fy=718.856, cx=607.1928, cy=185.2157, bf=386.1448, width=1241, height=376)


def _rot_y(deg):
    a = np.deg2rad(deg)
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])


def _small_rot(rng, sigma_deg):
    w = rng.normal(0, np.deg2rad(sigma_deg), 3)
    th = np.linalg.norm(w)
    if th < 1e-12:
        return np.eye(3)
    k = w / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def make_ba_problem(seed: int = 0, n_kf: int = 20, n_pts: int = 3000, n_fixed: int = 2, stereo_frac: float = 0.2,
                    outlier_frac: float = 0.03, cam=KITTI, yaw_per_kf: float = 0.5):
    """C4: a LocalBundleAdjustment problem in the flattened orbba_problem layout.

    n_kf local keyframes moving forward along +z (0.5 m apart, 0.5 deg yaw per KF); KF 0 is the
    fixed gauge (`localKF->id == 0`, Optimizer.cc:551) and `n_fixed` extra fixed cameras observe
    some points (the fixedCameras set, :524-537).  Each point is seen by a run of K ~ U{2..6}
    keyframes; 20 % of observations are stereo (ur >= 0), octaves U{0..7} with pixel noise
    N(0, 1.2^oct) and invSigma2 = 1/1.2^(2 oct); 3 % outliers get +-U(15,40) px.  Initial poses
    are perturbed by 0.2 deg / 2 cm and points by 2 % of depth.
    """
    rng = np.random.default_rng(seed)
    P = n_kf + n_fixed
    R_true, t_true, C = [], [], []
    for k in range(P):
        kk = k if k < n_kf else -(k - n_kf + 1)   # fixed cameras behind KF 0
        Rwc = _rot_y(yaw_per_kf * kk)   # long windows: a smaller yaw keeps points in front of every camera
        c = np.array([0.02 * np.sin(kk), 0.0, 0.5 * kk])
        Rcw = Rwc.T
        R_true.append(Rcw)
        t_true.append(-Rcw @ c)
        C.append(c)
    fixed = np.zeros(P, np.uint8)
    fixed[0] = 1
    fixed[n_kf:] = 1
    pts, ep, ek, obs, info, camv = [], [], [], [], [], []
    for p in range(n_pts):
        K = int(rng.integers(2, 7))
        s = int(rng.integers(-n_fixed, n_kf - K + 1))
        kfs = [(k if k >= 0 else n_kf + (-k - 1)) for k in range(s, s + K)]
        zc = max(C[k][2] for k in kfs)
        X = np.array([rng.uniform(-15, 15), rng.uniform(-3, 3), zc + rng.uniform(5, 40)])
        pid = len(pts)
        pts.append(X)
        for k in kfs:
            Xc = R_true[k] @ X + t_true[k]
            u = cam["fx"] * Xc[0] / Xc[2] + cam["cx"]
            v = cam["fy"] * Xc[1] / Xc[2] + cam["cy"]
            octv = int(rng.integers(0, 8))
            sig = 1.2 ** octv
            u += rng.normal(0, sig)
            v += rng.normal(0, sig)
            ur = -1.0
            if rng.random() < stereo_frac:
                ur = u - cam["bf"] / Xc[2] + rng.normal(0, sig)
            if rng.random() < outlier_frac:
                u += rng.choice([-1, 1]) * rng.uniform(15, 40)
                v += rng.choice([-1, 1]) * rng.uniform(15, 40)
                if ur >= 0:
                    ur = u - cam["bf"] / Xc[2]
            ep.append(pid)
            ek.append(k)
            # measurements are floats in the reference (cv::KeyPoint pt, uright)
            obs.append([np.float32(u), np.float32(v), np.float32(ur) if ur >= 0 else -1.0])
            info.append(np.float32(1.0 / (sig * sig)))
            camv.append([np.float32(cam[k2]) for k2 in ("fx", "fy", "cx", "cy", "bf")])
    pose_R = np.zeros((P, 9))
    pose_t = np.zeros((P, 3))
    for k in range(P):
        R, t = R_true[k], t_true[k]
        if not fixed[k]:
            R = _small_rot(rng, 0.2) @ R
            t = t + rng.normal(0, 0.02, 3)
        pose_R[k] = R.reshape(-1)
        pose_t[k] = t
    pts = np.array(pts)
    depth = np.abs(pts[:, 2] - np.mean([c[2] for c in C]))
    pts0 = pts + rng.normal(0, 1, pts.shape) * (0.02 * depth)[:, None]
    return dict(pose_R=pose_R.astype(np.float32).astype(np.float64), pose_t=pose_t.astype(np.float32).astype(np.float64),
                pose_fixed=fixed, points=pts0.astype(np.float32).astype(np.float64),
                edge_point=np.array(ep, np.int32), edge_pose=np.array(ek, np.int32),
                edge_obs=np.array(obs, np.float64), edge_inv_sigma2=np.array(info, np.float64),
                edge_cam=np.array(camv, np.float64), gt_R=np.array([r.reshape(-1) for r in R_true]),
                gt_t=np.array(t_true), gt_points=pts)


STEREO_Z = (5.0, 7.0, 10.0, 14.0, 20.0, 28.0, 40.0, 56.0)   # SURVEY.md §8d C3 band depths (m)


def stereo_pair(seed: int, width: int = 1242, height: int = 375, bf: float = KITTI["bf"]):
    """C3 pair: L = G(seed, W, H); R = L warped by 8 vertical bands at depths STEREO_Z with disparity
    round(bf / Z) (R[y, x] = L[y, x + d]); pixels with no source (x + d >= W) are noise-filled; fresh
    noise U{-3..3} on R.  Returns (L, R, band_depth_of_right_column)."""
    L = synth_image(seed, width, height)
    rng = np.random.default_rng(seed + 2000)
    R = np.empty_like(L, dtype=np.int16)
    zcol = np.empty(width, np.float32)
    edges = np.linspace(0, width, len(STEREO_Z) + 1).astype(int)
    for b, z in enumerate(STEREO_Z):
        d = int(round(bf / z))
        for x in range(edges[b], edges[b + 1]):
            zcol[x] = z
            R[:, x] = L[:, x + d] if x + d < width else rng.integers(0, 256, size=height)
    R += rng.integers(-3, 4, size=R.shape).astype(np.int16)
    return L, np.clip(R, 0, 255).astype(np.uint8), zcol


def stereo_tri_geometry(cam=KITTI):
    """SearchForTriangulation geometry of the C3 setup: KF1 = the left camera at
    [I|0], KF2 = the right camera at [I|(-bf/fx, 0, 0)].  Returns (F12, ep2) in float32 as the caller
    computes them: F12 = K1^-T [t12]x R12 K2^-1 (ComputeF12, LocalMapping.cc:55-71, with the closed
    -form inverse of the upper-triangular K) and ep2 = CameraProjection(pose2).WorldToImage(Ow1)
    (ORBmatcher.cc:772-773, CameraProjection.h:49-55).  KF1's centre lies on KF2's principal plane,
    so 1/Z = inf and ep2 = (-inf, NaN), exactly as the reference's float arithmetic gives it."""
    f32 = np.float32
    fx, fy, cx, cy = f32(cam["fx"]), f32(cam["fy"]), f32(cam["cx"]), f32(cam["cy"])
    b = f32(cam["bf"]) / fx
    t12 = np.array([b, 0, 0], f32)          # -R1w R2w^T t2w + t1w with t2w = (-b, 0, 0)
    tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]], f32)
    Kinv = np.array([[f32(1) / fx, 0, -cx / fx], [0, f32(1) / fy, -cy / fy], [0, 0, 1]], f32)
    F12 = (Kinv.T @ tx @ Kinv).astype(f32)
    with np.errstate(divide="ignore", invalid="ignore"):
        Xc = np.array([-b, 0, 0], f32)      # Rcw * Ow1 + tcw with Ow1 = 0
        invz = f32(1) / Xc[2]
        ep2 = np.array([invz * fx * Xc[0] + cx, invz * fy * Xc[1] + cy], f32)
    return F12.reshape(9), ep2


def make_pose_batch(seed: int = 0, n_frames: int = 8, n_edges=600, stereo_frac: float = 0.4,
                    outlier_frac: float = 0.1, rot_deg: float = 0.5, trans_m: float = 0.1, cam=KITTI):
    """C5: a batch of PoseOptimization problems in the orbba_pose_batch layout.

    Per frame: a random camera pose (yaw U(-180,180) deg, position U(-50,50) m in x/z), map points
    back-projected from uniform pixels at depth U(3, 60) m, octaves U{0..7} with pixel noise
    N(0, 1.2^oct) and invSigma2 = 1/1.2^(2 oct) (float, like Frame::pyramid.invSigmaSq);
    `stereo_frac` of the observations carry ur = u - bf/z + noise; `outlier_frac` are moved by
    +-U(10, 60) px.  The initial pose (the motion-model prediction) is the true pose perturbed by
    N(0, rot_deg) rotation and N(0, trans_m) translation.  Measurements, map points and
    intrinsics are rounded to float32, as the reference stores them.  n_edges: int or per-frame list.
    """
    rng = np.random.default_rng(seed)
    counts = [int(n_edges)] * n_frames if np.isscalar(n_edges) else [int(n) for n in n_edges]
    assert len(counts) == n_frames
    eb = np.zeros(n_frames + 1, np.int32)
    eb[1:] = np.cumsum(counts)
    camv = np.array([cam[k] for k in ("fx", "fy", "cx", "cy", "bf")], np.float32).astype(np.float64)
    fx, fy, cx, cy, bf = camv
    pose_R, pose_t, gt_R, gt_t = [], [], [], []
    xw, obs, info = [], [], []
    for f, n in enumerate(counts):
        Rcw = _rot_y(rng.uniform(-180, 180)) @ _small_rot(rng, 3.0)
        C = np.array([rng.uniform(-50, 50), rng.uniform(-2, 2), rng.uniform(-50, 50)])
        tcw = -Rcw @ C
        gt_R.append(Rcw.reshape(-1))
        gt_t.append(tcw)
        u = rng.uniform(0, cam["width"], n)
        v = rng.uniform(0, cam["height"], n)
        z = rng.uniform(3, 60, n)
        Xc = np.stack([(u - cx) * z / fx, (v - cy) * z / fy, z], 1)
        Xw = (Xc - tcw) @ Rcw   # Rcw^T (Xc - t)
        octv = rng.integers(0, 8, n)
        sig = 1.2 ** octv
        uo = u + rng.normal(0, 1, n) * sig
        vo = v + rng.normal(0, 1, n) * sig
        st = rng.random(n) < stereo_frac
        ur = np.where(st, u - bf / z + rng.normal(0, 1, n) * sig, -1.0)
        out = rng.random(n) < outlier_frac
        du = rng.choice([-1, 1], n) * rng.uniform(10, 60, n)
        dv = rng.choice([-1, 1], n) * rng.uniform(10, 60, n)
        uo = np.where(out, uo + du, uo)
        vo = np.where(out, vo + dv, vo)
        ur = np.where(out & st, ur + du, ur)
        o = np.stack([uo, vo, ur], 1).astype(np.float32).astype(np.float64)
        o[~st, 2] = -1.0
        obs.append(o)
        xw.append(Xw.astype(np.float32).astype(np.float64))
        info.append((1.0 / (sig * sig)).astype(np.float32).astype(np.float64))
        R0 = _small_rot(rng, rot_deg) @ Rcw
        t0 = tcw + rng.normal(0, trans_m, 3)
        pose_R.append(R0.astype(np.float32).astype(np.float64).reshape(-1))
        pose_t.append(t0.astype(np.float32).astype(np.float64))
    cat = (lambda a, w: np.concatenate(a).reshape(-1, w) if sum(counts) else np.zeros((0, w)))
    return dict(edge_begin=eb, pose_R=np.array(pose_R).reshape(n_frames, 9), pose_t=np.array(pose_t).reshape(n_frames, 3),
                cam=np.tile(camv, (n_frames, 1)), xw=cat(xw, 3), obs=cat(obs, 3),
                inv_sigma2=np.concatenate(info) if sum(counts) else np.zeros(0),
                gt_R=np.array(gt_R).reshape(n_frames, 9), gt_t=np.array(gt_t).reshape(n_frames, 3))


ORB_QUOTA_2000 = (434, 362, 302, 251, 209, 175, 145, 122)


def make_proj_batch(seed: int = 0, n_frames: int = 4, n_kp=2000, n_mp=1500, width: float = 1241.0,
                    height: float = 376.0, th: float = 1.0, nnratio: float = 0.8, dup_frac: float = 0.15,
                    odd_bounds: bool = False):
    """C6: SearchByProjection(Frame, local map points) inputs in the orbm_proj_batch layout (§8f row 2).

    Per frame: n_kp keypoints uniform over the image with octaves drawn by the 2000-feature
    quotas, random descriptors, 40 % stereo (ur = x - U(5, 60)), 5 % already claimed.  Map points:
    70 % are re-observations of a keypoint (projection = keypoint + N(0, 1.5 * 1.2^oct) px,
    descriptor = the keypoint's with U{0..60} bits flipped, trackScaleLevel = octave or octave+1),
    `dup_frac` of those reuse an already used keypoint (claim conflicts) and some carry an exact copy
    of another candidate's descriptor (distance ties); the rest are random.  90 % trackInView,
    95 % with observations, viewCos U(0.5, 1) with a third above 0.998.  Bounds are (0, W, 0, H) or
    fractional undistortion-like bounds when `odd_bounds`.  n_kp / n_mp: int or per-frame list.
    """
    rng = np.random.default_rng(seed)
    kps = [int(n_kp)] * n_frames if np.isscalar(n_kp) else [int(v) for v in n_kp]
    mps = [int(n_mp)] * n_frames if np.isscalar(n_mp) else [int(v) for v in n_mp]
    q = np.array(ORB_QUOTA_2000, float)
    q /= q.sum()
    scale = (1.2 ** np.arange(8)).astype(np.float32)
    F = dict(kp_xy=[], kp_octave=[], kp_uright=[], kp_desc=[], kp_claimed=[], bounds=[], mp_valid=[], mp_proj=[],
             mp_view_cos=[], mp_level=[], mp_desc=[], mp_has_obs=[])
    for f in range(n_frames):
        n, m = kps[f], mps[f]
        if odd_bounds:
            b = np.array([rng.uniform(-8, 2), width + rng.uniform(-2, 8), rng.uniform(-6, 2), height + rng.uniform(-2, 6)])
        else:
            b = np.array([0.0, width, 0.0, height])
        x = rng.uniform(b[0] - 4, b[1] + 4, n)   # a few fall outside the grid (undistorted points)
        y = rng.uniform(b[2] - 4, b[3] + 4, n)
        octv = rng.choice(8, size=n, p=q)
        desc = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
        st = rng.random(n) < 0.4
        ur = np.where(st, x - rng.uniform(5, 60, n), -1.0)
        claimed = (rng.random(n) < 0.05).astype(np.uint8)
        F["kp_xy"].append(np.stack([x, y], 1).astype(np.float32))
        F["kp_octave"].append(octv.astype(np.int32))
        F["kp_uright"].append(ur.astype(np.float32))
        F["kp_desc"].append(desc)
        F["kp_claimed"].append(claimed)
        F["bounds"].append(b.astype(np.float32))
        proj = np.zeros((m, 3))
        lvl = np.zeros(m, np.int32)
        mdesc = rng.integers(0, 256, size=(m, 32), dtype=np.uint8)
        used = []
        for j in range(m):
            if n > 0 and rng.random() < 0.7:
                i = int(rng.choice(used)) if used and rng.random() < dup_frac else int(rng.integers(0, n))
                used.append(i)
                s = 1.5 * scale[octv[i]]
                u, v = x[i] + rng.normal(0, s), y[i] + rng.normal(0, s)
                d = desc[i].copy()
                if rng.random() < 0.1:
                    # an exact copy of a random keypoint's descriptor: ties with the true match
                    d = desc[int(rng.integers(0, n))].copy()
                flips = rng.choice(256, size=int(rng.integers(0, 61)), replace=False)
                for bit in flips:
                    d[bit >> 3] ^= np.uint8(1 << (bit & 7))
                mdesc[j] = d
                lvl[j] = min(int(octv[i]) + int(rng.integers(0, 2)), 7)
                uR = (u - (x[i] - ur[i]) + rng.normal(0, 1.0)) if st[i] else u - rng.uniform(5, 60)
                if rng.random() < 0.1:
                    uR += rng.uniform(-30, 30)
                proj[j] = (u, v, uR)
            else:
                proj[j] = (rng.uniform(b[0], b[1]), rng.uniform(b[2], b[3]), 0.0)
                proj[j, 2] = proj[j, 0] - rng.uniform(5, 60)
                lvl[j] = int(rng.integers(0, 8))
        F["mp_valid"].append((rng.random(m) < 0.9).astype(np.uint8))
        F["mp_proj"].append(proj.astype(np.float32))
        vc = rng.uniform(0.5, 1.0, m)
        vc = np.where(rng.random(m) < 0.33, rng.uniform(0.9975, 1.0, m), vc)
        F["mp_view_cos"].append(vc.astype(np.float32))
        F["mp_level"].append(lvl)
        F["mp_desc"].append(mdesc)
        F["mp_has_obs"].append((rng.random(m) < 0.95).astype(np.uint8))
    out = {}
    for k, v in F.items():
        out[k] = np.concatenate(v) if k != "bounds" else np.stack(v)
    out["kp_begin"] = np.concatenate([[0], np.cumsum(kps)]).astype(np.int32)
    out["mp_begin"] = np.concatenate([[0], np.cumsum(mps)]).astype(np.int32)
    out["scale_factors"] = scale
    out["th"] = float(th)
    out["nnratio"] = float(nnratio)
    return out


def tile_proj_batch(b: dict, reps: int) -> dict:
    """`reps` copies of a make_proj_batch batch back to back (a large batch without regenerating)."""
    out = dict(b)
    F = len(b["kp_begin"]) - 1
    for k in ("kp_xy", "kp_octave", "kp_uright", "kp_desc", "kp_claimed", "mp_valid", "mp_proj", "mp_view_cos",
              "mp_level", "mp_desc", "mp_has_obs"):
        if b.get(k) is not None:
            out[k] = np.concatenate([b[k]] * reps)
    out["bounds"] = np.concatenate([b["bounds"]] * reps)
    for k in ("kp_begin", "mp_begin"):
        per = np.diff(b[k])
        out[k] = np.concatenate([[0], np.cumsum(np.tile(per, reps))]).astype(np.int32)
    assert len(out["kp_begin"]) == F * reps + 1
    return out


def tile_ragged_batch(b: dict, reps: int) -> dict:
    """`reps` copies of a ragged batch back to back (a large batch without regenerating).  Every
    `*_begin` array (n + 1 prefix offsets) is re-prefixed; an array whose length equals the total of
    one prefix, or the number of batch entries, is repeated; other values (scalars, host tables such
    as scale_factors) are kept."""
    out = dict(b)
    begins = {k: v for k, v in b.items() if k.endswith("_begin")}
    n = len(next(iter(begins.values()))) - 1
    totals = {int(v[-1]) for v in begins.values()}
    for k, v in b.items():
        if k in begins:
            out[k] = np.concatenate([[0], np.cumsum(np.tile(np.diff(v), reps))]).astype(v.dtype)
        elif isinstance(v, np.ndarray) and v.ndim >= 1 and k != "scale_factors" and (len(v) in totals or len(v) == n):
            out[k] = np.concatenate([v] * reps)
    return out


def make_vocabulary(seed: int = 0, k: int = 10, L: int = 4, scoring: int = 0, weighting: int = 0,
                    early_leaf: float = 0.05, stop_frac: float = 0.03, order: str = "bfs"):
    """A synthetic DBoW2 ORB vocabulary (the real ORBvoc.txt is not available offline).

    A k-ary tree of depth L: children descriptors are the parent's with U{16..48} bits flipped (root
    children random), so descriptor distance follows the tree.  `early_leaf` of the internal nodes
    below level 2 stop early (leaves above level L, as k-means trees have), leaves get idf-like
    weights U(0.5, 8) and `stop_frac` of them weight 0 (stopped words); internal nodes weight 0.
    Nodes are numbered in `order` ("bfs" or "dfs"; the text format only needs parents first).
    Returns dict(k, L, scoring, weighting, parent, is_leaf, desc, weight) with node 0 = root."""
    rng = np.random.default_rng(seed)
    parent, is_leaf, desc, weight, depth = [0], [0], [np.zeros(32, np.uint8)], [0.0], [0]

    def new_node(p, d):
        i = len(parent)
        parent.append(p)
        depth.append(d)
        if p == 0:
            desc.append(rng.integers(0, 256, 32, dtype=np.uint8))
        else:
            x = desc[p].copy()
            for bit in rng.choice(256, size=int(rng.integers(16, 49)), replace=False):
                x[bit >> 3] ^= np.uint8(1 << (bit & 7))
            desc.append(x)
        leaf = d == L or (d >= 2 and rng.random() < early_leaf)
        is_leaf.append(1 if leaf else 0)
        weight.append(0.0 if not leaf else (0.0 if rng.random() < stop_frac else float(rng.uniform(0.5, 8.0))))
        return i

    if order == "bfs":
        frontier = [0]
        while frontier:
            nxt = []
            for p in frontier:
                if p != 0 and is_leaf[p]:
                    continue
                for _ in range(k):
                    nxt.append(new_node(p, depth[p] + 1))
            frontier = nxt
    else:
        def rec(p):
            for _ in range(k):
                c = new_node(p, depth[p] + 1)
                if not is_leaf[c]:
                    rec(c)
        rec(0)
    # text round trip precision: weights as the reference's ostream << double (6 significant digits)
    w = np.array([float(f"{x:g}") for x in weight])
    return dict(k=k, L=L, scoring=scoring, weighting=weighting, parent=np.array(parent, np.int32),
                is_leaf=np.array(is_leaf, np.uint8), desc=np.stack(desc).astype(np.uint8), weight=w)


def write_vocabulary_text(voc: dict, path) -> None:
    """saveToTextFile format (TemplatedVocabulary.h:1434-1450)."""
    lines = [f"{voc['k']} {voc['L']}  {voc['scoring']} {voc['weighting']}"]
    for i in range(1, len(voc["parent"])):
        d = " ".join(str(int(b)) for b in voc["desc"][i])
        lines.append(f"{voc['parent'][i]} {int(voc['is_leaf'][i])} {d}  {voc['weight'][i]:g}")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def vocabulary_features(voc: dict, seed: int, n: int, near: float = 0.8) -> np.ndarray:
    """n descriptors: `near` of them a random leaf's descriptor with U{0..40} flips, the rest random,
    some repeated (same word several times)."""
    rng = np.random.default_rng(seed)
    leaves = np.nonzero(voc["is_leaf"])[0]
    out = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    for i in range(n):
        if rng.random() < near and len(leaves):
            x = voc["desc"][int(rng.choice(leaves))].copy()
            for bit in rng.choice(256, size=int(rng.integers(0, 41)), replace=False):
                x[bit >> 3] ^= np.uint8(1 << (bit & 7))
            out[i] = x
        if i > 0 and rng.random() < 0.05:
            out[i] = out[int(rng.integers(0, i))]
    return out


def make_full_vocabulary(seed: int = 0, k: int = 10, L: int = 6):
    """A full k-ary depth-L tree built level by level (ORBvoc.txt's shape: k = 10, L = 6, ~1.1 M nodes),
    BFS-numbered, children = parent with ~32 bits flipped, leaf weights U(0.5, 8), TF-IDF / L1."""
    rng = np.random.default_rng(seed)
    parents = [np.zeros(1, np.int64)]
    descs = [np.zeros((1, 32), np.uint8)]
    start = 0
    for d in range(1, L + 1):
        prev = descs[-1]
        pids = np.repeat(np.arange(start, start + len(prev)), k)
        base = np.repeat(prev, k, axis=0)
        if d == 1:
            base = rng.integers(0, 256, size=base.shape, dtype=np.uint8)
        else:
            flips = np.packbits(rng.integers(0, 256, size=(len(base), 256), dtype=np.uint8) < 32, axis=1)
            base = base ^ flips
        start += len(prev)
        parents.append(pids)
        descs.append(base)
    parent = np.concatenate(parents).astype(np.int32)
    desc = np.concatenate(descs)
    n = len(parent)
    is_leaf = np.zeros(n, np.uint8)
    is_leaf[n - k ** L:] = 1
    weight = np.zeros(n)
    weight[n - k ** L:] = rng.uniform(0.5, 8.0, k ** L)
    return dict(k=k, L=L, scoring=0, weighting=0, parent=parent, is_leaf=is_leaf, desc=desc, weight=weight)


def make_init_batch(seed: int = 0, n_pairs: int = 4, n1=4000, n2=4000, width: float = 1280.0, height: float = 720.0,
                    window: int = 100, nnratio: float = 0.9, check_orientation: bool = True, dup_frac: float = 0.25,
                    twin_frac: float = 0.15, dense: bool = False):
    """SearchForInitialization inputs (orbm_init_batch, host arrays) shaped like
    Tracking::MonocularInitialization (Tracking.cc:1050-1052: the initial extractor's 2x features,
    windowSize 100, ORBmatcher(0.9f, true)).

    F1 (initial frame): n1 keypoints over the image, octaves by the 2000-feature quotas, random
    descriptors, angles around a dominant value.  F2 (current frame): for 70 % of F1's keypoints a
    displaced copy (a common image motion + noise, 0-40 flipped bits, the same octave 75 % of the
    time), the rest random; a fraction `dup_frac` of F2's copies duplicate an F1 keypoint that already
    has one (several queries competing for one idx2, so later, closer queries take it from earlier
    ones), some with an exact descriptor copy (distance ties); `twin_frac` of F1's keypoints sit next
    to an earlier one with a similar descriptor (the later query takes the feature when it is closer).
    prevMatched = F1's positions.
    `dense`: a cluster of 300 octave-0 keypoints in a 150-px box puts more than PI_CAP candidates in
    the windows around it.  n1 / n2: int or per-pair list."""
    rng = np.random.default_rng(seed)
    n1s = [int(n1)] * n_pairs if np.isscalar(n1) else [int(v) for v in n1]
    n2s = [int(n2)] * n_pairs if np.isscalar(n2) else [int(v) for v in n2]
    q = np.array(ORB_QUOTA_2000, float)
    q /= q.sum()
    F = dict(kp_xy=[], kp_octave=[], kp_desc=[], kp_angle=[], bounds=[], q_octave=[], q_desc=[], q_angle=[],
             prev_matched=[])

    def flip(d, nbits):
        d = d.copy()
        for bit in rng.choice(256, size=nbits, replace=False):
            d[bit >> 3] ^= np.uint8(1 << (bit & 7))
        return d

    for p in range(n_pairs):
        a, b = n1s[p], n2s[p]
        x1 = rng.uniform(0, width, a)
        y1 = rng.uniform(0, height, a)
        o1 = rng.choice(8, size=a, p=q)
        if dense and a > 300:
            cx, cy = rng.uniform(200, width - 200), rng.uniform(200, height - 200)
            x1[:300] = cx + rng.uniform(-75, 75, 300)
            y1[:300] = cy + rng.uniform(-75, 75, 300)
            o1[:300] = 0
        d1 = rng.integers(0, 256, size=(a, 32), dtype=np.uint8)
        for i in range(1, a):   # twins: a later query near an earlier one with a similar descriptor
            if rng.random() < twin_frac:
                j = int(rng.integers(0, i))
                x1[i], y1[i], o1[i] = x1[j] + rng.normal(0, 2), y1[j] + rng.normal(0, 2), o1[j]
                d1[i] = flip(d1[j], int(rng.integers(0, 31)))
        rot = rng.uniform(0, 360)
        a1 = (rot + rng.normal(0, 20, a)) % 360
        mot = rng.normal(0, 15, 2)
        x2 = rng.uniform(0, width, b)
        y2 = rng.uniform(0, height, b)
        o2 = rng.choice(8, size=b, p=q)
        d2 = rng.integers(0, 256, size=(b, 32), dtype=np.uint8)
        a2 = rng.uniform(0, 360, b)
        used = []
        for k in range(b):
            if a == 0 or rng.random() >= 0.7:
                continue
            i = int(rng.choice(used)) if used and rng.random() < dup_frac else int(rng.integers(0, a))
            used.append(i)
            x2[k] = x1[i] + mot[0] + rng.normal(0, 3)
            y2[k] = y1[i] + mot[1] + rng.normal(0, 3)
            o2[k] = o1[i] if rng.random() < 0.75 else int(rng.integers(0, 8))
            d2[k] = flip(d1[i], int(rng.integers(0, 41)))
            if rng.random() < 0.08:
                d2[k] = d1[i].copy() if rng.random() < 0.5 else d2[int(rng.integers(0, b))].copy()
            a2[k] = (a1[i] + 25 + rng.normal(0, 8)) % 360
        F["kp_xy"].append(np.stack([x2, y2], 1).astype(np.float32))
        F["kp_octave"].append(o2.astype(np.int32))
        F["kp_desc"].append(d2)
        F["kp_angle"].append(np.clip(a2, 0, np.nextafter(np.float32(360), np.float32(0))).astype(np.float32))
        F["bounds"].append(np.array([0.0, width, 0.0, height], np.float32))
        F["q_octave"].append(o1.astype(np.int32))
        F["q_desc"].append(d1)
        F["q_angle"].append(np.clip(a1, 0, np.nextafter(np.float32(360), np.float32(0))).astype(np.float32))
        F["prev_matched"].append(np.stack([x1, y1], 1).astype(np.float32))
    shapes = dict(kp_xy=((0, 2), np.float32), kp_octave=((0,), np.int32), kp_desc=((0, 32), np.uint8),
                  kp_angle=((0,), np.float32), bounds=((0, 4), np.float32), q_octave=((0,), np.int32),
                  q_desc=((0, 32), np.uint8), q_angle=((0,), np.float32), prev_matched=((0, 2), np.float32))
    out = {}
    for k, (shape, dt) in shapes.items():
        v = F[k] if k != "bounds" else [x[None] for x in F[k]]
        out[k] = np.ascontiguousarray(np.concatenate(v).astype(dt) if v else np.zeros(shape, dt))
    out["kp_begin"] = np.concatenate([[0], np.cumsum(n2s)]).astype(np.int32)
    out["q_begin"] = np.concatenate([[0], np.cumsum(n1s)]).astype(np.int32)
    out.update(window=int(window), nnratio=float(nnratio), check_orientation=bool(check_orientation))
    return out


def make_reloc_batch(seed: int = 0, n_frames: int = 4, n_kp=2000, n_mp=600, th: float = 10.0, orb_dist: int = 100,
                     check_orientation: bool = True, dup_frac: float = 0.15, claimed_frac: float = 0.1):
    """SearchByProjection(Frame&, KeyFrame*, alreadyFound, th, ORBdist) inputs (orbm_reloc_batch, host arrays)
    shaped like Tracking::Relocalization (Tracking.cc:403,417: th 10 / ORBdist 100, then 3 / 64) on a
    KITTI camera.  Per frame: a pose (small rotation, a few metres of translation); the candidate
    keyframe's points in front of it (90 % valid), maxDistance_ = dist * 1.2^o * U(0.9, 1.1) for a random
    octave o and minDistance_ = maxDistance_ / 1.2^7 (MapPoint.cc:369-377), 5 % outside the invariance
    range; 70 % of the points observed by a keypoint near the projection (octave = the predicted scale
    +- 1 or off-window, 0-60 flipped bits), `dup_frac` of them sharing a keypoint with another point,
    plus random keypoints; `claimed_frac` of the keypoints already hold a map point.  Angles around a
    dominant rotation for CheckOrientation.  n_kp / n_mp: int or per-frame list."""
    rng = np.random.default_rng(seed)
    kps = [int(n_kp)] * n_frames if np.isscalar(n_kp) else [int(v) for v in n_kp]
    mps = [int(n_mp)] * n_frames if np.isscalar(n_mp) else [int(v) for v in n_mp]
    fx, fy, cx, cy = np.float32(KITTI["fx"]), np.float32(KITTI["fx"]), np.float32(607.1928), np.float32(185.2157)
    W, H = 1241.0, 376.0
    cum = np.ones(8, np.float32)
    for i in range(1, 8):
        cum[i] = np.float32(cum[i - 1] * np.float32(1.2))
    F = dict(kp_xy=[], kp_octave=[], kp_desc=[], kp_angle=[], kp_claimed=[], bounds=[], pose=[], camera=[],
             mp_valid=[], mp_xw=[], mp_max_min=[], mp_desc=[], mp_angle=[])
    for f in range(n_frames):
        n, m = kps[f], mps[f]
        Rcw = _small_rot(rng, 3.0).astype(np.float32)
        tcw = rng.normal(0, 2.0, 3).astype(np.float32)
        # points in the camera frame, then to the world: Xw = Rcw^T (Xc - tcw)
        z = rng.uniform(4, 40, m)
        u = rng.uniform(-20, W + 20, m)
        v = rng.uniform(-10, H + 10, m)
        Xc = np.stack([(u - cx) * z / fx, (v - cy) * z / fy, z], 1)
        Xw = ((Xc - tcw[None]) @ Rcw).astype(np.float32)
        Ow = -(Rcw.T @ tcw)
        dist = np.linalg.norm(Xw - Ow[None], axis=1)
        o = rng.integers(0, 8, m)
        maxd = dist * (1.2 ** o) * rng.uniform(0.9, 1.1, m)
        bad = rng.random(m) < 0.05
        maxd = np.where(bad, dist * rng.choice([0.5, 3.0], m), maxd)
        mind = maxd / cum[7]
        mdesc = rng.integers(0, 256, size=(m, 32), dtype=np.uint8)
        rot = rng.uniform(0, 360)
        mang = rng.uniform(0, 360, m)
        x = rng.uniform(0, W, n)
        y = rng.uniform(0, H, n)
        octv = rng.integers(0, 8, n)
        desc = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
        ang = rng.uniform(0, 360, n)
        used = []
        for j in range(m):
            if n == 0 or rng.random() >= 0.7:
                continue
            i = int(rng.choice(used)) if used and rng.random() < dup_frac else int(rng.integers(0, n))
            used.append(i)
            x[i] = u[j] + rng.normal(0, 1.5)
            y[i] = v[j] + rng.normal(0, 1.5)
            ratio = maxd[j] / max(dist[j], 1e-6)
            ps = int(min(7, max(0, np.ceil(np.log(ratio) / np.log(1.2)))))
            octv[i] = min(7, max(0, ps + int(rng.choice([-1, 0, 0, 1, 3]))))
            d = mdesc[j].copy()
            for bit in rng.choice(256, size=int(rng.integers(0, 61)), replace=False):
                d[bit >> 3] ^= np.uint8(1 << (bit & 7))
            desc[i] = d
            ang[i] = (mang[j] - rot + rng.normal(0, 6)) % 360
        F["kp_xy"].append(np.stack([x, y], 1).astype(np.float32))
        F["kp_octave"].append(octv.astype(np.int32))
        F["kp_desc"].append(desc)
        F["kp_angle"].append(np.minimum(ang, 359.99).astype(np.float32))
        F["kp_claimed"].append((rng.random(n) < claimed_frac).astype(np.uint8))
        F["bounds"].append(np.array([[0.0, W, 0.0, H]], np.float32))
        F["pose"].append(np.concatenate([Rcw.reshape(-1), tcw])[None].astype(np.float32))
        F["camera"].append(np.array([[fx, fy, cx, cy]], np.float32))
        F["mp_valid"].append((rng.random(m) < 0.9).astype(np.uint8))
        F["mp_xw"].append(Xw)
        F["mp_max_min"].append(np.stack([maxd, mind], 1).astype(np.float32))
        F["mp_desc"].append(mdesc)
        F["mp_angle"].append(np.minimum(mang, 359.99).astype(np.float32))
    shapes = dict(kp_xy=(0, 2), kp_octave=(0,), kp_desc=(0, 32), kp_angle=(0,), kp_claimed=(0,), bounds=(0, 4),
                  pose=(0, 12), camera=(0, 4), mp_valid=(0,), mp_xw=(0, 3), mp_max_min=(0, 2), mp_desc=(0, 32),
                  mp_angle=(0,))
    out = {}
    for k, shape in shapes.items():
        dt = np.uint8 if k in ("kp_desc", "mp_desc", "kp_claimed", "mp_valid") else (np.int32 if k == "kp_octave" else np.float32)
        out[k] = np.ascontiguousarray(np.concatenate(F[k]).astype(dt) if F[k] else np.zeros(shape, dt))
    out["kp_begin"] = np.concatenate([[0], np.cumsum(kps)]).astype(np.int32)
    out["mp_begin"] = np.concatenate([[0], np.cumsum(mps)]).astype(np.int32)
    out.update(scale_factors=cum, log_scale_factor=float(np.float32(np.log(np.float64(np.float32(1.2))))), th=float(th),
               orb_dist=int(orb_dist), check_orientation=bool(check_orientation))
    return out
