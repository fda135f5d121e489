"""Synthetic SearchForTriangulation inputs (C3 shape): two keyframes of a stereo-like
rig with a multi-node FeatureVector, used by both the CPU oracle test and the GPU parity test."""
import numpy as np


def make_case(seed, n1=600, n2=650, n_nodes=7, only_single_node=False):
    rng = np.random.default_rng(seed)
    fx = 718.856
    bf = 386.1448
    K = np.array([[fx, 0, 607.19], [0, fx, 185.21], [0, 0, 1.0]], np.float32)
    # KF1 at origin, KF2 translated by baseline along x: F12 = K1^-T [t12]x R12 K2^-1
    t12 = np.array([bf / fx, 0.02, 0.01], np.float32)
    tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]], np.float32)
    F12 = (np.linalg.inv(K).T @ tx @ np.linalg.inv(K)).astype(np.float32)
    ep2 = np.array([607.19 + fx * (-t12[0]) / 1e-3, 185.21], np.float32)   # far away epipole
    pts = rng.uniform([0, 0], [1241, 376], size=(n1, 2)).astype(np.float32)
    xy2 = np.concatenate([pts[: min(n1, n2)] + rng.normal(0, 1.5, (min(n1, n2), 2)),
                          rng.uniform([0, 0], [1241, 376], size=(max(0, n2 - n1), 2))]).astype(np.float32)[:n2]
    base = rng.integers(0, 256, (n1, 32), dtype=np.uint8)
    d1 = base.copy()
    d2 = np.concatenate([base[: min(n1, n2)], rng.integers(0, 256, (max(0, n2 - n1), 32), dtype=np.uint8)])[:n2].copy()
    flips = rng.integers(0, 256, d2.shape, dtype=np.uint8) & rng.integers(0, 256, d2.shape, dtype=np.uint8) & \
        rng.integers(0, 256, d2.shape, dtype=np.uint8)
    d2 ^= flips
    d2[5] = d2[4]   # exact duplicate -> equal distances, "last index wins"
    o1 = rng.integers(0, 8, n1).astype(np.int32)
    o2 = rng.integers(0, 8, n2).astype(np.int32)
    ur1 = np.where(rng.random(n1) < 0.3, rng.uniform(0, 1241, n1), -1).astype(np.float32)
    ur2 = np.where(rng.random(n2) < 0.3, rng.uniform(0, 1241, n2), -1).astype(np.float32)
    mp1 = (rng.random(n1) < 0.1).astype(np.uint8)
    mp2 = (rng.random(n2) < 0.1).astype(np.uint8)

    # vocabulary nodes: corresponding features share a node id; each frame also has a node the
    # other lacks (exercises the FeatureVectorIterator skip)
    assign1 = rng.integers(0, n_nodes, n1)
    assign2 = np.concatenate([assign1[: min(n1, n2)], rng.integers(0, n_nodes + 1, max(0, n2 - n1))])[:n2]
    assign1 = np.where(rng.random(n1) < 0.05, n_nodes + 1, assign1)   # node only kf1 has

    def fv(n, assign):
        if only_single_node:
            return np.array([0], np.uint32), np.array([0, n], np.int32), np.arange(n, dtype=np.int32)
        present = np.unique(assign)
        ids = (present * 3 + 1).astype(np.uint32)
        order = np.argsort(assign, kind="stable")
        counts = np.array([(assign == p).sum() for p in present])
        off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
        return ids, off, order.astype(np.int32)

    fv1 = fv(n1, assign1)
    fv2 = fv(n2, assign2)
    s = np.float32(1.0)
    scale, sigma2 = [], []
    for _ in range(8):
        scale.append(s)
        sigma2.append(s * s)
        s = np.float32(s * np.float32(1.2))
    kf1 = dict(xy=pts, octave=o1, uright=ur1, has_mappoint=mp1, desc=d1, fv=fv1)
    kf2 = dict(xy=xy2, octave=o2, uright=ur2, has_mappoint=mp2, desc=d2, fv=fv2,
               scale_factors=np.array(scale, np.float32), sigma2=np.array(sigma2, np.float32), ep2=ep2)
    return kf1, kf2, F12


def oracle_run(O, kf1, kf2, F12, only_stereo=False):
    keep = O._Keep()
    f1 = O.tri_frame(keep, kf1["xy"], kf1["octave"], kf1["uright"], kf1["has_mappoint"], kf1["desc"], *kf1["fv"])
    f2 = O.tri_frame(keep, kf2["xy"], kf2["octave"], kf2["uright"], kf2["has_mappoint"], kf2["desc"], *kf2["fv"])
    return O.search_for_triangulation(f1, f2, F12, kf2["ep2"], kf2["scale_factors"], kf2["sigma2"], only_stereo)
