"""The oracle's relocalisation SearchByProjection (oracle/orb_oracle.cpp) against a pure-Python
restatement of src/ORBmatcher.cc:1364-1445 on the oracle's GetFeaturesInArea (Frame.cc:102-145,
pinned by tests/test_projection_oracle.py): the float projection (CameraProjection.h:44-60), the
image-bounds test, the distance-invariance gate, PredictScale (MapPoint.cc:405-415, libm log), the
level window predictedScale +- 1, the skip of every keypoint holding a map point (claims of the call
included), bestDist <= ORBdist and CheckOrientation (libstdc++ bin order via oracle_std_sort_sizes)."""
import math

import numpy as np
import pytest

from orb_slam2_refactored_amd.synth import make_reloc_batch

f32 = np.float32


def _py_reloc(O, b):
    F = len(b["kp_begin"]) - 1
    out = np.full(int(b["kp_begin"][-1]), -1, np.int32)
    ns = np.zeros(F, np.int32)
    nl = len(b["scale_factors"])
    stats = dict(accepted=0, projected=0)
    for f in range(F):
        k0, k1 = int(b["kp_begin"][f]), int(b["kp_begin"][f + 1])
        m0, m1 = int(b["mp_begin"][f]), int(b["mp_begin"][f + 1])
        xy, oc = b["kp_xy"][k0:k1], b["kp_octave"][k0:k1]
        holds = b["kp_claimed"][k0:k1].astype(bool).copy()
        owner = np.full(k1 - k0, -1)
        P = b["pose"][f]
        R, t = P[:9].reshape(3, 3), P[9:]
        fx, fy, cx, cy = b["camera"][f]
        bd = b["bounds"][f]
        Ow = []
        for i in range(3):
            s = f32(0)
            for k in range(3):
                s = f32(s + f32(-R[k, i]) * t[k])
            Ow.append(s)
        pairs = []
        for i1 in range(m1 - m0):
            j = m0 + i1
            if not b["mp_valid"][j]:
                continue
            X = b["mp_xw"][j]
            Xc = []
            for i in range(3):
                s = f32(0)
                for k in range(3):
                    s = f32(s + R[i, k] * X[k])
                Xc.append(f32(s + t[i]))
            invZ = f32(f32(1) / Xc[2])
            u = f32(f32(invZ * fx) * Xc[0]) + cx
            v = f32(f32(invZ * fy) * Xc[1]) + cy
            if not (u >= bd[0] and u < bd[1] and v >= bd[2] and v < bd[3]):
                continue
            sq = 0.0
            for i in range(3):
                d = float(f32(X[i] - Ow[i]))
                sq += d * d
            dist3D = f32(math.sqrt(sq))
            maxd, mind = b["mp_max_min"][j]
            if dist3D < f32(f32(0.8) * mind) or dist3D > f32(f32(1.2) * maxd):
                continue
            stats["projected"] += 1
            ratio = f32(maxd / dist3D)
            ps = max(0, min(int(math.ceil(math.log(float(ratio)) / float(f32(b["log_scale_factor"])))), nl - 1))
            r = f32(f32(b["th"]) * b["scale_factors"][ps])
            idx = O.features_in_area(xy, oc, bd, nl, u, v, r, ps - 1, ps + 1)
            best, bi = 256, -1
            for i2 in idx:
                if holds[i2]:
                    continue
                d = int(np.unpackbits(b["mp_desc"][j] ^ b["kp_desc"][k0 + i2]).sum())
                if d < best:
                    best, bi = d, int(i2)
            if best <= b["orb_dist"]:
                holds[bi] = True
                owner[bi] = i1
                pairs.append((i1, bi))
        n = len(pairs)
        stats["accepted"] += n
        if b["check_orientation"]:
            hist = [[] for _ in range(30)]
            for i1, i2 in pairs:
                diff = f32(b["mp_angle"][m0 + i1]) - f32(b["kp_angle"][k0 + i2])
                if diff < 0:
                    diff += f32(360)
                bn = int(np.rint(f32(1.0 / 30) * diff))
                hist[0 if bn == 30 else bn].append(i2)
            order = [int(i) for i in O.std_sort_perm([len(h) for h in hist])]
            sizes = [len(hist[i]) for i in order]
            erase = 1 if sizes[1] < 0.1 * sizes[0] else (2 if sizes[2] < 0.1 * sizes[0] else 3)
            gone = [i2 for i in order[erase:] for i2 in hist[i]]
            for i2 in gone:
                owner[i2] = -1
            n -= len(gone)
        out[k0:k1] = owner
        ns[f] = n
    return out, ns, stats


@pytest.mark.parametrize("seed,th,orb,check_ori", [(1, 10.0, 100, True), (2, 3.0, 64, True), (3, 10.0, 100, False)])
def test_oracle_reloc_projection(oracle, seed, th, orb, check_ori):
    b = make_reloc_batch(seed, n_frames=3, n_kp=[600, 300, 0], n_mp=[250, 200, 40], th=th, orb_dist=orb,
                         check_orientation=check_ori)
    exp, en, st = _py_reloc(oracle, b)
    got, gn = oracle.search_by_projection_reloc(b)
    assert np.array_equal(got, exp)
    assert np.array_equal(gn, en)
    assert st["projected"] > 100 and en[0] > 20
