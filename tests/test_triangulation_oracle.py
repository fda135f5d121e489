"""Oracle SearchForTriangulation vs a direct numpy restatement (ORBmatcher.cc:768-866). CPU only."""
import numpy as np
import pytest

from tri_case import make_case, oracle_run


def np_search(kf1, kf2, F, only_stereo):
    out = np.full(len(kf1["xy"]), -1, np.int32)
    ids1, off1, idx1 = kf1["fv"]
    ids2, off2, idx2 = kf2["fv"]
    common = sorted(set(ids1.tolist()) & set(ids2.tolist()))
    for nid in common:
        a = int(np.nonzero(ids1 == nid)[0][0])
        b = int(np.nonzero(ids2 == nid)[0][0])
        for i1 in idx1[off1[a]:off1[a + 1]]:
            if kf1["has_mappoint"][i1]:
                continue
            st1 = kf1["uright"][i1] >= 0
            if only_stereo and not st1:
                continue
            x1, y1 = kf1["xy"][i1]
            la = np.float32(x1 * F[0, 0] + y1 * F[1, 0] + F[2, 0])
            lb = np.float32(x1 * F[0, 1] + y1 * F[1, 1] + F[2, 1])
            lc = np.float32(x1 * F[0, 2] + y1 * F[1, 2] + F[2, 2])
            best, bi = 50, -1
            for i2 in idx2[off2[b]:off2[b + 1]]:
                if kf2["has_mappoint"][i2]:
                    continue
                st2 = kf2["uright"][i2] >= 0
                if only_stereo and not st2:
                    continue
                d = int(np.unpackbits(np.bitwise_xor(kf1["desc"][i1], kf2["desc"][i2])).sum())
                if d > 50 or d > best:
                    continue
                x2, y2 = kf2["xy"][i2]
                o2 = kf2["octave"][i2]
                if not st1 and not st2:
                    dx, dy = np.float32(kf2["ep2"][0] - x2), np.float32(kf2["ep2"][1] - y2)
                    if np.float32(dx * dx + dy * dy) < np.float32(100 * kf2["scale_factors"][o2]):
                        continue
                num = np.float32(la * x2 + lb * y2 + lc)
                den = np.float32(la * la + lb * lb)
                if den == 0:
                    continue
                if float(np.float32(num * num / den)) < 3.84 * float(kf2["sigma2"][o2]):
                    bi, best = int(i2), d
            out[i1] = bi
    return out


@pytest.mark.parametrize("seed,stereo", [(0, False), (1, True), (2, False)])
def test_oracle_triangulation_vs_numpy(oracle, seed, stereo):
    kf1, kf2, F = make_case(seed, n1=150, n2=170, n_nodes=4)
    got, n = oracle_run(oracle, kf1, kf2, F, stereo)
    exp = np_search(kf1, kf2, F, stereo)
    assert np.array_equal(got, exp)
    assert n == int((exp >= 0).sum())
    assert n > 0
