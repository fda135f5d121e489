"""The oracle's SearchByBoW restatements (oracle/orb_oracle.cpp) against a pure-Python restatement of
src/ORBmatcher.cc:452-516 (KeyFrame, Frame) and :696-766 (KeyFrame, KeyFrame), including
FeatureVectorIterator (:406-450) and CheckOrientation (:249-309).
Small random cases with clustered descriptors so that claims, ratio rejections and the rotation
filter all occur.  The bin order is libstdc++'s std::sort permutation of the sizes
(oracle_std_sort_sizes, itself checked against std::sort in tests/test_qt_sort.py)."""
import numpy as np
import pytest

TH_LOW, HISTO = 50, 30


def _hamming(a, b):
    return int(np.unpackbits(a ^ b).sum())


def _fv_join(n1, n2):
    a = b = 0
    while a < len(n1[0]) and b < len(n2[0]):
        if n1[0][a] == n2[0][b]:
            yield n1[1][n1[2][a]:n1[2][a + 1]], n2[1][n2[2][b]:n2[2][b + 1]]
            a += 1
            b += 1
        elif n1[0][a] < n2[0][b]:
            a += 1
        else:
            b += 1


def _check_orientation(O, pairs, ang_first, ang_second):
    hist = [[] for _ in range(HISTO)]
    for p in pairs:
        diff = np.float32(ang_first[p[0]]) - np.float32(ang_second[p[1]])
        if diff < 0:
            diff += np.float32(360)
        b = int(np.rint(np.float32(1.0 / HISTO) * diff))
        hist[0 if b == HISTO else b].append(p)
    order = [int(i) for i in O.std_sort_perm([len(h) for h in hist])]
    sizes = [len(hist[i]) for i in order]
    erase = 3 if sizes[2] >= 0.1 * sizes[0] else 2
    if sizes[1] < 0.1 * sizes[0]:
        erase = 1
    gone = [p for i in order[erase:] for p in hist[i]]
    return gone, len(pairs) - len(gone)


def _py_bow(O, D1, fv1, mp1, D2, fv2, ang1, ang2, ratio, check_ori, kf_form, mp2=None):
    n1, n2 = len(D1), len(D2)
    out = np.full(n1 if kf_form else n2, -1, np.int32)
    taken = np.zeros(n2, bool)
    pairs, nm = [], 0
    for ids1, ids2 in _fv_join(fv1, fv2):
        for i1 in ids1:
            if not mp1[i1]:
                continue
            best, bi, second = 256, -1, 256
            for i2 in ids2:
                if taken[i2] or (kf_form and not mp2[i2]):
                    continue
                d = _hamming(D1[i1], D2[i2])
                if d < best:
                    second, best, bi = best, d, i2
                elif d < second:
                    second = d
            ok = best < TH_LOW if kf_form else best <= TH_LOW
            if ok and np.float32(best) < np.float32(ratio) * np.float32(second):
                taken[bi] = True
                if kf_form:
                    out[i1] = bi
                    pairs.append((bi, i1))
                else:
                    out[bi] = i1
                    pairs.append((i1, bi))
                nm += 1
    if check_ori:
        if kf_form:
            gone, nm = _check_orientation(O, pairs, ang2, ang1)
            for _, i1 in gone:
                out[i1] = -1
        else:
            gone, nm = _check_orientation(O, pairs, ang1, ang2)
            for _, i2 in gone:
                out[i2] = -1
    return out, nm


def _case(seed, n1=120, n2=130, nodes=6):
    rng = np.random.default_rng(seed)
    centers = rng.integers(0, 256, (12, 32), dtype=np.uint8)

    def descs(n):
        c = centers[rng.integers(0, 12, n)]
        flip = np.packbits(rng.random((n, 256)) < 0.08, axis=1)
        return c ^ flip

    def fv(n):
        node = np.sort(rng.choice(np.arange(3, 40), nodes, replace=False)).astype(np.uint32)
        assign = rng.integers(0, nodes, n)
        off = np.zeros(nodes + 1, np.int32)
        idx = []
        for k in range(nodes):
            members = np.nonzero(assign == k)[0]
            idx.extend(members.tolist())
            off[k + 1] = len(idx)
        return node, np.array(idx, np.int32), off

    ang1 = (rng.normal(30, 6, n1) % 360).astype(np.float32)
    ang2 = (rng.normal(10, 6, n2) % 360).astype(np.float32)
    ang2[: n2 // 5] = rng.uniform(0, 360, n2 // 5)
    return descs(n1), fv(n1), descs(n2), fv(n2), ang1, ang2, rng


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("check_ori", [False, True])
def test_oracle_search_by_bow_frame(oracle, seed, check_ori):
    D1, fv1, D2, fv2, a1, a2, rng = _case(seed)
    mp1 = (rng.random(len(D1)) < 0.8).astype(np.uint8)
    exp, n = _py_bow(oracle, D1, fv1, mp1, D2, fv2, a1, a2, 0.9, check_ori, False)
    keep = oracle._Keep()
    z = lambda k: np.zeros(k, np.float32)   # noqa: E731
    kf = oracle.tri_frame(keep, np.zeros((len(D1), 2), np.float32), np.zeros(len(D1), np.int32), z(len(D1)), mp1, D1,
                          fv1[0], fv1[2], fv1[1])
    fr = oracle.tri_frame(keep, np.zeros((len(D2), 2), np.float32), np.zeros(len(D2), np.int32), z(len(D2)),
                          np.zeros(len(D2), np.uint8), D2, fv2[0], fv2[2], fv2[1])
    got, gn = oracle.search_by_bow(kf, fr, a1, a2, 0.9, check_ori)
    assert np.array_equal(got, exp) and gn == n
    assert n > 0


@pytest.mark.parametrize("seed", [4, 5])
@pytest.mark.parametrize("check_ori", [False, True])
def test_oracle_search_by_bow_keyframes(oracle, seed, check_ori):
    D1, fv1, D2, fv2, a1, a2, rng = _case(seed)
    mp1 = (rng.random(len(D1)) < 0.8).astype(np.uint8)
    mp2 = (rng.random(len(D2)) < 0.8).astype(np.uint8)
    exp, n = _py_bow(oracle, D1, fv1, mp1, D2, fv2, a1, a2, 0.9, check_ori, True, mp2)
    keep = oracle._Keep()
    z = lambda k: np.zeros(k, np.float32)   # noqa: E731
    k1 = oracle.tri_frame(keep, np.zeros((len(D1), 2), np.float32), np.zeros(len(D1), np.int32), z(len(D1)), mp1, D1,
                          fv1[0], fv1[2], fv1[1])
    k2 = oracle.tri_frame(keep, np.zeros((len(D2), 2), np.float32), np.zeros(len(D2), np.int32), z(len(D2)), mp2, D2,
                          fv2[0], fv2[2], fv2[1])
    got, gn = oracle.search_by_bow_kf(k1, k2, a1, a2, 0.9, check_ori)
    assert np.array_equal(got, exp) and gn == n
    assert n > 0
