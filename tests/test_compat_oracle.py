"""The oracle's OpenCV-build switches on CPU (oracle_set_compat).

* resize tail: where the vertical SIMD loop of cv::resize INTER_LINEAR 8U stops, per build width V
  ([ext] VResizeLinearVec_32s8u: `x <= w - V` by V, then `x < w - V/2` by V/2), and that the scalar
  tail rounds as FixedPtCast<int, uchar, 22> -- checked against a numpy restatement of both loops.
* trig: ::cos(double) vs cosf change no sample offset outside 96 of the 1.14e9 float angles
  (tools/probe/trig_angle_sensitivity.cpp); on the golden frames the descriptors are identical.
"""
import numpy as np
import pytest

from orb_slam2_refactored_amd.synth import synth_image


def np_tail_x(w, V):
    if V == 0:
        return w
    if V == 1:
        return 0
    x = 0
    while x <= w - V:
        x += V
    while x < w - V // 2:
        x += V // 2
    return x


@pytest.mark.parametrize("V", [0, 1, 8, 16, 32, 64])
def test_resize_tail_start(oracle, V):
    for w in list(range(1, 200)) + [357, 429, 514, 617, 741, 889, 1067, 1280]:
        assert oracle.resize_tail_x(w, V) == np_tail_x(w, V), (w, V)
    # C2 level 1 (1067 px): 66 vector iterations of 16, no half step (1056 < 1059 -> 1064), 3 scalar columns
    assert oracle.resize_tail_x(1067, 16) == 1064


def np_resize(src, dw, dh, V):
    """numpy restatement of cv::resize INTER_LINEAR 8U (generic path; vertical SIMD / scalar split)."""
    sh, sw = src.shape
    sx_scale, sy_scale = sw / dw, sh / dh
    out = np.zeros((dh, dw), np.uint8)

    def coefs(n, scale, size):
        pos, a0, a1 = [], [], []
        lim = n
        for d in range(n):
            f = np.float32((d + 0.5) * scale - 0.5)
            s = int(np.floor(f))
            f = np.float32(f - np.float32(s))
            if s < 0:
                f, s = np.float32(0), 0
            if s + 1 >= size:
                lim = min(lim, d)
                if s >= size - 1:
                    f, s = np.float32(0), size - 1
            pos.append(s)
            a0.append(int(np.rint(np.float32((np.float32(1) - f) * np.float32(2048)))))
            a1.append(int(np.rint(np.float32(f * np.float32(2048)))))
        return pos, a0, a1, lim

    xo, xa0, xa1, xmax = coefs(dw, sx_scale, sw)
    xt = np_tail_x(dw, V)

    def hrow(y):
        S = src[y].astype(np.int64)
        D = np.zeros(dw, np.int64)
        for x in range(dw):
            D[x] = S[xo[x]] * xa0[x] + S[xo[x] + 1] * xa1[x] if x < xmax else S[xo[x]] * 2048
        return D

    for dy in range(dh):
        fy = np.float32((dy + 0.5) * sy_scale - 0.5)
        sy = int(np.floor(fy))
        fy = np.float32(fy - np.float32(sy))
        b0 = int(np.rint(np.float32((np.float32(1) - fy) * np.float32(2048))))
        b1 = int(np.rint(np.float32(fy * np.float32(2048))))
        r0, r1 = hrow(min(max(sy, 0), sh - 1)), hrow(min(max(sy + 1, 0), sh - 1))
        simd = (((np.minimum(r0 >> 4, 32767) * b0) >> 16) + ((np.minimum(r1 >> 4, 32767) * b1) >> 16) + 2) >> 2
        scal = (r0 * b0 + r1 * b1 + (1 << 21)) >> 22
        v = np.where(np.arange(dw) < xt, simd, scal)
        out[dy] = np.clip(v, 0, 255)
    return out


@pytest.mark.parametrize("V", [0, 1, 16, 32])
def test_pyramid_level1_matches_numpy(oracle, V):
    img = synth_image(3, 200, 120)
    with oracle.compat("double", V):
        lv = oracle.pyramid(oracle.params(1000), img)
    h, w = lv[1].shape
    assert np.array_equal(lv[1], np_resize(img, w, h, V))


def test_tail_changes_only_tail_columns(oracle):
    img = synth_image(4, 1280, 720)
    with oracle.compat("double", 0):
        a = oracle.pyramid(oracle.params(2000), img)
    with oracle.compat("double", 16):
        b = oracle.pyramid(oracle.params(2000), img)
    # level 1 is computed from the same level 0: only its tail columns can differ
    xt = oracle.resize_tail_x(a[1].shape[1], 16)
    assert np.array_equal(a[1][:, :xt], b[1][:, :xt])
    assert not np.array_equal(a[1][:, xt:], b[1][:, xt:])


def test_trig_modes_identical_on_golden_frames(oracle):
    p = oracle.params(1000)
    for seed in range(4):
        img = synth_image(seed, 640, 480)
        with oracle.compat("double", 0):
            k0, d0, _ = oracle.extract(p, img)
        with oracle.compat("float", 0):
            k1, d1, _ = oracle.extract(p, img)
        assert np.array_equal(k0, k1) and np.array_equal(d0, d1)


def test_compat_restores(oracle):
    prev = oracle.set_compat()
    with oracle.compat("float", 1):
        assert oracle.set_compat() == ("float", 1)
    assert oracle.set_compat() == prev == ("double", 0)
