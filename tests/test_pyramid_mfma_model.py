"""The arithmetic identity behind pyramid_pair_mfma_kernel (orbx.hip), checked on the CPU.

The horizontal pass of cv::resize INTER_LINEAR 8U (src/ORBextractor.cc:1080-1090 calls it through
ComputePyramid) is one f16 matrix product per block of 16 output columns: A = the column taps a0 /
a1 at their source offsets from the block's dword-aligned first tap kb, B = 1024 + pixel (f16), C =
2^23 - 1024 (a0 + a1).  Every partial sum is an integer of magnitude below 2^24, so the f32 result
is 2^23 + h exactly for any summation order, and its float bits hold h (and h & 0xffff0, the
vertical pass's operand) in their low 20 bits.  This test builds the tables as the host does
(pyr_mfma_tables) for the C1 / C2 level widths at scale 1.2 and checks the identity against the
integer sum on random rows, with the products summed in float32 in a random order."""
import math

import numpy as np
import pytest


def xtab(sw, dw):
    """cv::resize's horizontal taps as orbx.hip setup_geometry builds them (sx0, sx1, a0, a1)."""
    scale = 1.0 / (dw / sw)
    sx0, sx1, a0, a1 = [], [], [], []
    xmax = dw
    raw = []
    for dx in range(dw):
        fx = np.float32((dx + 0.5) * scale - 0.5)
        sx = int(math.floor(fx))
        fx = np.float32(fx - np.float32(sx))
        if sx < 0:
            fx, sx = np.float32(0), 0
        if sx + 1 >= sw:
            xmax = min(xmax, dx)
            if sx >= sw - 1:
                fx, sx = np.float32(0), sw - 1
        raw.append((sx, int(np.rint(np.float32(1 - fx) * np.float32(2048))), int(np.rint(fx * np.float32(2048)))))
    for dx, (sx, w0, w1) in enumerate(raw):
        s1 = min(sx + 1, sw - 1)
        if dx >= xmax:
            s1, w0, w1 = sx, 2048, 0
        sx0.append(sx), sx1.append(s1), a0.append(w0), a1.append(w1)
    return np.array(sx0), np.array(sx1), np.array(a0), np.array(a1)


def blocks(sx0, sx1, a0, a1):
    """Per 16-column block: kb and the dense 16 x 32 weight matrix (None when K = 32 does not fit)."""
    out = []
    dw = len(sx0)
    for j in range((dw + 15) // 16):
        kb = sx0[16 * j] & ~3
        A = np.zeros((16, 32), np.float64)
        C = np.full(16, 2.0 ** 23)
        for m in range(16):
            c = 16 * j + m
            if c >= dw:
                continue
            e0, e1 = sx0[c] - kb, sx1[c] - kb
            if e1 > 31:
                return None
            A[m, e0] += a0[c]
            A[m, e1] += a1[c]
            C[m] = 2.0 ** 23 - 1024 * (a0[c] + a1[c])
        assert A.max() <= 2048 and np.all(A == A.astype(np.float16).astype(np.float64)), "taps exact in f16"
        out.append((kb, A, C))
    return out


@pytest.mark.parametrize("cols", [640, 752, 1241])
def test_horizontal_sums_from_float_bits(cols):
    rng = np.random.default_rng(cols)
    sw = cols
    for level in range(1, 8):
        dw = int(np.rint(np.float32(1 / 1.2 ** level) * np.float32(cols)))
        sx0, sx1, a0, a1 = xtab(sw, dw)
        bl = blocks(sx0, sx1, a0, a1)
        assert bl is not None, f"level {level}: a block's taps exceed K = 32"
        row = rng.integers(0, 256, sw + 40).astype(np.int64)
        row[:8] = 255   # saturated runs: the largest sums
        for j, (kb, A, C) in enumerate(bl):
            B = 1024.0 + row[kb:kb + 32]
            for m in range(16):
                c = 16 * j + m
                if c >= dw:
                    continue
                h = int(row[sx0[c]] * a0[c] + row[sx1[c]] * a1[c])
                terms = np.concatenate([[C[m]], A[m] * B]).astype(np.float32)
                assert np.all(np.abs(terms) < 2 ** 24)
                acc = np.float32(0)
                for t in rng.permutation(terms):   # any order: every partial sum stays an integer < 2^24
                    acc = np.float32(acc + t)
                    assert abs(float(acc)) < 2 ** 24 and float(acc) == math.floor(float(acc))
                bits = int(np.float32(acc).view(np.uint32))
                assert bits & 0xFFFFF == h and bits & 0xFFFF0 == h & 0xFFFF0, (level, c)
        sw = dw
