"""Oracle matcher semantics vs an independent numpy statement of the reference loops. CPU only."""
import numpy as np
import pytest


def np_hamming(A, B):
    x = np.bitwise_xor(A[:, None, :], B[None, :, :])
    return np.unpackbits(x, axis=2).sum(axis=2)


def np_top2(A, B):
    """best / lowest-index argmin / second order statistic, both initialised to 256 (ORBmatcher.cc:477-498)."""
    nA = len(A)
    bi = np.full(nA, -1, np.int32)
    bd = np.full(nA, 256, np.int32)
    sd = np.full(nA, 256, np.int32)
    if len(B) == 0:
        return bi, bd, sd
    D = np_hamming(A, B)
    for i in range(nA):
        row = D[i]
        j = int(np.argmin(row))
        if row[j] < 256:
            bi[i], bd[i] = j, row[j]
            srt = np.sort(row)
            sd[i] = min(srt[1] if len(srt) > 1 else 256, 256)
        else:
            sd[i] = 256
    return bi, bd, sd


@pytest.mark.parametrize("nA,nB,bits", [(50, 70, 0.5), (40, 1, 0.5), (30, 0, 0.5), (64, 200, 0.05)])
def test_oracle_top2_matches_numpy(oracle, nA, nB, bits):
    rng = np.random.default_rng(nA * 1000 + nB)
    A = (rng.random((nA, 256)) < bits).astype(np.uint8)
    B = (rng.random((nB, 256)) < bits).astype(np.uint8)
    if nB > 3:
        B[3] = B[1]   # duplicate rows -> ties
    A8, B8 = np.packbits(A, axis=1, bitorder="little"), np.packbits(B, axis=1, bitorder="little")
    bi, bd, sd, m = oracle.bf_match(A8, B8)
    ebi, ebd, esd = np_top2(A8, B8)
    assert np.array_equal(bd, ebd) and np.array_equal(sd, esd) and np.array_equal(bi, ebi)
    acc = (ebd <= 50) & (ebd.astype(np.float32) < np.float32(0.6) * esd.astype(np.float32))
    assert np.array_equal(m, np.where(acc, ebi, -1))


def test_oracle_all_256_keeps_minus_one(oracle):
    A = np.zeros((2, 32), np.uint8)
    B = np.full((3, 32), 255, np.uint8)
    bi, bd, sd, m = oracle.bf_match(A, B)
    assert bi.tolist() == [-1, -1] and bd.tolist() == [256, 256] and sd.tolist() == [256, 256]


def test_descriptor_distance(oracle):
    a = np.zeros(32, np.uint8)
    b = np.zeros(32, np.uint8)
    b[0], b[31] = 0b1011, 0x80
    assert oracle.descriptor_distance(a, b) == 4
