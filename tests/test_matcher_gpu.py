"""GPU parity of the Hamming matchers against the oracle (exact integers / indices)."""
from pathlib import Path

import numpy as np
import pytest

from orb_slam2_refactored_amd import ORBmatcher
from tri_case import make_case, oracle_run

pytestmark = pytest.mark.gpu
GOLDEN = Path(__file__).resolve().parent / "golden"


def rand_desc(rng, n, p=0.5):
    bits = (rng.random((n, 256)) < p).astype(np.uint8)
    return np.packbits(bits, axis=1, bitorder="little")


@pytest.mark.parametrize("nA,nB", [(1, 1), (300, 1), (257, 513), (2000, 2000), (1000, 0), (0, 10), (64, 255)])
def test_bf_match_random(oracle, nA, nB):
    rng = np.random.default_rng(nA * 7 + nB)
    A = rand_desc(rng, nA)
    B = rand_desc(rng, nB)
    if nB > 10:
        B[7] = B[3]
        A[: min(nA, 5)] = B[3] ^ np.uint8(1)   # ties on best
    m = ORBmatcher(0.6, False)
    got = m.MatchBruteForce(A, B)
    exp = oracle.bf_match(A, B)
    for g, e in zip(got, exp):
        assert np.array_equal(g, e)


@pytest.mark.parametrize("fp4", ["0", "1"])
@pytest.mark.parametrize("nA,nB", [(1, 1), (257, 513), (2000, 2000), (300, 2049), (100, 4500)])
def test_bf_match_both_matrix_paths(oracle, monkeypatch, fp4, nA, nB):
    """The FP4 block-scaled MFMA kernel (default) and the i8 MFMA kernel (ORBM_FP4=0) are both exact:
    random descriptors with best / second ties, all-ones and all-zeros rows (distance 0 and 256)."""
    monkeypatch.setenv("ORBM_FP4", fp4)
    rng = np.random.default_rng(nA * 3 + nB)
    A = rand_desc(rng, nA)
    B = rand_desc(rng, nB)
    if nB > 10 and nA > 6:
        B[7] = B[3]
        A[:5] = B[3] ^ np.uint8(1)
        A[5] = 0xFF
        B[9] = 0xFF
        A[6] = 0
    got = ORBmatcher(0.6, False).MatchBruteForce(A, B)
    exp = oracle.bf_match(A, B)
    for g, e in zip(got, exp):
        assert np.array_equal(g, e)


@pytest.mark.parametrize("nA,nB", [(300, 2048), (300, 2049), (100, 4500)])
def test_bf_match_chunked(oracle, nA, nB):
    """More than 2048 columns: the chunked kernel carries the top-2 across 2048-column chunks.
    Ties on best / second straddle the chunk boundaries (the lower index must win)."""
    rng = np.random.default_rng(nB)
    A = rand_desc(rng, nA)
    B = rand_desc(rng, nB)
    for j in (2047, 2048, nB - 1):
        if j < nB:
            B[j] = B[5]
    A[:10] = B[5] ^ np.uint8(3)      # best tied across chunks
    A[10:20] = B[nB - 1] ^ np.uint8(1)
    B[nB - 2] = B[nB - 1] ^ np.uint8(1)   # second in the last chunk
    got = ORBmatcher(0.6, False).MatchBruteForce(A, B)
    exp = oracle.bf_match(A, B)
    for g, e in zip(got, exp):
        assert np.array_equal(g, e)


def test_bf_match_near_duplicates(oracle):
    rng = np.random.default_rng(3)
    B = rand_desc(rng, 900, 0.5)
    A = B[rng.integers(0, 900, 700)].copy()
    flip = (rng.random(A.shape) < 0.02)
    A ^= (flip * rng.integers(1, 256, A.shape)).astype(np.uint8)
    got = ORBmatcher(0.6, False).MatchBruteForce(A, B)
    exp = oracle.bf_match(A, B)
    for g, e in zip(got, exp):
        assert np.array_equal(g, e)
    assert (got[3] >= 0).sum() > 100


def test_bf_match_all_256():
    A = np.zeros((3, 32), np.uint8)
    B = np.full((4, 32), 255, np.uint8)
    bi, bd, sd, m = ORBmatcher(0.6, False).MatchBruteForce(A, B)
    assert bi.tolist() == [-1] * 3 and bd.tolist() == [256] * 3 and sd.tolist() == [256] * 3 and m.tolist() == [-1] * 3


def test_bf_match_golden():
    g = np.load(GOLDEN / "bf_match_c1.npz")
    bi, bd, sd, m = ORBmatcher(0.6, False).MatchBruteForce(g["A"], g["B"])
    assert np.array_equal(bi, g["best_idx"]) and np.array_equal(bd, g["best"])
    assert np.array_equal(sd, g["second"]) and np.array_equal(m, g["match"])


def test_descriptor_distance(oracle):
    rng = np.random.default_rng(1)
    A = rand_desc(rng, 20)
    for i in range(19):
        assert ORBmatcher.DescriptorDistance(A[i], A[i + 1]) == oracle.descriptor_distance(A[i], A[i + 1])


def test_batch_device(oracle):
    import torch
    rng = np.random.default_rng(5)
    P, cap = 6, 700
    nA = rng.integers(0, cap, P).astype(np.int32)
    nB = rng.integers(0, cap, P).astype(np.int32)
    A = np.stack([rand_desc(rng, cap) for _ in range(P)])
    B = np.stack([rand_desc(rng, cap) for _ in range(P)])
    out = ORBmatcher(0.6, False).match_batch_device(torch.from_numpy(A).cuda(), torch.from_numpy(nA).cuda(),
                                          torch.from_numpy(B).cuda(), torch.from_numpy(nB).cuda())
    out = out.cpu().numpy()
    for p in range(P):
        exp = oracle.bf_match(A[p, :nA[p]], B[p, :nB[p]])
        for k in range(4):
            assert np.array_equal(out[k, p, :nA[p]], exp[k])
    # pair -> B-frame indirection (match each frame against its predecessor without a copy)
    pb = np.array([(p - 1) % P for p in range(P)], np.int32)
    out = ORBmatcher(0.6, False).match_batch_device(torch.from_numpy(A).cuda(), torch.from_numpy(nA).cuda(),
                                          torch.from_numpy(B).cuda(), torch.from_numpy(nB).cuda(),
                                          pair_b=torch.from_numpy(pb).cuda()).cpu().numpy()
    for p in range(P):
        exp = oracle.bf_match(A[p, :nA[p]], B[pb[p], :nB[pb[p]]])
        for k in range(4):
            assert np.array_equal(out[k, p, :nA[p]], exp[k])


@pytest.mark.parametrize("seed,stereo,single", [(0, False, False), (1, True, False), (2, False, True), (3, False, False)])
def test_search_for_triangulation(oracle, seed, stereo, single):
    kf1, kf2, F = make_case(seed, n1=1500, n2=1600, n_nodes=9, only_single_node=single)
    pairs, got = ORBmatcher(0.6, False).SearchForTriangulation(kf1, kf2, F, stereo)
    exp, n = oracle_run(oracle, kf1, kf2, F, stereo)
    assert np.array_equal(got, exp)
    assert len(pairs) == n and n > 0
    assert [p[0] for p in pairs] == sorted(p[0] for p in pairs)


def test_extract_then_match_same_stream_is_ordered(oracle):
    """Extraction and matching enqueued back to back on the default stream, no host sync between:
    the matcher must see this batch's descriptors (buffers pre-filled with garbage)."""
    import torch
    from orb_slam2_refactored_amd import ORBextractor, synth_image
    frames = np.stack([synth_image(40 + i, 640, 480) for i in range(8)])
    t = torch.from_numpy(frames).cuda()
    ex = ORBextractor(ORBextractor.Parameters(1000))
    cap = ex.max_keypoints(480, 640)
    kps = torch.empty((8, cap, 7), dtype=torch.int32, device="cuda")
    desc = torch.randint(0, 256, (8, cap, 32), dtype=torch.uint8, device="cuda")
    cnt = torch.full((8,), cap, dtype=torch.int32, device="cuda")
    prev = torch.tensor([(i - 1) % 8 for i in range(8)], dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ex.extract_batch_device(t, kps, desc, cnt)
    out = ORBmatcher(0.6, False).match_batch_device(desc, cnt, desc, cnt, pair_b=prev)
    torch.cuda.synchronize()
    d = desc.cpu().numpy()
    n = cnt.cpu().numpy()
    got = out[3].cpu().numpy()
    for i in range(8):
        exp = oracle.bf_match(d[i, :n[i]], d[(i - 1) % 8, :n[(i - 1) % 8]])
        assert np.array_equal(got[i, :n[i]], exp[3]), i
