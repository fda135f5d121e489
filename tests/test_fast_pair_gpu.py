"""fast_cells_kernel's PAIR form (ORBX_FAST_PAIR=1, round 6: two vertically consecutive cells of a strip
per pass as one merged zone with a zero separator row in the zone map) against the oracle's DetectFAST
(ORBextractor.cc:489-540: per-cell cv::FAST at iniThFAST, minThFAST retry, cell-local NMS), and
bit-identical batched output against the default one-cell form."""
import numpy as np
import pytest

from orb_slam2_refactored_amd import ORBextractor, synth_image
from orb_slam2_refactored_amd.synth import pan_sequence, textured_image

pytestmark = pytest.mark.gpu


def make(nf=1000, ini=20, mn=7):
    return ORBextractor(ORBextractor.Parameters(nf, 1.2, 8, ini, mn))


def candidates_match(oracle, img, nf=2000, ini=20, mn=7):
    ex = make(nf, ini, mn)
    ex.Extract(img)
    lv = oracle.pyramid(oracle.params(nf, ini=ini, mn=mn), img)
    for l in range(8):
        got = ex.debug_level(l, stage="candidates")
        exp = oracle.detect_fast(lv[l], ini, mn).astype(np.int32)
        assert np.array_equal(got, exp), (l, got.shape, exp.shape)


@pytest.mark.parametrize("kind", ["synth", "textured", "noise", "mixed", "c3"])
@pytest.mark.parametrize("spec", ["8", "1", "0"])
def test_fast_pair_candidates(oracle, monkeypatch, kind, spec):
    monkeypatch.setenv("ORBX_FAST_PAIR", "1")
    monkeypatch.setenv("ORBX_FAST_SPEC", spec)
    rng = np.random.default_rng(5)
    if kind == "synth":
        img = synth_image(3, 1280, 720)
    elif kind == "textured":
        img = textured_image(77, 640, 480)
    elif kind == "noise":   # every pair past the corner list: the zone-scan NMS
        img = rng.integers(0, 256, (480, 640)).astype(np.uint8)
    elif kind == "mixed":
        img = synth_image(21, 640, 480)
        img[100:300, 200:500] = rng.integers(0, 256, (200, 300)).astype(np.uint8)
    else:
        img = synth_image(8, 1242, 375)
    candidates_match(oracle, img)
    if kind in ("noise", "mixed"):
        candidates_match(oracle, img, 1000, 5, 2)


@pytest.mark.parametrize("cpw", ["16", "3", "1"])
def test_fast_pair_batch_identical(monkeypatch, cpw):
    """Batched pan and textured C2 frames: keypoints, descriptors and counts identical to the one-cell
    form, with even, odd and single-cell strips (ORBX_FAST_CPW)."""
    import torch
    frames = np.concatenate([pan_sequence(11, 1280, 720, 12), np.stack([textured_image(90 + i, 1280, 720) for i in range(4)])])
    t = torch.from_numpy(frames).cuda()
    monkeypatch.setenv("ORBX_FAST_CPW", cpw)
    outs = []
    for pair in ("0", "1"):
        monkeypatch.setenv("ORBX_FAST_PAIR", pair)
        ex = make(2000)
        for _ in range(2):   # the second batch runs with the first-cell speculation hints
            o = ex.extract_batch_device(t)
        torch.cuda.synchronize()
        assert ex.batch_status() == 0
        outs.append([x.cpu().numpy() for x in o])
    cnt = outs[0][2]
    assert np.array_equal(cnt, outs[1][2])
    for i, n in enumerate(cnt):
        assert np.array_equal(outs[0][0][i, :n], outs[1][0][i, :n]), i
        assert np.array_equal(outs[0][1][i, :n], outs[1][1][i, :n]), i
