"""pyramid_pair_mfma_kernel (ORBX_PYR_MFMA=1: the horizontal pass of cv::resize on v_mfma_f32_16x16x32_f16,
the vertical taps in source-row space through DPP; DESIGN §4 "Pyramid, round 5") against the oracle's
ComputePyramid (src/ORBextractor.cc:455-470), at the bench / config shapes, odd widths and heights,
both OpenCV resize-tail modes and the batched device path.  Off by default (slower than the VALU pair
kernel); these tests keep the kept code exact."""
import numpy as np
import pytest
import torch

from orb_slam2_refactored_amd import ORBextractor
from orb_slam2_refactored_amd.synth import synth_image, textured_image

pytestmark = pytest.mark.gpu


def make(nf=1000):
    return ORBextractor(ORBextractor.Parameters(nf, 1.2, 8, 20, 7))


@pytest.fixture
def mfma_env(monkeypatch):
    monkeypatch.setenv("ORBX_PYR_MFMA", "1")


@pytest.mark.parametrize("W,H,seed", [(640, 480, 0), (1280, 720, 1), (1242, 375, 2), (643, 481, 3), (752, 480, 4),
                                      (1241, 376, 5)])
def test_mfma_pyramid_bit_exact(oracle, mfma_env, W, H, seed):
    img = synth_image(seed, W, H) if seed % 2 == 0 else textured_image(seed, W, H)
    ex = make()
    ex.Extract(img)
    got = ex.GetImagePyramid()
    exp = oracle.pyramid(oracle.params(1000), img)
    for l, (g, e) in enumerate(zip(got, exp)):
        assert g.shape == e.shape, l
        assert np.array_equal(g, e), f"level {l}: {np.count_nonzero(g != e)} px differ"


@pytest.mark.parametrize("simd", [0, 1, 32])
def test_mfma_pyramid_resize_tail_modes(oracle, mfma_env, simd):
    """Every VResizeLinear tail mode (orbx_set_opencv_compat): the tail columns take the scalar formula
    from the full horizontal sums the matrix-core pass keeps for tail blocks."""
    from oracle_api import compat
    img = textured_image(11, 1280, 720)
    ex = make()
    ex.set_opencv_compat(resize_simd=simd)
    ex.Extract(img)
    got = ex.GetImagePyramid()
    with compat(resize_simd=simd):
        exp = oracle.pyramid(oracle.params(1000), img)
    for l, (g, e) in enumerate(zip(got, exp)):
        assert np.array_equal(g, e), f"simd {simd} level {l}: {np.count_nonzero(g != e)} px differ"


def test_mfma_pyramid_batch_keypoints_equal(mfma_env, monkeypatch):
    """A batch through the matrix-core pyramid gives the keypoints and descriptors of the VALU pyramid."""
    frames = np.stack([textured_image(20 + i, 1280, 720) if i % 2 else synth_image(20 + i, 1280, 720)
                       for i in range(6)])
    t = torch.from_numpy(frames).cuda()
    out_m = [x.cpu().numpy() for x in make(2000).extract_batch_device(t)]
    monkeypatch.setenv("ORBX_PYR_MFMA", "0")
    out_v = [x.cpu().numpy() for x in make(2000).extract_batch_device(t)]
    assert np.array_equal(out_m[2], out_v[2])
    for i, n in enumerate(out_v[2]):
        assert np.array_equal(out_m[0][i, :n], out_v[0][i, :n])
        assert np.array_equal(out_m[1][i, :n], out_v[1][i, :n])
