"""quadtree_kernel's wave-per-tree form (ORBX_QT_WAVE=1, round 6: the trailing levels whose cells one
wavefront's partitioned gather takes, four trees per workgroup, no workgroup barriers) against the
oracle's DistributeOctTree (ORBextractor.cc:542-693) level by level, including dense levels whose points
exceed the wavefront's LDS capacity (HBM path) and nodes past QT_BIG (split by one wavefront here), and
bit-identical batched output against the default workgroup-per-tree form."""
import numpy as np
import pytest

from orb_slam2_refactored_amd import ORBextractor, synth_image
from orb_slam2_refactored_amd.synth import pan_sequence, textured_image

pytestmark = pytest.mark.gpu


def make(nf):
    return ORBextractor(ORBextractor.Parameters(nf, 1.2, 8, 20, 7))


@pytest.mark.parametrize("kind,W,H,nf", [("synth", 1280, 720, 2000), ("synth", 640, 480, 5000),
                                         ("textured", 1280, 720, 2000), ("textured", 1920, 1080, 4000),
                                         ("noise", 1280, 720, 1000)])
@pytest.mark.parametrize("wg", ["2", "1"])
def test_quadtree_wave_per_level(oracle, monkeypatch, kind, W, H, nf, wg):
    monkeypatch.setenv("ORBX_QT_WAVE", "1")
    monkeypatch.setenv("ORBX_QT_WAVE_WG", wg)
    if kind == "synth":
        img = synth_image(3, W, H)
    elif kind == "textured":
        img = textured_image(9, W, H)
    else:
        img = np.random.default_rng(12).integers(0, 256, (H, W)).astype(np.uint8)
    ex = make(nf)
    ex.Extract(img)
    p = oracle.params(nf)
    lv = oracle.pyramid(p, img)
    quota = oracle.scale_tables(p)["quota"]
    for l in range(8):
        cand = oracle.detect_fast(lv[l])
        exp = oracle.quadtree(cand, lv[l].shape[0], lv[l].shape[1], int(quota[l])).astype(np.int32)
        got = ex.debug_level(l, stage="selected")
        assert np.array_equal(got, exp), (kind, l, len(cand), got.shape, exp.shape)


def test_quadtree_wave_batch_identical(monkeypatch):
    import torch
    frames = np.concatenate([pan_sequence(21, 1280, 720, 8), np.stack([textured_image(70 + i, 1280, 720) for i in range(4)])])
    t = torch.from_numpy(frames).cuda()
    outs = []
    for wave in ("0", "1"):
        monkeypatch.setenv("ORBX_QT_WAVE", wave)
        ex = make(2000)
        o = ex.extract_batch_device(t)
        torch.cuda.synchronize()
        assert ex.batch_status() == 0
        outs.append([x.cpu().numpy() for x in o])
    cnt = outs[0][2]
    assert np.array_equal(cnt, outs[1][2])
    for i, n in enumerate(cnt):
        assert np.array_equal(outs[0][0][i, :n], outs[1][0][i, :n]), i
        assert np.array_equal(outs[0][1][i, :n], outs[1][1][i, :n]), i
