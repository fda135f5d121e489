"""GPU DBoW2 transform (orbv_*, TemplatedVocabulary.h:1130-1263) vs the oracle: BowVector word ids and
weights (raw doubles) and FeatureVector CSR bit-identical."""
import numpy as np
import pytest

from orb_slam2_refactored_amd._lib import OrbError
from orb_slam2_refactored_amd.synth import make_vocabulary, synth_image, vocabulary_features, write_vocabulary_text
from orb_slam2_refactored_amd.vocabulary import ORBVocabulary

pytestmark = pytest.mark.gpu


def _same(g, o):
    (gw, gv), (gn, go, gi) = g
    (ow, ov), (on, oo, oi) = o
    assert np.array_equal(gw, ow)
    assert np.array_equal(gv.view(np.uint64), ov.view(np.uint64))
    assert np.array_equal(gn, on) and np.array_equal(go, oo) and np.array_equal(gi, oi)


@pytest.mark.parametrize("kw,levelsup,n", [
    (dict(seed=0), 4, 1000), (dict(seed=1, L=5, k=6), 2, 2000), (dict(seed=2, scoring=1, weighting=1), 1, 700),
    (dict(seed=3, scoring=5, weighting=0), 3, 300), (dict(seed=4, scoring=5, weighting=2, order="dfs"), 2, 500),
    (dict(seed=5, weighting=3, early_leaf=0.3), 0, 800), (dict(seed=6, k=12, L=3, early_leaf=0.0), 5, 4096),
    (dict(seed=7, k=20, L=2), 1, 600), (dict(seed=8, stop_frac=0.5), 2, 900),
])
def test_transform_matches_oracle(oracle, kw, levelsup, n):
    voc = make_vocabulary(**kw)
    X = vocabulary_features(voc, 200 + kw["seed"], n)
    g = ORBVocabulary.from_arrays(voc["k"], voc["L"], voc["scoring"], voc["weighting"], voc["parent"],
                                  voc["is_leaf"], voc["desc"], voc["weight"])
    _same(g.transform(X, levelsup), oracle.Vocabulary(voc).transform(X, levelsup))


def test_text_loader_and_limits(oracle, tmp_path):
    voc = make_vocabulary(11, order="dfs", early_leaf=0.2)
    p = tmp_path / "voc.txt"
    write_vocabulary_text(voc, p)
    g = ORBVocabulary.loadFromTextFile(p)
    o = oracle.Vocabulary(path=p)
    assert g.info() == o.info()
    X = vocabulary_features(voc, 12, 1500)
    _same(g.transform(X, 2), o.transform(X, 2))
    _same(g.transform(X[:0], 2), o.transform(X[:0], 2))
    with pytest.raises(OrbError):
        g.transform(np.zeros((4097, 32), np.uint8))
    bad = tmp_path / "bad.txt"
    bad.write_text("30 6 0 0\n")
    with pytest.raises(OrbError):
        ORBVocabulary.loadFromTextFile(bad)


def test_batch_device_on_extracted_frames(oracle):
    """ComputeBoW on a batch straight from orbx_extract_batch_device (descriptors never leave HBM)."""
    import torch
    from orb_slam2_refactored_amd import ORBextractor
    voc = make_vocabulary(13, L=5, k=8)
    g = ORBVocabulary.from_arrays(voc["k"], voc["L"], voc["scoring"], voc["weighting"], voc["parent"],
                                  voc["is_leaf"], voc["desc"], voc["weight"])
    ex = ORBextractor(ORBextractor.Parameters(1000), device=0)
    imgs = torch.from_numpy(np.stack([synth_image(300 + i, 640, 480) for i in range(6)])).cuda()
    kps, desc, counts = ex.extract_batch_device(imgs)
    out = g.transform_batch_device(desc, counts, levelsup=3)
    torch.cuda.synchronize()
    o = oracle.Vocabulary(voc)
    dh, ch = desc.cpu().numpy(), counts.cpu().numpy()
    for f in range(6):
        ow = o.transform(dh[f, :ch[f]], 3)
        nw, nn = int(out["n_words"][f]), int(out["n_nodes"][f])
        off = out["fv_off"][f, :nn + 1].cpu().numpy()
        gw = ((out["bow_word"][f, :nw].cpu().numpy().astype(np.uint32), out["bow_weight"][f, :nw].cpu().numpy()),
              (out["fv_node"][f, :nn].cpu().numpy().astype(np.uint32), off, out["fv_idx"][f, :off[-1]].cpu().numpy()))
        _same(gw, ow)
