"""CPU checks of the DBoW2 restatement (oracle/orb_oracle.cpp Vocabulary; TemplatedVocabulary.h
:1130-1263, :1341-1431) against an independent numpy restatement, and of the text loader against
the array form.  The real ORBvoc.txt is absent, so vocabularies are synthetic (synth.make_vocabulary);
the reference ships no BoW fixtures (parity unpinned vs a real DBoW2 build)."""
import numpy as np
import pytest

from orb_slam2_refactored_amd.synth import make_vocabulary, vocabulary_features, write_vocabulary_text


def _np_transform(voc, X, levelsup):
    parent, leaf, D, W = voc["parent"], voc["is_leaf"], voc["desc"], voc["weight"]
    n_nodes = len(parent)
    children = [[] for _ in range(n_nodes)]
    for i in range(1, n_nodes):
        children[parent[i]].append(i)
    word = np.zeros(n_nodes, np.int64)
    word[np.nonzero(leaf)[0]] = np.arange(int(leaf.sum()))
    bitsD = np.unpackbits(D, axis=1)
    nid_level = voc["L"] - levelsup
    bow, fv = {}, {}
    tf = voc["weighting"] in (0, 1)
    for i, x in enumerate(np.unpackbits(np.asarray(X, np.uint8), axis=1)):
        node, level, nid = 0, 0, (0 if nid_level <= 0 else None)
        while children[node]:
            level += 1
            ch = children[node]
            d = (bitsD[ch] != x).sum(axis=1)
            node = ch[int(np.argmin(d))]   # first minimum
            if level == nid_level:
                nid = node
        if nid is None:
            nid = node
        w = W[node]
        if w > 0:
            wid = int(word[node]) if leaf[node] else 0
            if tf:
                bow[wid] = bow[wid] + w if wid in bow else w
            elif wid not in bow:
                bow[wid] = w
            fv.setdefault(nid, []).append(i)
    keys = sorted(bow)
    vals = [bow[k] for k in keys]
    sc = voc["scoring"]
    if sc != 5:
        norm = 0.0
        if sc == 1:
            for v in vals:
                norm += v * v
            norm = np.sqrt(norm)
        else:
            for v in vals:
                norm += abs(v)
        if norm > 0:
            vals = [v / norm for v in vals]
    elif tf and vals:
        vals = [v / float(len(vals)) for v in vals]
    nodes = sorted(fv)
    off = np.concatenate([[0], np.cumsum([len(fv[k]) for k in nodes])]).astype(np.int32)
    idx = np.array([i for k in nodes for i in fv[k]], np.int32)
    return (np.array(keys, np.uint32), np.array(vals)), (np.array(nodes, np.uint32), off, idx)


@pytest.mark.parametrize("kw,levelsup", [
    (dict(seed=0), 4), (dict(seed=1, L=5, k=6), 2), (dict(seed=2, scoring=1, weighting=1), 1),
    (dict(seed=3, scoring=5, weighting=0), 3), (dict(seed=4, scoring=5, weighting=2, order="dfs"), 2),
    (dict(seed=5, weighting=3, early_leaf=0.3), 0), (dict(seed=6, k=12, L=3, early_leaf=0.0), 5),
])
def test_oracle_transform_matches_numpy(oracle, kw, levelsup):
    voc = make_vocabulary(**kw)
    X = vocabulary_features(voc, 100 + kw["seed"], 400)
    (bw, bv), (fn, fo, fi) = oracle.Vocabulary(voc).transform(X, levelsup)
    (nbw, nbv), (nfn, nfo, nfi) = _np_transform(voc, X, levelsup)
    assert np.array_equal(bw, nbw) and np.array_equal(bv, nbv)   # bit-exact doubles
    assert np.array_equal(fn, nfn) and np.array_equal(fo, nfo) and np.array_equal(fi, nfi)


def test_text_loader_equals_arrays(oracle, tmp_path):
    voc = make_vocabulary(7, order="dfs", early_leaf=0.2)
    p = tmp_path / "voc.txt"
    write_vocabulary_text(voc, p)
    a, b = oracle.Vocabulary(voc), oracle.Vocabulary(path=p)
    assert a.info() == b.info()
    X = vocabulary_features(voc, 8, 300)
    ra, rb = a.transform(X, 2), b.transform(X, 2)
    for u, v in zip(ra[0] + ra[1], rb[0] + rb[1]):
        assert np.array_equal(u, v)


def test_empty_input_and_stopped_words(oracle):
    voc = make_vocabulary(9, stop_frac=1.0)   # every word stopped: both vectors empty
    (bw, bv), (fn, fo, fi) = oracle.Vocabulary(voc).transform(vocabulary_features(voc, 1, 50))
    assert len(bw) == 0 and len(fn) == 0 and list(fo) == [0]
    (bw, bv), (fn, fo, fi) = oracle.Vocabulary(make_vocabulary(10)).transform(np.zeros((0, 32), np.uint8))
    assert len(bw) == 0 and len(fn) == 0
