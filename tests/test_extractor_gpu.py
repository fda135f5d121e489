"""GPU parity of ORBextractor::Extract against the CPU oracle: bit-identical pyramid, FAST
candidates, quadtree output, keypoints (all fields, order) and descriptors."""
from pathlib import Path

import numpy as np
import pytest

from orb_slam2_refactored_amd import ORBextractor, synth_image

pytestmark = pytest.mark.gpu
GOLDEN = Path(__file__).resolve().parent / "golden"
FIELDS = ("x", "y", "size", "angle", "response", "octave", "class_id")


def make(nf=1000, ini=20, mn=7, nlevels=8, scale=1.2):
    return ORBextractor(ORBextractor.Parameters(nf, scale, nlevels, ini, mn))


def assert_same_kps(kps, okps, desc, odesc):
    assert len(kps) == len(okps)
    for f in FIELDS:
        assert np.array_equal(kps[f], okps[f]), f
    assert np.array_equal(desc, odesc)


@pytest.mark.parametrize("W,H,seed", [(640, 480, 0), (1280, 720, 1), (1242, 375, 2)])
def test_pyramid_bit_exact(oracle, W, H, seed):
    img = synth_image(seed, W, H)
    ex = make()
    ex.Extract(img)
    got = ex.GetImagePyramid()
    exp = oracle.pyramid(oracle.params(1000), img)
    for l, (g, e) in enumerate(zip(got, exp)):
        assert g.shape == e.shape, l
        assert np.array_equal(g, e), f"level {l}: {np.count_nonzero(g != e)} px differ"


@pytest.mark.parametrize("W,H,seed", [(640, 480, 0), (1280, 720, 3)])
def test_fast_candidates_per_level(oracle, W, H, seed):
    img = synth_image(seed, W, H)
    ex = make(2000)
    ex.Extract(img)
    lv = oracle.pyramid(oracle.params(2000), img)
    for l in range(8):
        got = ex.debug_level(l, stage="candidates")
        exp = oracle.detect_fast(lv[l]).astype(np.int32)
        assert got.shape == exp.shape, (l, got.shape, exp.shape)
        assert np.array_equal(got, exp), l


@pytest.mark.parametrize("kind", ["noise", "smooth_noise", "mixed"])
def test_fast_candidates_dense_cells(oracle, kind):
    """Cells with more corners than the ordered corner list holds (FAST_CLIST_CAP = 256) take the
    zone-scan NMS; mixed images put dense and sparse cells side by side, ini / min thresholds low."""
    rng = np.random.default_rng({"noise": 1, "smooth_noise": 2, "mixed": 3}[kind])
    if kind == "noise":
        img = rng.integers(0, 256, (480, 640)).astype(np.uint8)
    elif kind == "smooth_noise":
        img = np.clip(128 + rng.normal(0, 12, (480, 640)), 0, 255).astype(np.uint8)
    else:
        img = synth_image(21, 640, 480)
        img[100:300, 200:500] = rng.integers(0, 256, (200, 300)).astype(np.uint8)
    for ini, mn in [(20, 7), (5, 2)]:
        ex = make(1000, ini, mn)
        ex.Extract(img)
        p = oracle.params(1000, ini=ini, mn=mn)
        lv = oracle.pyramid(p, img)
        for l in range(8):
            got = ex.debug_level(l, stage="candidates")
            exp = oracle.detect_fast(lv[l], ini, mn).astype(np.int32)
            assert np.array_equal(got, exp), (kind, ini, mn, l, got.shape, exp.shape)


def _patchwork(seed, W, H):
    """Textured, low-contrast-textured (many pixels pass the pre-test at minThFAST, few or no
    corners at iniThFAST) and flat cells side by side, in blocks of 1-3 cells."""
    from orb_slam2_refactored_amd.synth import textured_image
    rng = np.random.default_rng(seed)
    img = synth_image(seed, W, H).copy()
    tex = textured_image(seed + 1, W, H)
    weak = np.clip(128 + rng.normal(0, 4, (H, W)), 0, 255).astype(np.uint8)
    y = 0
    while y < H:
        h = int(rng.integers(30, 91))
        x = 0
        while x < W:
            w = int(rng.integers(30, 91))
            k = rng.integers(0, 3)
            if k == 1:
                img[y:y + h, x:x + w] = tex[y:y + h, x:x + w]
            elif k == 2:
                img[y:y + h, x:x + w] = weak[y:y + h, x:x + w]
            x += w
        y += h
    return img


@pytest.mark.parametrize("spec", [1, 8])
@pytest.mark.parametrize("kind", ["textured", "patchwork"])
def test_fast_speculative_pass(oracle, monkeypatch, spec, kind):
    """The speculative iniThFAST pass (ORBX_FAST_SPEC: run when the wavefront's previous cell
    kept >= spec corners at iniThFAST) and its fall-back full pass leave every candidate
    unchanged; spec 1 sends nearly every cell after a textured one through the fall-back."""
    from orb_slam2_refactored_amd.synth import textured_image
    img = textured_image(77, 640, 480) if kind == "textured" else _patchwork(5, 640, 480)
    monkeypatch.setenv("ORBX_FAST_SPEC", str(spec))
    ex = make(2000)
    ex.Extract(img)
    lv = oracle.pyramid(oracle.params(2000), img)
    for l in range(8):
        got = ex.debug_level(l, stage="candidates")
        exp = oracle.detect_fast(lv[l]).astype(np.int32)
        assert np.array_equal(got, exp), (kind, spec, l, got.shape, exp.shape)


def test_fast_speculative_pass_batch_equal(monkeypatch):
    """Batched device output with the speculative pass off (0) and on (1, 8) is bit-identical."""
    import torch
    frames = np.stack([_patchwork(40 + i, 320, 240) for i in range(24)])
    t = torch.from_numpy(frames).cuda()
    outs = []
    for spec in (0, 1, 8):
        monkeypatch.setenv("ORBX_FAST_SPEC", str(spec))
        o = make(500).extract_batch_device(t)
        torch.cuda.synchronize()
        outs.append([x.cpu().numpy() for x in o])
    cnt = outs[0][2]
    for o in outs[1:]:
        assert np.array_equal(cnt, o[2])
        for i, n in enumerate(cnt):
            assert np.array_equal(outs[0][0][i, :n], o[0][i, :n]), i
            assert np.array_equal(outs[0][1][i, :n], o[1][i, :n]), i


@pytest.mark.parametrize("W,H,seed,nf", [(640, 480, 0, 1000), (1280, 720, 3, 2000), (640, 480, 9, 5000)])
def test_quadtree_per_level(oracle, W, H, seed, nf):
    img = synth_image(seed, W, H)
    ex = make(nf)
    ex.Extract(img)
    lv = oracle.pyramid(oracle.params(nf), img)
    quota = oracle.scale_tables(oracle.params(nf))["quota"]
    for l in range(8):
        cand = oracle.detect_fast(lv[l])
        exp = oracle.quadtree(cand, lv[l].shape[0], lv[l].shape[1], int(quota[l])).astype(np.int32)
        got = ex.debug_level(l, stage="selected")
        assert np.array_equal(got, exp), l


@pytest.mark.parametrize("kind,W,H,nf", [("textured", 1280, 720, 2000), ("textured", 1920, 1080, 4000),
                                         ("patchwork", 1280, 720, 2000), ("noise", 1280, 720, 1000)])
def test_quadtree_per_level_dense(oracle, kind, W, H, nf):
    """Levels with tens of thousands of candidates: global candidate arrays, whole-block splits of
    nodes above QT_BIG points, register-resident wave splits, batched gathers of full cells."""
    from orb_slam2_refactored_amd.synth import textured_image
    if kind == "textured":
        img = textured_image(9, W, H)
    elif kind == "patchwork":
        img = _patchwork(11, W, H)
    else:
        img = np.random.default_rng(12).integers(0, 256, (H, W)).astype(np.uint8)
    ex = make(nf)
    kps, desc = ex.Extract(img)
    p = oracle.params(nf)
    lv = oracle.pyramid(p, img)
    quota = oracle.scale_tables(p)["quota"]
    for l in range(8):
        cand = oracle.detect_fast(lv[l])
        exp = oracle.quadtree(cand, lv[l].shape[0], lv[l].shape[1], int(quota[l])).astype(np.int32)
        got = ex.debug_level(l, stage="selected")
        assert np.array_equal(got, exp), (kind, l, len(cand), got.shape, exp.shape)
    okps, odesc, _ = oracle.extract(p, img)
    assert_same_kps(kps, okps, desc, odesc)


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_extract_c1_golden(seed):
    g = np.load(GOLDEN / f"extract_c1_seed{seed}.npz")
    img = synth_image(int(g["seed"]), int(g["width"]), int(g["height"]))
    assert np.array_equal(img, g["image"]), "synthetic generator changed"
    ex = make(int(g["nfeatures"]))
    ex.set_opencv_compat(str(g["trig"]), int(g["resize_simd"]))   # the switches the fixture was made with
    kps, desc = ex.Extract(img)
    okps = g["kps"].astype(np.int32).view(kps.dtype).reshape(-1)
    assert_same_kps(kps, okps, desc, g["desc"])


@pytest.mark.parametrize("W,H,seed,nf", [(1280, 720, 0, 2000), (1242, 375, 1, 2000), (640, 480, 11, 2000),
                                         (752, 480, 4, 1500), (320, 240, 5, 500)])
def test_extract_bit_exact(oracle, W, H, seed, nf):
    img = synth_image(seed, W, H)
    kps, desc = make(nf).Extract(img)
    okps, odesc, _ = oracle.extract(oracle.params(nf), img)
    assert_same_kps(kps, okps, desc, odesc)


@pytest.mark.parametrize("seed", [0, 1])
def test_extract_noise_image(oracle, seed):
    """Pure noise: thousands of FAST candidates per level, deep quadtree phase-2 rounds."""
    rng = np.random.default_rng(100 + seed)
    img = rng.integers(0, 256, (480, 640)).astype(np.uint8)
    kps, desc = make(1000).Extract(img)
    okps, odesc, _ = oracle.extract(oracle.params(1000), img)
    assert_same_kps(kps, okps, desc, odesc)


def test_extract_params_variants(oracle):
    rng = np.random.default_rng(7)
    for k in range(4):
        nf = int(rng.integers(100, 3000))
        ini = int(rng.integers(8, 40))
        mn = int(rng.integers(3, ini))
        nl = int(rng.integers(3, 9))
        sc = float(np.float32(rng.uniform(1.1, 1.5)))
        W, H = int(rng.integers(200, 900)), int(rng.integers(150, 600))
        img = synth_image(200 + k, W, H)
        p = oracle.params(nf, sc, nl, ini, mn)
        okps, odesc, _ = oracle.extract(p, img)
        kps, desc = make(nf, ini, mn, nl, sc).Extract(img)
        if len(okps) == 0:
            assert desc is None
        else:
            assert_same_kps(kps, okps, desc, odesc)


def test_no_keypoints_quirk():
    ex = make()
    sentinel = ["untouched"]
    kps, desc = ex.Extract(np.full((480, 640), 90, np.uint8), sentinel)
    assert kps is sentinel and desc is None


def test_strided_input(oracle):
    big = synth_image(12, 700, 500)
    view = big[10:490, 30:670]   # non-contiguous rows (step 700)
    kps, desc = make().Extract(view)
    okps, odesc, _ = oracle.extract(oracle.params(1000), np.ascontiguousarray(view))
    assert_same_kps(kps, okps, desc, odesc)


@pytest.mark.parametrize("W", [641, 643, 1277])
def test_odd_row_step(oracle, W):
    """A level-0 row step that is not a dword multiple (the host API uploads with step = cols)
    takes the per-group realignment path of the FAST crop staging; every pyramid level has a
    16-B aligned stride."""
    img = synth_image(13 + W, W, 480)
    kps, desc = make().Extract(img)
    okps, odesc, _ = oracle.extract(oracle.params(1000), img)
    assert_same_kps(kps, okps, desc, odesc)


def test_batch_device_odd_step(oracle):
    import torch
    frames = np.stack([synth_image(40 + i, 701, 480) for i in range(3)])
    t = torch.from_numpy(frames).cuda()[:, :, 3:643]   # row step 701, base offset 3
    assert t.stride(1) == 701
    ex = make()
    kps_t, desc_t, cnt_t = ex.extract_batch_device(t)
    torch.cuda.synchronize()
    for i in range(3):
        okps, odesc, _ = oracle.extract(oracle.params(1000), np.ascontiguousarray(frames[i][:, 3:643]))
        n = int(cnt_t[i])
        kps = ex.kps_to_numpy(kps_t[i, :n].cpu().numpy())
        assert_same_kps(kps, okps, desc_t[i, :n].cpu().numpy(), odesc)


def test_batch_device_matches_single(oracle):
    import torch
    frames = np.stack([synth_image(20 + i, 640, 480) for i in range(5)])
    ex = make()
    t = torch.from_numpy(frames).cuda()
    kps_t, desc_t, cnt_t = ex.extract_batch_device(t)
    torch.cuda.synchronize()
    cnt = cnt_t.cpu().numpy()
    kps_all = kps_t.cpu().numpy()
    desc_all = desc_t.cpu().numpy()
    for i in range(5):
        okps, odesc, _ = oracle.extract(oracle.params(1000), frames[i])
        n = int(cnt[i])
        kps = ORBextractor.kps_to_numpy(kps_all[i, :n])
        assert_same_kps(kps, okps, desc_all[i, :n], odesc)


def test_extract_batch_repeatable():
    """The same batch extracted three times gives bit-identical keypoints and descriptors (round 4: two
    builds broke this while every parity test against the oracle still passed)."""
    import torch
    frames = np.stack([_patchwork(60 + i, 320, 240) for i in range(16)])
    t = torch.from_numpy(frames).cuda()
    ex = make(500)
    outs = []
    for _ in range(3):
        o = ex.extract_batch_device(t)
        torch.cuda.synchronize()
        outs.append([x.cpu().numpy() for x in o])
    for o in outs[1:]:
        assert np.array_equal(outs[0][2], o[2])
        for i, n in enumerate(outs[0][2]):
            assert np.array_equal(outs[0][0][i, :n], o[0][i, :n]), i
            assert np.array_equal(outs[0][1][i, :n], o[1][i, :n]), i


@pytest.mark.parametrize("nsub,cpw", [(1, 1), (2, 4), (3, 3)])
def test_batch_sub_streams_and_cells_per_wave(monkeypatch, nsub, cpw):
    """Sub-batches on side streams (ORBX_NSUB) and the FAST cells-per-wave pipelining
    (ORBX_FAST_CPW) must not change a bit of the output; 50 frames -> ragged chunks."""
    import torch
    frames = np.stack([synth_image(100 + (i % 7), 320, 240) for i in range(50)])
    t = torch.from_numpy(frames).cuda()
    ref = make(500).extract_batch_device(t)
    torch.cuda.synchronize()
    monkeypatch.setenv("ORBX_NSUB", str(nsub))
    monkeypatch.setenv("ORBX_FAST_CPW", str(cpw))
    out = make(500).extract_batch_device(t)
    torch.cuda.synchronize()
    cnt = ref[2].cpu().numpy()
    assert np.array_equal(cnt, out[2].cpu().numpy())
    k0, k1 = ref[0].cpu().numpy(), out[0].cpu().numpy()
    d0, d1 = ref[1].cpu().numpy(), out[1].cpu().numpy()
    for i, n in enumerate(cnt):
        assert np.array_equal(k0[i, :n], k1[i, :n]), i
        assert np.array_equal(d0[i, :n], d1[i, :n]), i


def test_batch_status_clean_and_induced_fault():
    """The batched path reports device capacity faults: clean batches read 0; a handle whose quadtree
    node capacity is shrunk (ORBX_DEBUG_NC test hook) trips FAULT_QT_NODES (bit 0) on a dense level,
    truncates instead of writing out of bounds, and the word clears once read."""
    import os
    import torch
    from orb_slam2_refactored_amd._lib import OrbError
    frames = torch.from_numpy(np.stack([synth_image(500 + i, 1280, 720) for i in range(4)])).cuda()
    ex = ORBextractor(ORBextractor.Parameters(2000))
    ex.extract_batch_device(frames)
    assert ex.batch_status() == 0
    os.environ["ORBX_DEBUG_NC"] = "256"
    try:
        bad = ORBextractor(ORBextractor.Parameters(2000))
    finally:
        del os.environ["ORBX_DEBUG_NC"]
    _, _, cnt = bad.extract_batch_device(frames)
    with pytest.raises(OrbError, match="fault mask 1"):
        bad.batch_status()
    assert bad.batch_status() == 0   # cleared by the read
    assert (cnt.cpu().numpy() <= ex.max_keypoints(720, 1280)).all()


@pytest.mark.parametrize("env", [{"ORBX_DESC_DENSE": "1"}, {"ORBX_DESC_DENSE": "1", "ORBX_DESC_C": "64"},
                                 {"ORBX_DESC_DENSE": "1", "ORBX_DESC_C": "1000"}])
def test_describe_grids_equal(env):
    """describe's grids give identical output: the dense grid (ORBX_DESC_DENSE=1: slot = output row, C
    from the previous batch's largest total) against the default slot-table grid, and a forced small C
    (ORBX_DESC_C) that sends most rows through describe_overflow_kernel."""
    import os
    import torch
    frames = torch.from_numpy(np.stack([synth_image(60 + i, 1280, 720) for i in range(6)])).cuda()
    ref = ORBextractor(ORBextractor.Parameters(2000))
    for _ in range(2):
        r = [t.cpu().numpy() for t in ref.extract_batch_device(frames)]
    os.environ.update(env)
    try:
        alt = ORBextractor(ORBextractor.Parameters(2000))
    finally:
        for k in env:
            del os.environ[k]
    for _ in range(2):
        a = [t.cpu().numpy() for t in alt.extract_batch_device(frames)]
    assert ref.batch_status() == 0 and alt.batch_status() == 0
    assert np.array_equal(r[2], a[2])
    for i, n in enumerate(r[2]):
        assert np.array_equal(r[0][i, :n], a[0][i, :n]) and np.array_equal(r[1][i, :n], a[1][i, :n]), i


@pytest.mark.parametrize("wave", ["0", "1"])
def test_quadtree_block_size_guard(wave, monkeypatch):
    """quadtree_kernel is written for 256-thread blocks (qt_block_split sums 4 per-wave partials and
    scatters 4 x 256-point tiles); round 5's 64-thread experiment wrote out of bounds on dense levels.
    A launch with another block size (ORBX_DEBUG_QT_BLOCK test hook) must set FAULT_BLOCK_SIZE (16),
    write empty levels and touch nothing else -- on the pure-noise frames that faulted."""
    import os
    import torch
    from orb_slam2_refactored_amd._lib import OrbError
    rng = np.random.default_rng(40)
    frames = torch.from_numpy(rng.integers(0, 256, (2, 480, 640)).astype(np.uint8)).cuda()
    monkeypatch.setenv("ORBX_QT_WAVE", wave)   # (1: the wave-per-tree launch clears its four levels too)
    os.environ["ORBX_DEBUG_QT_BLOCK"] = "64"
    try:
        bad = ORBextractor(ORBextractor.Parameters(1000))
    finally:
        del os.environ["ORBX_DEBUG_QT_BLOCK"]
    _, _, cnt = bad.extract_batch_device(frames)
    with pytest.raises(OrbError, match="fault mask 16"):
        bad.batch_status()
    assert (cnt.cpu().numpy() == 0).all()
    ok = ORBextractor(ORBextractor.Parameters(1000))
    _, _, cnt = ok.extract_batch_device(frames)
    assert ok.batch_status() == 0 and (cnt.cpu().numpy() > 0).all()


def test_batch_device_rejects_bad_output_buffers():
    import torch
    frames = torch.from_numpy(np.stack([synth_image(1, 640, 480)] * 2)).cuda()
    ex = ORBextractor(ORBextractor.Parameters(1000))
    cap = ex.max_keypoints(480, 640)
    good_k = torch.empty((2, cap, 7), dtype=torch.int32, device="cuda")
    good_d = torch.empty((2, cap, 32), dtype=torch.uint8, device="cuda")
    good_c = torch.empty(2, dtype=torch.int32, device="cuda")
    with pytest.raises(ValueError):
        ex.extract_batch_device(frames, good_k[:, : cap - 1], good_d, good_c)
    with pytest.raises(ValueError):
        ex.extract_batch_device(frames, good_k, torch.empty((2, cap, 64), dtype=torch.uint8, device="cuda")[:, :, :32],
                                good_c)
    with pytest.raises(ValueError):
        ex.extract_batch_device(frames, good_k, good_d, good_c[:1])
    with pytest.raises(ValueError):
        ex.extract_batch_device(frames.transpose(1, 2).contiguous().transpose(1, 2), good_k, good_d, good_c)
