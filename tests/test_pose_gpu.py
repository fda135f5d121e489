"""GPU PoseOptimization (orbba_pose_optimization*, Optimizer.cc:345-489) vs the oracle's restatement.

Bar: identical inlier counts and outlier flags, poses within TOL (fp64 on both sides; the GPU
sums edges in a different, fixed order, so results agree to rounding, far inside the north
star's 1e-4 pose tolerance)."""
from pathlib import Path

import numpy as np
import pytest

from orb_slam2_refactored_amd._lib import OrbError
from orb_slam2_refactored_amd.optimizer import PoseOptimization, pose_optimization_device
from orb_slam2_refactored_amd.synth import make_pose_batch

pytestmark = pytest.mark.gpu
GOLDEN = Path(__file__).resolve().parent / "golden"
TOL = 1e-6


def test_wave_primitives_lane_mapping():
    """permlane32/16 swaps + DPP rotates/quad perms must pair each lane with lane ^ m."""
    import ctypes as C
    from orb_slam2_refactored_amd._lib import check, lib, ptr
    rng = np.random.default_rng(0)
    # integers (exact in fp64 whatever the summation order)
    x = rng.integers(-2**20, 2**20, size=(64, 32)).astype(np.float64)
    sc, sm = np.zeros(64), np.zeros(64)
    check(lib().orbba_debug_po_wave(ptr(x), ptr(sc), ptr(sm)), "orbba_debug_po_wave")
    tot = x.sum(axis=0)
    assert np.array_equal(sc, tot[np.arange(64) >> 1])
    assert np.array_equal(sm, np.full(64, tot[0]))


def compare(g, o):
    assert np.array_equal(g["n_inliers"], o["n_inliers"])
    assert np.array_equal(g["outlier"], o["outlier"])
    assert np.abs(g["pose_R"] - o["pose_R"]).max() < TOL
    assert np.abs(g["pose_t"] - o["pose_t"]).max() < TOL


@pytest.mark.parametrize("kw", [
    dict(seed=0, n_frames=16, n_edges=600),
    dict(seed=1, n_frames=8, n_edges=[0, 1, 2, 3, 9, 10, 11, 257]),
    dict(seed=2, n_frames=6, n_edges=1500, stereo_frac=0.0),
    dict(seed=3, n_frames=6, n_edges=800, stereo_frac=1.0),
    dict(seed=4, n_frames=6, n_edges=400, outlier_frac=0.4, rot_deg=2.0, trans_m=0.3),
    dict(seed=5, n_frames=64, n_edges=300),
])
def test_pose_matches_oracle(oracle, kw):
    b = make_pose_batch(**kw)
    compare(PoseOptimization(b), oracle.pose_optimization(b))


def test_pose_golden():
    z = np.load(GOLDEN / "pose_opt_small.npz")
    b = {k: z[k] for k in z.files if not k.startswith("out_")}
    g = PoseOptimization(b)
    compare(g, dict(pose_R=z["out_pose_R"], pose_t=z["out_pose_t"], n_inliers=z["out_n_inliers"],
                    outlier=z["out_outlier"]))


def test_pose_all_outliers(oracle):
    b = make_pose_batch(seed=7, n_frames=2, n_edges=40, outlier_frac=1.0)
    b["obs"][:, 0] += 400.0
    g = PoseOptimization(b)
    compare(g, oracle.pose_optimization(b))
    assert max(g["n_inliers"]) <= 1   # a garbage point can land inside the chi2 gate by chance


def test_pose_max_edges(oracle):
    b = make_pose_batch(seed=8, n_frames=2, n_edges=[16384, 5])
    compare(PoseOptimization(b), oracle.pose_optimization(b))
    big = make_pose_batch(seed=9, n_frames=1, n_edges=16385)
    with pytest.raises(OrbError):
        PoseOptimization(big)


def test_pose_device_matches_host_and_is_deterministic():
    import torch
    b = make_pose_batch(seed=10, n_frames=32, n_edges=700)
    h = PoseOptimization(b)
    dev = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in b.items() if not k.startswith("gt_")}
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        d1 = pose_optimization_device(dev, stream=s)
        d2 = pose_optimization_device(dev, stream=s)
    s.synchronize()
    for k in ("pose_R", "pose_t", "n_inliers"):
        assert np.array_equal(d1[k].cpu().numpy(), h[k])
        assert torch.equal(d1[k], d2[k])
    assert np.array_equal(d1["outlier"].cpu().numpy()[:len(h["outlier"])], h["outlier"])


def test_pose_device_oversized_frame_flags_minus_one():
    import torch
    b = make_pose_batch(seed=11, n_frames=2, n_edges=[16385, 50])
    dev = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in b.items() if not k.startswith("gt_")}
    d = pose_optimization_device(dev)
    torch.cuda.synchronize()
    n = d["n_inliers"].cpu().numpy()
    assert n[0] == -1 and n[1] > 0
    assert np.array_equal(d["pose_R"][0].cpu().numpy(), b["pose_R"][0])
