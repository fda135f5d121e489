"""GPU LocalBundleAdjustment vs the oracle's g2o restatement: poses within 1e-4 RMSE, identical
outlier set and LM iteration counts (BASELINE.json north star)."""
from pathlib import Path

import numpy as np
import pytest

from orb_slam2_refactored_amd.optimizer import LocalBundleAdjustment
from orb_slam2_refactored_amd.synth import make_ba_problem

pytestmark = pytest.mark.gpu
GOLDEN = Path(__file__).resolve().parent / "golden"
TOL = 1e-4   # pose RMSE tolerance (north star)


def rmse(a, b):
    return float(np.sqrt(np.mean((np.asarray(a) - np.asarray(b)) ** 2)))


def compare(g, o):
    assert rmse(g["pose_t"], o["pose_t"]) < TOL
    assert rmse(g["pose_R"], o["pose_R"]) < TOL
    assert rmse(g["points"], o["points"]) < 10 * TOL
    assert np.array_equal(g["edge_outlier"], o["edge_outlier"])
    assert tuple(g["iterations"]) == tuple(o["iterations"])


@pytest.mark.parametrize("seed,kf,pts,fixed", [(0, 20, 3000, 2), (1, 20, 3000, 2), (2, 12, 1500, 0), (3, 5, 200, 1)])
def test_local_ba_matches_oracle(oracle, seed, kf, pts, fixed):
    pr = make_ba_problem(seed, n_kf=kf, n_pts=pts, n_fixed=fixed)
    g = LocalBundleAdjustment(pr)
    o = oracle.local_ba(pr)
    compare(g, o)
    assert g["chi2"][1] < g["chi2"][0]


def test_local_ba_golden():
    z = np.load(GOLDEN / "local_ba_small.npz")
    pr = {k: z[k] for k in z.files if not k.startswith("out_")}
    g = LocalBundleAdjustment(pr)
    assert rmse(g["pose_t"], z["out_pose_t"]) < TOL
    assert np.array_equal(g["edge_outlier"], z["out_outlier"])
    assert tuple(g["iterations"]) == tuple(z["out_iterations"])


def test_local_ba_stop_flag(oracle):
    pr = make_ba_problem(4, n_kf=6, n_pts=300, n_fixed=1)
    g = LocalBundleAdjustment(pr, stop_flag=1)
    assert tuple(g["iterations"]) == (0, 0)
    assert not g["edge_outlier"].any()
    assert rmse(g["points"], pr["points"]) == 0


def test_local_ba_deterministic():
    pr = make_ba_problem(6, n_kf=10, n_pts=800, n_fixed=1)
    a = LocalBundleAdjustment(pr)
    b = LocalBundleAdjustment(pr)
    assert np.array_equal(a["pose_t"], b["pose_t"]) and np.array_equal(a["points"], b["points"])
