"""Host-side validation of the batched matcher wrappers (no GPU: the checks run before any C-ABI call).

The kernels behind orbm_search_for_initialization / orbm_search_by_projection_reloc index their arrays
by the batch totals (kp_begin[-1], q_begin[-1], mp_begin[-1]) with no bound of their own, so a short
array must be refused by the wrapper instead of being read out of bounds."""
import numpy as np
import pytest

from orb_slam2_refactored_amd import matcher as M


def _init_batch(K=5, Q=4):
    return {
        "kp_begin": np.array([0, K], np.int32), "kp_xy": np.zeros((K, 2), np.float32),
        "kp_octave": np.zeros(K, np.int32), "kp_desc": np.zeros((K, 32), np.uint8),
        "kp_angle": np.zeros(K, np.float32), "bounds": np.array([[0, 640, 0, 480]], np.float32),
        "q_begin": np.array([0, Q], np.int32), "q_octave": np.zeros(Q, np.int32),
        "q_desc": np.zeros((Q, 32), np.uint8), "q_angle": np.zeros(Q, np.float32),
        "prev_matched": np.zeros((Q, 2), np.float32), "window": 100, "nnratio": 0.9, "check_orientation": True,
    }


def _reloc_batch(K=6, Mp=3):
    return {
        "kp_begin": np.array([0, K], np.int32), "kp_xy": np.zeros((K, 2), np.float32),
        "kp_octave": np.zeros(K, np.int32), "kp_desc": np.zeros((K, 32), np.uint8),
        "kp_angle": np.zeros(K, np.float32), "kp_claimed": None, "bounds": np.array([[0, 640, 0, 480]], np.float32),
        "pose": np.zeros((1, 12), np.float32), "camera": np.array([[500, 500, 320, 240]], np.float32),
        "mp_begin": np.array([0, Mp], np.int32), "mp_valid": np.ones(Mp, np.uint8),
        "mp_xw": np.zeros((Mp, 3), np.float32), "mp_max_min": np.ones((Mp, 2), np.float32),
        "mp_desc": np.zeros((Mp, 32), np.uint8), "mp_angle": np.zeros(Mp, np.float32),
        "scale_factors": np.ones(8, np.float32), "log_scale_factor": 0.18, "th": 10.0, "orb_dist": 100,
        "check_orientation": True,
    }


@pytest.mark.parametrize("key,bad", [("kp_desc", np.zeros((4, 32), np.uint8)), ("q_desc", np.zeros((3, 32), np.uint8)),
                                     ("kp_xy", np.zeros((5, 1), np.float32)), ("bounds", np.zeros(3, np.float32))])
def test_search_for_initialization_refuses_short_arrays(key, bad):
    b = _init_batch()
    b[key] = bad
    with pytest.raises(ValueError, match=key):
        M.SearchForInitialization(b)


def test_search_for_initialization_prev_matched_short():
    b = _init_batch()
    b["prev_matched"] = np.zeros((3, 2), np.float32)   # contiguous float32, but one row short
    with pytest.raises(ValueError, match="prev_matched"):
        M.SearchForInitialization(b)


@pytest.mark.parametrize("key,bad", [("mp_desc", np.zeros((2, 32), np.uint8)), ("mp_xw", np.zeros((3, 2), np.float32)),
                                     ("pose", np.zeros((1, 9), np.float32)), ("kp_angle", np.zeros(5, np.float32))])
def test_search_by_projection_reloc_refuses_short_arrays(key, bad):
    b = _reloc_batch()
    b[key] = bad
    with pytest.raises(ValueError, match=key):
        M.SearchByProjectionReloc(b)


def test_row_check_accepts_exact_and_longer_arrays():
    b = _init_batch()
    b["kp_desc"] = np.zeros((7, 32), np.uint8)   # longer than kp_begin[-1] rows: only a prefix is read
    M._check_batch_rows(b, ["kp_xy", "kp_desc", "q_desc", "prev_matched", "bounds"],
                        {"F": 1, "F1": 2, "K": 5, "Q": 4}, "t")


def test_local_ba_refuses_short_arrays():
    from orb_slam2_refactored_amd.optimizer import LocalBundleAdjustment
    from orb_slam2_refactored_amd.synth import make_ba_problem
    pr = make_ba_problem(3, n_kf=5, n_pts=200, n_fixed=1)
    for key in ("edge_cam", "edge_obs", "pose_t", "pose_fixed"):
        bad = dict(pr)
        bad[key] = np.asarray(pr[key])[:-1]
        with pytest.raises(ValueError, match=key):
            LocalBundleAdjustment(bad)


def test_pose_optimization_refuses_short_arrays():
    from orb_slam2_refactored_amd.optimizer import PoseOptimization
    from orb_slam2_refactored_amd.synth import make_pose_batch
    pb = make_pose_batch(2, n_frames=3, n_edges=[5, 9, 20])
    for key in ("xw", "cam", "inv_sigma2"):
        bad = dict(pb)
        bad[key] = np.asarray(pb[key])[:-1]
        with pytest.raises(ValueError, match=key):
            PoseOptimization(bad)
