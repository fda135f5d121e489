"""SearchByProjection(Frame& currFrame, const Frame& lastFrame, th, monocular) (ORBmatcher.cc:1279-1362,
TrackWithMotionModel) on the device against the oracle's literal restatement: identical kp_match
(the last assignment per keypoint, erased by CheckOrientation) and match counts.  Inputs from
make_proj_batch (claims, overwrites by points without observations, distance ties, stereo gate,
out-of-grid keypoints) with the level windows of the forward / backward / neither cases."""
import numpy as np
import pytest

from orb_slam2_refactored_amd.matcher import search_by_projection_motion_device
from orb_slam2_refactored_amd.synth import make_proj_batch

pytestmark = pytest.mark.gpu


def _motion_batch(seed, th, check_ori, concentrated, odd_bounds=False):
    b = make_proj_batch(seed, n_frames=6, n_kp=[2000, 1500, 2500, 800, 2000, 0], n_mp=[1500, 1200, 1800, 600, 0, 300],
                        th=th, odd_bounds=odd_bounds)
    rng = np.random.default_rng(seed + 1)
    K, M = int(b["kp_begin"][-1]), int(b["mp_begin"][-1])
    if concentrated:   # a dominant rotation: most pairs in one or two bins
        kp_angle = (40 + rng.normal(0, 4, K)) % 360
        mp_angle = (52 + rng.normal(0, 4, M)) % 360
    else:
        kp_angle = rng.uniform(0, 360, K)
        mp_angle = rng.uniform(0, 360, M)
    m = dict(kp_begin=b["kp_begin"], kp_xy=b["kp_xy"], kp_octave=b["kp_octave"], kp_uright=b["kp_uright"],
             kp_desc=b["kp_desc"], kp_angle=kp_angle.astype(np.float32), kp_claimed=b["kp_claimed"],
             bounds=b["bounds"], mp_begin=b["mp_begin"], mp_valid=b["mp_valid"], mp_proj=b["mp_proj"],
             mp_octave=np.minimum(b["mp_level"], 7).astype(np.int32), mp_desc=b["mp_desc"],
             mp_has_obs=b["mp_has_obs"], mp_angle=mp_angle.astype(np.float32),
             motion=np.array([0, 1, 2, 0, 1, 2], np.int32), scale_factors=b["scale_factors"], th=th,
             check_orientation=check_ori)
    return m


@pytest.mark.parametrize("th", [7.0, 15.0])
@pytest.mark.parametrize("check_ori,concentrated", [(False, False), (True, False), (True, True)])
def test_motion_projection_vs_oracle(oracle, th, check_ori, concentrated):
    import torch
    m = _motion_batch(int(th) * 10 + int(check_ori) + 2 * int(concentrated), th, check_ori, concentrated)
    exp_match, exp_n = oracle.search_by_projection_motion(m)
    g = {k: (torch.from_numpy(np.ascontiguousarray(v)).cuda() if isinstance(v, np.ndarray) and
             k not in ("scale_factors",) else v) for k, v in m.items()}
    km, nm = search_by_projection_motion_device(g)
    torch.cuda.synchronize()
    K = int(m["kp_begin"][-1])
    assert np.array_equal(km.cpu().numpy()[:K], exp_match)
    assert np.array_equal(nm.cpu().numpy(), exp_n)
    assert exp_n[:4].min() > 0


def test_motion_projection_odd_bounds_no_claims(oracle):
    import torch
    m = _motion_batch(77, 7.0, True, True, odd_bounds=True)
    m["kp_claimed"] = None
    m["motion"] = None
    exp_match, exp_n = oracle.search_by_projection_motion(m)
    g = {k: (torch.from_numpy(np.ascontiguousarray(v)).cuda() if isinstance(v, np.ndarray) and
             k not in ("scale_factors",) else v) for k, v in m.items()}
    km, nm = search_by_projection_motion_device(g)
    torch.cuda.synchronize()
    K = int(m["kp_begin"][-1])
    assert np.array_equal(km.cpu().numpy()[:K], exp_match)
    assert np.array_equal(nm.cpu().numpy(), exp_n)


def test_motion_projection_bad_octave_is_skipped(oracle):
    """A last-frame point whose octave lies outside the pyramid has no level to project at: the kernel
    gives it no candidate, the same result as the oracle with that point skipped (mp_valid = 0)."""
    import torch
    m = _motion_batch(91, 7.0, True, False)
    M = int(m["mp_begin"][-1])
    bad = np.arange(0, M, 7)
    m["mp_octave"] = m["mp_octave"].copy()
    m["mp_octave"][bad[0::2]] = -1
    m["mp_octave"][bad[1::2]] = len(m["scale_factors"])
    ref = dict(m)
    ref["mp_valid"] = m["mp_valid"].copy()
    ref["mp_valid"][bad] = 0
    ref["mp_octave"] = np.clip(m["mp_octave"], 0, len(m["scale_factors"]) - 1).astype(np.int32)
    exp_match, exp_n = oracle.search_by_projection_motion(ref)
    g = {k: (torch.from_numpy(np.ascontiguousarray(v)).cuda() if isinstance(v, np.ndarray) and
             k not in ("scale_factors",) else v) for k, v in m.items()}
    km, nm = search_by_projection_motion_device(g)
    torch.cuda.synchronize()
    K = int(m["kp_begin"][-1])
    assert np.array_equal(km.cpu().numpy()[:K], exp_match)
    assert np.array_equal(nm.cpu().numpy(), exp_n)


def test_motion_projection_over_limit_frame_reports_minus_one():
    """A frame above the device keypoint limit gets n_matches = -1 and kp_match = -1 on every keypoint
    (initialised, never garbage), the other frames are unaffected."""
    import torch
    b = make_proj_batch(5, n_frames=2, n_kp=[9000, 500], n_mp=[100, 100], th=7.0)
    K = int(b["kp_begin"][-1])
    rng = np.random.default_rng(5)
    m = dict(kp_begin=b["kp_begin"], kp_xy=b["kp_xy"], kp_octave=b["kp_octave"], kp_uright=b["kp_uright"],
             kp_desc=b["kp_desc"], kp_angle=rng.uniform(0, 360, K).astype(np.float32), kp_claimed=b["kp_claimed"],
             bounds=b["bounds"], mp_begin=b["mp_begin"], mp_valid=b["mp_valid"], mp_proj=b["mp_proj"],
             mp_octave=np.minimum(b["mp_level"], 7).astype(np.int32), mp_desc=b["mp_desc"],
             mp_has_obs=b["mp_has_obs"], mp_angle=rng.uniform(0, 360, int(b["mp_begin"][-1])).astype(np.float32),
             motion=None, scale_factors=b["scale_factors"], th=7.0, check_orientation=True)
    g = {k: (torch.from_numpy(np.ascontiguousarray(v)).cuda() if isinstance(v, np.ndarray) and
             k not in ("scale_factors",) else v) for k, v in m.items()}
    kp_match = torch.full((K,), 12345, dtype=torch.int32, device="cuda")
    km, nm = search_by_projection_motion_device(g, kp_match=kp_match)
    torch.cuda.synchronize()
    assert int(nm[0]) == -1
    assert bool((km[:9000] == -1).all())
