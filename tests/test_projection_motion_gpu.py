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
