"""GPU FeaturesGrid + SearchByProjection (orbm_search_by_projection*, ORBmatcher.cc:315-382) vs the
oracle: kp_match (which map point each keypoint got) and n_matches bit-identical."""
import numpy as np
import pytest

from orb_slam2_refactored_amd._lib import OrbError
from orb_slam2_refactored_amd.matcher import SearchByProjection, search_by_projection_device
from orb_slam2_refactored_amd.synth import make_proj_batch

pytestmark = pytest.mark.gpu


def _check(b, oracle):
    km, n = SearchByProjection(b)
    okm, on = oracle.search_by_projection(b)
    assert np.array_equal(n, on), (n, on)
    assert np.array_equal(km, okm)
    return km, n


@pytest.mark.parametrize("kw", [
    dict(seed=0),
    dict(seed=1, th=3.0),
    dict(seed=2, th=5.0, odd_bounds=True),
    dict(seed=3, dup_frac=0.7),                       # many claim conflicts -> K exhausted -> rescans
    dict(seed=4, th=5.0, dup_frac=0.9, n_kp=600),     # dense conflicts in big windows
    dict(seed=5, n_kp=[0, 10, 2000, 3000], n_mp=[50, 0, 1500, 2500]),
])
def test_search_by_projection_matches_oracle(oracle, kw):
    kw = dict(dict(n_frames=4, n_kp=2000, n_mp=1500), **kw)
    _check(make_proj_batch(**kw), oracle)


def test_search_by_projection_all_claimed_and_no_claims(oracle):
    b = make_proj_batch(6, n_frames=2, n_kp=800, n_mp=600)
    b["kp_claimed"][:] = 1
    km, n = _check(b, oracle)
    assert list(n) == [0, 0] and (km == -1).all()
    b["kp_claimed"] = None
    _check(b, oracle)


def test_search_by_projection_max_keypoints(oracle):
    b = make_proj_batch(7, n_frames=2, n_kp=[8192, 100], n_mp=[3000, 50])
    _check(b, oracle)
    big = make_proj_batch(8, n_frames=1, n_kp=8193, n_mp=20)
    with pytest.raises(OrbError):
        SearchByProjection(big)


def _to_dev(b):
    import torch
    return {k: (torch.from_numpy(np.ascontiguousarray(v)).cuda() if isinstance(v, np.ndarray) and k != "scale_factors"
                else v) for k, v in b.items()}


def test_search_by_projection_device_matches_host():
    import torch
    b = make_proj_batch(9, n_frames=8, n_kp=2000, n_mp=1500, th=3.0)
    km, n = SearchByProjection(b)
    d = _to_dev(b)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        dk, dn = search_by_projection_device(d, stream=s)
        dk2, dn2 = search_by_projection_device(d, stream=s)
    s.synchronize()
    assert np.array_equal(dk.cpu().numpy(), km) and np.array_equal(dn.cpu().numpy(), n)
    assert torch.equal(dk, dk2) and torch.equal(dn, dn2)


def test_search_by_projection_device_oversized_frame():
    import torch
    b = make_proj_batch(10, n_frames=2, n_kp=[8193, 300], n_mp=[10, 200])
    dk, dn = search_by_projection_device(_to_dev(b))
    torch.cuda.synchronize()
    n = dn.cpu().numpy()
    assert n[0] == -1 and n[1] >= 0
    assert (dk.cpu().numpy()[:8193] == -1).all()
