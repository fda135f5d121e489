"""SearchByProjection(Frame&, KeyFrame*, alreadyFound, th, ORBdist) (src/ORBmatcher.cc:1364-1445,
Tracking::Relocalization) on the device against the oracle's literal restatement (pinned by
tests/test_projection_reloc_oracle.py): identical kp_match and match counts through the host and the
batched device entries, for both calls of Tracking.cc:403,417 (th 10 / ORBdist 100, th 3 / ORBdist
64), with and without CheckOrientation, keypoints shared by several points (claims made during the
call), entry claims, invariance-gate rejections, empty and over-limit frames."""
import numpy as np
import pytest

from orb_slam2_refactored_amd.matcher import SearchByProjectionReloc, search_by_projection_reloc_device
from orb_slam2_refactored_amd.synth import make_reloc_batch

pytestmark = pytest.mark.gpu


def _device(b, kp_match=None):
    import torch
    g = {k: (torch.from_numpy(np.ascontiguousarray(v)).cuda() if isinstance(v, np.ndarray) and k != "scale_factors"
             else v) for k, v in b.items()}
    km, nm = search_by_projection_reloc_device(g, kp_match=kp_match)
    torch.cuda.synchronize()
    K, F = int(b["kp_begin"][-1]), len(b["kp_begin"]) - 1
    return km.cpu().numpy()[:K], nm.cpu().numpy()[:F]


def _check(oracle, b):
    exp, en = oracle.search_by_projection_reloc(b)
    got, gn = _device(b)
    assert np.array_equal(got, exp)
    assert np.array_equal(gn, en)
    hm, hn = SearchByProjectionReloc(b)
    assert np.array_equal(hm, exp) and np.array_equal(hn, en)
    return en


@pytest.mark.parametrize("th,orb", [(10.0, 100), (3.0, 64)])
@pytest.mark.parametrize("check_ori", [True, False])
def test_reloc_vs_oracle(oracle, th, orb, check_ori):
    b = make_reloc_batch(int(th) * 7 + orb + int(check_ori), n_frames=6, n_kp=[2000, 1500, 2500, 800, 2000, 0],
                         n_mp=[600, 500, 900, 300, 0, 200], th=th, orb_dist=orb, check_orientation=check_ori)
    en = _check(oracle, b)
    assert en[:4].min() > 10


def test_reloc_heavy_sharing_no_claims(oracle):
    b = make_reloc_batch(77, n_frames=4, n_kp=1200, n_mp=800, dup_frac=0.6, claimed_frac=0.0)
    b["kp_claimed"] = None
    _check(oracle, b)


def test_reloc_over_limit_frame():
    b = make_reloc_batch(88, n_frames=2, n_kp=[9000, 500], n_mp=[100, 100])
    import torch
    km, nm = _device(b, kp_match=torch.full((9500,), 12345, dtype=torch.int32, device="cuda"))
    assert nm[0] == -1 and (km[:9000] == -1).all()
