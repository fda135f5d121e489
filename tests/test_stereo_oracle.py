"""CPU checks of the ComputeStereoMatches restatement (oracle/orb_oracle.cpp) on the C3 synthetic
stereo pair: the reference has no fixtures for this path (parity unpinned), so the restatement
is checked against the scene it is run on — matched depths fall on the warped band depths."""
import numpy as np

from orb_slam2_refactored_amd.synth import KITTI, STEREO_Z, stereo_pair

BASELINE = KITTI["bf"] / KITTI["fx"]


def test_stereo_oracle_recovers_band_depths(oracle):
    L, R, zcol = stereo_pair(3)
    p = oracle.params(2000)
    t = oracle.scale_tables(p)
    scale, inv = t["scale"], t["inv_scale"]
    kl, dl, _ = oracle.extract(p, L)
    kr, dr, _ = oracle.extract(p, R)
    ur, depth = oracle.compute_stereo_matches(kl, dl, oracle.pyramid(p, L), kr, dr, oracle.pyramid(p, R), scale, inv,
                                              KITTI["bf"], BASELINE)
    m = depth > 0
    assert m.sum() > 0.3 * len(kl), m.sum()
    # true depth of a left keypoint: the band of its right-image column x - d
    good = 0
    for i in np.nonzero(m)[0]:
        xr = ur[i]
        z = zcol[int(np.clip(round(float(xr)), 0, len(zcol) - 1))]
        good += abs(depth[i] - z) < 0.15 * z
    assert good > 0.8 * m.sum(), (good, m.sum())
    # unmatched entries are exactly -1 in both outputs
    assert np.all((ur == -1) == (depth == -1))


def test_stereo_oracle_no_right_keypoints(oracle):
    L, _, _ = stereo_pair(4, 320, 240)
    p = oracle.params(500)
    t = oracle.scale_tables(p)
    scale, inv = t["scale"], t["inv_scale"]
    kl, dl, _ = oracle.extract(p, L)
    pyr = oracle.pyramid(p, L)
    ur, depth = oracle.compute_stereo_matches(kl, dl, pyr, kl[:0], dl[:0], pyr, scale, inv, KITTI["bf"], BASELINE)
    assert np.all(ur == -1) and np.all(depth == -1)
