"""CPU: the oracle's CheckOrientation (a literal restatement with std::vector bins and libstdc++
std::sort) against an independent Python restatement (ORBmatcher.cc:249-309)."""
import numpy as np
import pytest

from orientation_case import make_case, reference_filter


@pytest.mark.parametrize("seed", range(24))
def test_oracle_check_orientation(oracle, seed):
    angA, angB, match = make_case(seed, nA=50 + 37 * seed, nB=300)
    got, n = oracle.check_orientation(angA, angB, match)
    exp, ne = reference_filter(angA, angB, match, oracle.std_sort_perm)
    assert np.array_equal(got, exp)
    assert n == ne


def test_oracle_check_orientation_edges(oracle):
    # no match at all; a single match; everything in one bin (eraseBin = 1)
    for m in (np.full(10, -1, np.int32), np.array([3, -1], np.int32), np.arange(40, dtype=np.int32)):
        angA = np.full(len(m), 10.0, np.float32)
        angB = np.full(64, 40.0, np.float32)
        got, n = oracle.check_orientation(angA, angB, m)
        assert np.array_equal(got, m) and n == int((m >= 0).sum())
    # bin sizes 11 / 1 / 1: the second bin < 10 % of the first -> only the largest bin survives;
    # at 10 / 1 / 1 (1 < 1.0 is false) all three survive
    for big, keep in ((11, 11), (10, 12)):
        angA = np.zeros(big + 2, np.float32)
        angB = np.array([0.0] * big + [90.0, 180.0], np.float32)
        got, n = oracle.check_orientation(angA, angB, np.arange(big + 2, dtype=np.int32))
        assert n == keep and (got[:big] >= 0).all() and ((got[big:] == -1).all() if keep == big else (got >= 0).all())
