"""The quadtree's std::sort emulation (orb_slam2_refactored_amd/csrc/qt_sort.h) against the real
libstdc++ std::sort: the sequential port and the data-parallel formulation (CPU, native harness),
and the on-device wavefront version (GPU)."""
import ctypes as C
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


def test_qt_sort_native(tmp_path):
    exe = tmp_path / "qtsc"
    subprocess.run(["g++", "-O2", "-std=c++14", f"-I{ROOT / 'orb_slam2_refactored_amd' / 'csrc'}",
                    str(ROOT / "tests" / "native" / "qt_sort_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "6000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.startswith("OK"), out.stdout + out.stderr


def test_oracle_sort_matches_argsort_order(oracle):
    sizes = np.array([3, 7, 7, 2, 9, 7, 3], np.int32)
    perm = oracle.std_sort_perm(sizes)
    assert np.all(np.diff(sizes[perm]) <= 0)
    assert sorted(perm.tolist()) == list(range(len(sizes)))


@pytest.mark.gpu
def test_device_wave_sort_matches_std_sort(oracle):
    from orb_slam2_refactored_amd._lib import lib, ptr
    rng = np.random.default_rng(1)
    for case in range(300):
        n = int(rng.integers(0, 40 if case % 3 else 1500))
        sizes = rng.integers(2, 2 + int(rng.integers(1, 30)), n).astype(np.int32)
        if case % 11 == 0:
            sizes = np.sort(sizes)
        exp = oracle.std_sort_perm(sizes)
        got = np.zeros(n, np.int32)
        assert lib().orbx_debug_qt_sort(ptr(sizes), n, ptr(got)) == 0
        assert np.array_equal(got, exp), case
