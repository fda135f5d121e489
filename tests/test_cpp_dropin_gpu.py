"""Runs the C++ drop-in classes (include/orbslam2_amd.hpp: ORBextractor::Extract, ORBmatcher with
checkOri, LocalBundleAdjustment, ComputeStereoMatches on two extractors) — the boundary the reference would link — on the GPU through
tests/native/cpp_dropin_main.cpp (built by __graft_entry__.build()), and compares their outputs with
the committed golden fixtures and the oracle."""
import subprocess
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
EXE = ROOT / "tests" / "native" / "_build" / "cpp_dropin"
GOLDEN = ROOT / "tests" / "golden"


def run(mode, d):
    assert EXE.exists(), "build the drop-in driver with __graft_entry__.build()"
    r = subprocess.run([str(EXE), mode, str(d)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_cpp_extract_matches_golden(tmp_path, seed):
    g = np.load(GOLDEN / f"extract_c1_seed{seed}.npz")
    img = g["image"]
    img.tofile(tmp_path / "image.u8")
    np.array([img.shape[0], img.shape[1], int(g["nfeatures"])], np.int32).tofile(tmp_path / "meta.i32")
    run("extract", tmp_path)
    n = int(np.fromfile(tmp_path / "n.i32", np.int32)[0])
    kps = np.fromfile(tmp_path / "kps.i32", np.int32).reshape(n, 7)
    desc = np.fromfile(tmp_path / "desc.u8", np.uint8).reshape(n, 32)
    assert np.array_equal(kps, g["kps"]) and np.array_equal(desc, g["desc"])


@pytest.mark.parametrize("check_ori", [0, 1])
def test_cpp_matcher_check_orientation(tmp_path, oracle, check_ori):
    a = np.load(GOLDEN / "extract_c1_seed0.npz")
    b = np.load(GOLDEN / "extract_c1_seed1.npz")
    A, B = a["desc"], b["desc"]
    angA = a["kps"].view(np.float32)[:, 3].copy()
    angB = b["kps"].view(np.float32)[:, 3].copy()
    A.tofile(tmp_path / "A.u8")
    B.tofile(tmp_path / "B.u8")
    angA.tofile(tmp_path / "angA.f32")
    angB.tofile(tmp_path / "angB.f32")
    np.array([len(A), len(B), check_ori], np.int32).tofile(tmp_path / "meta.i32")
    run("match", tmp_path)
    got = np.fromfile(tmp_path / "match.i32", np.int32)
    n = int(np.fromfile(tmp_path / "n.i32", np.int32)[0])
    _, _, _, exp = oracle.bf_match(A, B)
    ne = int((exp >= 0).sum())
    if check_ori:
        exp, ne = oracle.check_orientation(angA, angB, exp)
    assert np.array_equal(got, exp) and n == ne


def _write_ba(d, pr, stop=0):
    P, N, E = len(pr["pose_R"]), len(pr["points"]), len(pr["edge_point"])
    np.array([P, N, E, stop], np.int32).tofile(d / "meta.i32")
    for k, dt, ext in (("pose_R", np.float64, "f64"), ("pose_t", np.float64, "f64"), ("pose_fixed", np.uint8, "u8"),
                       ("points", np.float64, "f64"), ("edge_point", np.int32, "i32"), ("edge_pose", np.int32, "i32"),
                       ("edge_obs", np.float64, "f64"), ("edge_inv_sigma2", np.float64, "f64"),
                       ("edge_cam", np.float64, "f64")):
        np.ascontiguousarray(pr[k], dt).tofile(d / f"{k}.{ext}")


@pytest.mark.parametrize("mode", ["localba", "localba_twice"])
def test_cpp_local_ba_matches_golden(tmp_path, mode):
    z = np.load(GOLDEN / "local_ba_small.npz")
    pr = {k: z[k] for k in z.files if not k.startswith("out_")}
    _write_ba(tmp_path, pr)
    run(mode, tmp_path)
    P = len(pr["pose_R"])
    t = np.fromfile(tmp_path / "out_pose_t.f64").reshape(P, 3)
    outl = np.fromfile(tmp_path / "out_outlier.u8", np.uint8)
    it = np.fromfile(tmp_path / "out_iterations.i32", np.int32)
    assert np.sqrt(np.mean((t - z["out_pose_t"]) ** 2)) < 1e-4
    assert np.array_equal(outl, z["out_outlier"])
    assert tuple(it) == tuple(z["out_iterations"])
    assert int(np.fromfile(tmp_path / "out_ran.i32", np.int32)[0]) == 1


def test_cpp_stereo_two_threads(tmp_path, oracle):
    """The reference's stereo call shape in C++ (System.cc:449-461): Extract L and R on two std::threads,
    then ComputeStereoMatches on the two extractors (orbx_stereo_matches_last); uright / depth bit-identical
    to the oracle's ComputeStereoMatches on its own extraction and pyramids."""
    from orb_slam2_refactored_amd.synth import KITTI, stereo_pair
    L, R, _ = stereo_pair(0, 1242, 375)
    bf, baseline = np.float32(KITTI["bf"]), np.float32(KITTI["bf"] / KITTI["fx"])
    L.tofile(tmp_path / "left.u8")
    R.tofile(tmp_path / "right.u8")
    np.array([L.shape[0], L.shape[1], 2000], np.int32).tofile(tmp_path / "meta.i32")
    np.array([bf, baseline], np.float32).tofile(tmp_path / "cam.f32")
    run("stereo", tmp_path)
    got_u = np.fromfile(tmp_path / "uright.f32", np.float32)
    got_d = np.fromfile(tmp_path / "depth.f32", np.float32)
    p = oracle.params(2000)
    t = oracle.scale_tables(p)
    kl, dl, _ = oracle.extract(p, L)
    kr, dr, _ = oracle.extract(p, R)
    exp_u, exp_d = oracle.compute_stereo_matches(kl, dl, oracle.pyramid(p, L), kr, dr, oracle.pyramid(p, R), t["scale"],
                                                 t["inv_scale"], float(bf), float(baseline))
    assert int(np.fromfile(tmp_path / "nL.i32", np.int32)[0]) == len(kl)
    assert (exp_d > 0).sum() > 0.3 * len(kl)
    assert np.array_equal(got_u.view(np.int32), exp_u.view(np.int32))
    assert np.array_equal(got_d.view(np.int32), exp_d.view(np.int32))


def test_cpp_local_ba_stop_on_entry(tmp_path):
    z = np.load(GOLDEN / "local_ba_small.npz")
    pr = {k: z[k] for k in z.files if not k.startswith("out_")}
    _write_ba(tmp_path, pr, stop=1)
    run("localba", tmp_path)
    assert int(np.fromfile(tmp_path / "out_ran.i32", np.int32)[0]) == 0
    assert tuple(np.fromfile(tmp_path / "out_iterations.i32", np.int32)) == (0, 0)
