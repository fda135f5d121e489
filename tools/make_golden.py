#!/usr/bin/env python3
"""Regenerate the committed golden fixtures (tests/golden/*.npz) from the CPU oracle.

The reference ships no tests, fixtures or golden vectors and cannot be built here, so
these fixtures are oracle outputs on seeded synthetic inputs: they freeze the oracle's behaviour
(regression guard) and give the GPU tests inputs/outputs that do not need the oracle at run time.
Inputs are regenerated from their seeds by orb_slam2_refactored_amd.synth (numpy PCG64), and also
stored so that a change of the generator is detected.
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import oracle_api as O  # noqa: E402
from orb_slam2_refactored_amd.synth import make_ba_problem, make_pose_batch, synth_image  # noqa: E402

OUT = ROOT / "tests" / "golden"


def pose_opt():
    # PoseOptimization: ragged batch incl. the < 3 / < 10 edge cases
    b = make_pose_batch(6, n_frames=6, n_edges=[0, 2, 7, 60, 300, 900])
    r = O.pose_optimization(b)
    keep = {k: v for k, v in b.items() if not k.startswith("gt_")}
    np.savez_compressed(OUT / "pose_opt_small.npz", **keep, out_pose_R=r["pose_R"], out_pose_t=r["pose_t"],
                        out_n_inliers=r["n_inliers"], out_outlier=r["outlier"])


def main(only=None):
    OUT.mkdir(parents=True, exist_ok=True)
    if only == "pose":
        pose_opt()
        return
    pose_opt()
    trig, simd = O.set_compat()   # the OpenCV-build switches the fixtures were made with (defaults)
    for seed in range(4):
        img = synth_image(seed, 640, 480)
        kps, desc, per = O.extract(O.params(1000), img)
        np.savez_compressed(OUT / f"extract_c1_seed{seed}.npz", seed=seed, width=640, height=480, nfeatures=1000,
                            image=img, kps=kps.view(np.int32).reshape(-1, 7), desc=desc, per_level=per,
                            trig=trig, resize_simd=simd)
    # matcher: descriptors of two C1 frames
    d0 = np.load(OUT / "extract_c1_seed0.npz")["desc"]
    d1 = np.load(OUT / "extract_c1_seed1.npz")["desc"]
    bi, bd, sd, m = O.bf_match(d0, d1)
    np.savez_compressed(OUT / "bf_match_c1.npz", A=d0, B=d1, best_idx=bi, best=bd, second=sd, match=m)
    # LocalBA, small problem (full C4 is regenerated from its seed in the tests)
    pr = make_ba_problem(5, n_kf=8, n_pts=400, n_fixed=1)
    r = O.local_ba(pr)
    keep = {k: v for k, v in pr.items() if not k.startswith("gt_")}
    np.savez_compressed(OUT / "local_ba_small.npz", **keep, out_pose_R=r["pose_R"], out_pose_t=r["pose_t"],
                        out_points=r["points"], out_outlier=r["edge_outlier"],
                        out_iterations=np.array(r["iterations"]), out_chi2=np.array(r["chi2"]))
    for p in sorted(OUT.glob("*.npz")):
        print(p.name, p.stat().st_size)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)   # "pose": only the PoseOptimization fixture
