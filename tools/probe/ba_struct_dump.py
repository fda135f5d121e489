#!/usr/bin/env python3
"""Dumps the C4 LocalBA graph (20 KF x 3000 MP, bench.py's localba leg) for tools/probe/ba_struct_bench."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from orb_slam2_refactored_amd.synth import make_ba_problem  # noqa: E402

p = make_ba_problem(0, n_kf=20, n_pts=3000, n_fixed=2)
out = sys.argv[1] if len(sys.argv) > 1 else "/tmp/c4_graph.bin"
with open(out, "wb") as f:
    np.array([len(p["pose_fixed"]), len(p["points"]), len(p["edge_point"])], np.int32).tofile(f)
    p["pose_fixed"].astype(np.uint8).tofile(f)
    p["edge_point"].astype(np.int32).tofile(f)
    p["edge_pose"].astype(np.int32).tofile(f)
print(out)
