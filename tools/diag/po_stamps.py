"""Diagnostic: where PoseOptimization's cycles go (ORB_PO_STAMPS build), block 0 of one launch."""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
os.environ["ORBSLAM2_AMD_LIB"] = os.environ.get("PO_LIB", str(ROOT / "tools" / "diag" / "liborbslam2_amd_postamps.so"))
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402  (HIP initialised by torch first, as in bench.py)
torch.cuda.init()
from orb_slam2_refactored_amd._lib import lib  # noqa: E402
from orb_slam2_refactored_amd.optimizer import PoseOptimization  # noqa: E402
from orb_slam2_refactored_amd.synth import make_pose_batch  # noqa: E402

edges = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 256
b = make_pose_batch(12, n_frames=frames, n_edges=edges)
f = lib().orbba_debug_po_stamps
f.argtypes = [C.c_void_p]
buf = (C.c_ulonglong * 8)()
PoseOptimization(b)
assert f(C.cast(buf, C.c_void_p)) == 0   # reset
PoseOptimization(b)
assert f(C.cast(buf, C.c_void_p)) == 0
v = list(buf)
names = ["linearize pass", "reduce 28", "6x6 solve", "exp update", "chi pass+reduce", "classify/other"]
tot = sum(v[:6])
print(f"edges/frame {edges}: LM iterations {v[6]}, trials {v[7]}, total {tot} ticks")
for i, n in enumerate(names):
    per = v[i] / max(v[6] if i < 2 else v[7] if i < 5 else 1, 1)
    print(f"  {n:18s} {v[i]:9d} ticks {100.0 * v[i] / max(tot, 1):5.1f} %  per-call {per:8.0f}")

import numpy as np  # noqa: E402
from orb_slam2_refactored_amd.optimizer import pose_optimization_device  # noqa: E402
d = {k: torch.from_numpy(np.ascontiguousarray(x)).cuda() for k, x in b.items() if not k.startswith("gt_")}
o = pose_optimization_device(d)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    pose_optimization_device(d, out=o)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 10
print(f"  device launch (stamps build): {ms:.3f} ms for {frames} frames = {frames / ms * 1e3:.0f} frames/s")
