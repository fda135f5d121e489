"""Diagnostic: describe_kernel phase stamps (every 16th wavefront) with the ORB_DESC_STAMPS build."""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
os.environ["ORBSLAM2_AMD_LIB"] = str(ROOT / "tools" / "diag" / "liborbslam2_amd_descstamps.so")
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from orb_slam2_refactored_amd import ORBextractor  # noqa: E402
from orb_slam2_refactored_amd._lib import lib  # noqa: E402
from orb_slam2_refactored_amd.synth import synth_image  # noqa: E402

F = 128
kind = sys.argv[1] if len(sys.argv) > 1 else "pan"
if kind == "pan":
    from orb_slam2_refactored_amd.synth import pan_sequence
    pool = pan_sequence(0, 1280, 720, 16)
    frames = torch.from_numpy(np.stack([pool[i % 16] for i in range(F)])).cuda()
else:
    from orb_slam2_refactored_amd.synth import textured_image
    gen = textured_image if kind == "textured" else synth_image
    frames = torch.from_numpy(np.stack([gen(i % 16, 1280, 720) for i in range(F)])).cuda()
ex = ORBextractor(ORBextractor.Parameters(nfeatures=2000))
for _ in range(3):
    ex.extract_batch_device(frames)
torch.cuda.synchronize()
buf = (C.c_ulonglong * (64 + 8192))()
lib().orbx_debug_qt_stamps.argtypes = [C.c_void_p]
assert lib().orbx_debug_qt_stamps(C.cast(buf, C.c_void_p)) == 0
st = np.array(list(buf)[64:], dtype=np.int64).reshape(1024, 8)
st = st[(st[:, 0] > 0) & (st[:, 6] > 0)]
d = np.diff(st[:, :7], axis=1)
names = ["patch load+stage", "blur+angle+atan", "barrier", "sincos", "samples+ballots", "stores"]
print(f"{len(st)} sampled wavefronts; median ticks per phase:")
pre = st[:, 0] - st[:, 7]   # stamp 7: entry, before the keypoint-word / count load and the level lookup
print(f"  {'preamble (kp load)':18s} {int(np.median(pre)):8d}  (p90 {int(np.percentile(pre, 90))})")
for i, n in enumerate(names):
    print(f"  {n:18s} {int(np.median(d[:, i])):8d}  (p90 {int(np.percentile(d[:, i], 90))})")
print("  total", int(np.median(st[:, 6] - st[:, 7])))
