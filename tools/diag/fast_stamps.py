"""Diagnostic: per-phase s_memtime stamps of sampled FAST waves (ORB_FAST_STAMPS build).
Phases: 0 start, 1 crop in LDS, 2 compass + full tests, 3 strengths, 4 NMS, 5 end."""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
os.environ["ORBSLAM2_AMD_LIB"] = str(ROOT / "tools" / "diag" / "liborbslam2_amd_faststamps.so")
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from orb_slam2_refactored_amd import ORBextractor  # noqa: E402
from orb_slam2_refactored_amd._lib import lib  # noqa: E402
from orb_slam2_refactored_amd.synth import synth_image  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 128
frames = torch.from_numpy(np.stack([synth_image(i % 16, 1280, 720) for i in range(F)])).cuda()
ex = ORBextractor(ORBextractor.Parameters(nfeatures=2000))
for _ in range(3):
    ex.extract_batch_device(frames)
torch.cuda.synchronize()
N = 8192
buf = (C.c_ulonglong * (N * 8))()
fn = lib().orbx_debug_fast_stamps
fn.argtypes = [C.c_void_p, C.c_int]
assert fn(C.cast(buf, C.c_void_p), N * 8) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(N, 8).astype(np.int64)
a = a[a[:, 5] > 0]
t = a[:, :6] - a[:, :1].min()
lvl = (a[:, 6] >> 48) & 0xffff
nc = (a[:, 6] >> 16) & 0xffffffff
span = t[:, 5].max() - t[:, 0].min()
print(f"sampled waves {len(a)}, kernel span {span} ticks, mean wave life {np.mean(t[:, 5] - t[:, 0]):.0f}")
names = ["crop", "compass+full", "strength", "nms", "emit"]
for L in range(int(lvl.max()) + 1):
    m = lvl == L
    if not m.any():
        continue
    d = np.diff(t[m], axis=1).mean(axis=0)
    print(f"level {L}: n {m.sum():5d} corners {nc[m].mean():6.1f} " + " ".join(f"{k} {v:7.0f}" for k, v in zip(names, d)))
d = np.diff(t, axis=1).mean(axis=0)
print("all     : " + " ".join(f"{k} {v:7.0f}" for k, v in zip(names, d)))
# concurrency: waves alive over time
ts = np.sort(t[:, 0]); te = np.sort(t[:, 5])
grid = np.linspace(0, span, 20)
alive = [(np.searchsorted(ts, x) - np.searchsorted(te, x)) * 64 for x in grid]
print("est. waves alive over kernel (x64 sampling):", [int(v) for v in alive])
