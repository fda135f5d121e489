"""Diagnostic: s_memtime stamps of sampled FAST waves (ORB_FAST_STAMPS build): 0 wave start, 1 first\ncrop in LDS, 2 first item done, 5 wave end; 6 first item level/corners; 7 items in the wave."""
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
from orb_slam2_refactored_amd.synth import synth_image, textured_image  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 128
kind = sys.argv[2] if len(sys.argv) > 2 else "g"
if kind == "pan":
    from orb_slam2_refactored_amd.synth import pan_sequence
    pool = pan_sequence(0, 1280, 720, 16)
    frames = torch.from_numpy(np.stack([pool[i % 16] for i in range(F)])).cuda()
else:
    gen = textured_image if kind == "textured" else synth_image
    frames = torch.from_numpy(np.stack([gen(i % 16, 1280, 720) for i in range(F)])).cuda()
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
t = a[:, :6] - a[:, :1]
lvl = (a[:, 6] >> 48) & 0xffff
nc = (a[:, 6] >> 16) & 0xffffffff
nit = a[:, 7]
print(f"sampled waves {len(a)}, items/wave {nit.mean():.2f}, mean wave life {t[:, 5].mean():.0f} ticks")
print(f"first crop (unhidden load) {t[:, 1].mean():.0f}, first item body {np.mean(t[:, 2] - t[:, 1]):.0f}")
m = nit > 1
if m.any():
    print(f"later items: {np.mean((t[m, 5] - t[m, 2]) / (nit[m] - 1)):.0f} ticks per item (crop prefetched)")
for L in range(int(lvl.max()) + 1):
    k = lvl == L
    if k.any():
        print(f"level {L}: n {k.sum():5d} corners {nc[k].mean():6.1f} crop {t[k, 1].mean():7.0f} body {np.mean(t[k, 2] - t[k, 1]):7.0f}"
              f" (pretest+strength {np.mean(t[k, 3] - t[k, 1]):7.0f} nms {np.mean(t[k, 4] - t[k, 3]):6.0f} emit {np.mean(t[k, 2] - t[k, 4]):6.0f})")
