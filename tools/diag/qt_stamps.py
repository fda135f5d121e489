"""Diagnostic: quadtree phase stamps of (frame 0, level 0) with the ORB_QT_STAMPS build."""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
# QT_STAMPS_LIB: a build with -DQT_STAMP_LEVEL=<l> stamps level l's frame-0 workgroup instead of level 0's
os.environ["ORBSLAM2_AMD_LIB"] = os.environ.get("QT_STAMPS_LIB", str(ROOT / "tools" / "diag" / "liborbslam2_amd_stamps.so"))
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from orb_slam2_refactored_amd import ORBextractor  # noqa: E402
from orb_slam2_refactored_amd._lib import lib  # noqa: E402
from orb_slam2_refactored_amd.synth import synth_image, textured_image  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 128
gen = textured_image if len(sys.argv) > 2 and sys.argv[2] == "textured" else synth_image
frames = torch.from_numpy(np.stack([gen(i % 16, 1280, 720) for i in range(F)])).cuda()
ex = ORBextractor(ORBextractor.Parameters(nfeatures=2000))
for _ in range(3):
    ex.extract_batch_device(frames)
torch.cuda.synchronize()
buf = (C.c_ulonglong * (64 + 8192))()
lib().orbx_debug_qt_stamps.argtypes = [C.c_void_p]
assert lib().orbx_debug_qt_stamps(C.cast(buf, C.c_void_p)) == 0
v = list(buf)
t0 = v[0]
print("gather", v[1] - t0, "roots", v[2] - v[1])
i = 0
prev = v[2]
while 3 + 2 * i < 63 and v[3 + 2 * i] > 0 and 4 + 2 * i < 64:
    st = v[4 + 2 * i]
    print(f"iter {i}: state {st >> 32} n {st & 0xffffffff} t {v[3 + 2 * i] - t0} (+{v[3 + 2 * i] - prev})")
    prev = v[3 + 2 * i]
    if (st >> 32) == 2:
        break
    i += 1
print("end", v[63] - t0, "(+", v[63] - prev, ")   [s_memtime ticks]")

# g_qt_wg holds 4096 (frame, level) workgroups: frames past 4096 / 8 = 512 are not recorded
Fw = min(F, 4096 // 8)
wg = np.array(list(buf)[64:64 + 2 * Fw * 8], dtype=np.int64).reshape(Fw, 8, 2)
dur = wg[:, :, 1] - wg[:, :, 0]
for l in range(8):
    print(f"level {l}: WG ticks mean {dur[:, l].mean():8.0f} max {dur[:, l].max():8.0f}")

for r in range(3):
    a = list(buf)[40 + 4 * r:44 + 4 * r]
    if a[0] and a[3] > a[0]:
        print(f"phase-2 round {r}: sort {a[1] - a[0]} counts+stop {a[2] - a[1]} split+emit {a[3] - a[2]}")

SUB = int(os.environ.get("QT_SUB_ITER", "5"))   # the build's -DQT_SUB_ITER (sub-phase stamps 55-59)
if v[56] and v[59] > v[3 + 2 * SUB]:
    b = v[3 + 2 * SUB]
    print(f"phase-1 pass {SUB} sub-phases: compaction {v[56] - b} split {v[57] - v[56]} "
          f"emit (thread 0) {v[55] - v[57]} copy+commit {v[58] - v[55]} state {v[59] - v[58]}")
