"""Diagnostic: phase stamps of the LocalBA solve kernel (ORB_BA_STAMPS build), last launch."""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
os.environ["ORBSLAM2_AMD_LIB"] = str(ROOT / "tools" / "diag" / "liborbslam2_amd_bastamps.so")
sys.path.insert(0, str(ROOT))
from orb_slam2_refactored_amd._lib import lib  # noqa: E402
from orb_slam2_refactored_amd.optimizer import LocalBundleAdjustment  # noqa: E402
from orb_slam2_refactored_amd.synth import make_ba_problem  # noqa: E402

pr = make_ba_problem(0)
for _ in range(3):
    LocalBundleAdjustment(pr)
buf = (C.c_ulonglong * 64)()
f = lib().orbba_debug_stamps
f.argtypes = [C.c_void_p]
assert f(C.cast(buf, C.c_void_p)) == 0
v = list(buf)
t0 = v[0]
prev = t0
last = t0
for blk in range(16):
    a, b_, c = v[1 + 3 * blk], v[2 + 3 * blk], v[3 + 3 * blk]
    if a == 0 or a < t0:
        break
    line = f"block {blk}: diag-wait {a - prev:6d}"
    if b_ >= a:
        line += f" panel {b_ - a:6d}"
        last = b_
    if c >= b_ >= a:
        line += f" lookahead(trailing+diag) {c - b_:6d}"
        last = c
    print(line)
    prev = last
print(f"back-substitution {v[40] - last}, total {v[40] - t0} ticks; block 0 staged by wavefront 0 {v[0] - v[41]} "
      f"(block 0's diag-wait = its factorisation beside the other wavefronts' load of S), pose update tail {v[42] - v[40]}")
b2 = v[2 + 3 * 2]   # block 2 panel end = start of its lookahead phase
if v[44] > b2:
    print(f"block 2 lookahead by wave: w0 trailing tile {v[44] - b2}, w0 diag factor {v[45] - v[44]} (ends {v[45] - b2}), "
          f"w1 inverse ends {v[46] - b2}, w2 tiles end {v[47] - b2}, w3 tiles end {v[48] - b2}")
