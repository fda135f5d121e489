#!/usr/bin/env python3
"""LocalBA timing driver (C4: 20 KF x 3000 MP): GPU calls/s and LM iterations/s."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from orb_slam2_refactored_amd.optimizer import LocalBundleAdjustment  # noqa: E402
from orb_slam2_refactored_amd.synth import make_ba_problem  # noqa: E402

pr = make_ba_problem(0)
LocalBundleAdjustment(pr)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
t = time.perf_counter()
it = 0
for _ in range(n):
    r = LocalBundleAdjustment(pr)
    it += sum(r["iterations"])
dt = time.perf_counter() - t
print(f"LocalBA {1e3 * dt / n:.3f} ms/call, {it / dt:.0f} LM iters/s, iterations {r['iterations']}")
