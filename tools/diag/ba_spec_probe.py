"""Diagnostic: which LocalBA loop ends were enqueued ahead and used, over tests/test_ba_gpu.py's loop-end cases."""
import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), 'tests'))
os.environ["ORBBA_DEBUG_TIMING"] = "1"
import test_ba_gpu as T
from orb_slam2_refactored_amd.optimizer import LocalBundleAdjustment
for c in T._LOOP_END_CASES:
    print(c, flush=True)
    r = LocalBundleAdjustment(T._loop_end_problem(*c))
