"""Does the i8 matcher kernel (ORBM_FP4=0, hamming_top2_mfma_kernel), whose listing has the LDS-load-over-
MFMA-source pattern of the nondeterministic describe builds (tools/mfma_raw_check.py), give results that
differ from the FP4 kernel (exact; no such pattern) or between identical runs?  Random descriptors,
65536 query rows x 2048 / 4500 train rows, repeated."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from orb_slam2_refactored_amd.matcher import ORBmatcher  # noqa: E402

REPS = int(os.environ.get("WAR_REPS", 6))
rng = np.random.default_rng(7)
bad = 0
for nA, nB in ((65536, 2048), (16384, 4500)):
    A = rng.integers(0, 256, (nA, 32), dtype=np.uint8)
    B = rng.integers(0, 256, (nB, 32), dtype=np.uint8)
    B[100:140] = A[:40] ^ np.uint8(1)   # near matches
    os.environ["ORBM_FP4"] = "1"
    ref = ORBmatcher(0.6, False).MatchBruteForce(A, B)
    os.environ["ORBM_FP4"] = "0"
    for r in range(REPS):
        got = ORBmatcher(0.6, False).MatchBruteForce(A, B)
        nd = sum(int(np.count_nonzero(np.asarray(g) != np.asarray(e))) for g, e in zip(got, ref))
        bad += nd
        print(f"nA={nA} nB={nB} rep {r}: {nd} elements differ from the FP4 kernel", flush=True)
print("differences:", bad)
sys.exit(1 if bad else 0)
