import sys; sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import numpy as np
from orb_slam2_refactored_amd import ORBmatcher
from conftest import *  # noqa
import importlib
def rand_desc(rng, n, p=0.5):
    bits = (rng.random((n, 256)) < p).astype(np.uint8)
    return np.packbits(bits, axis=1, bitorder="little")
def hd(a, b):
    return int(np.unpackbits(a ^ b).sum())
for nA, nB in [(257, 513), (2000, 2000), (64, 255), (300, 40)]:
    rng = np.random.default_rng(nA * 7 + nB)
    A = rand_desc(rng, nA); B = rand_desc(rng, nB)
    if nB > 10:
        B[7] = B[3]; A[: min(nA, 5)] = B[3] ^ np.uint8(1)
    bi, bd, sd, m = ORBmatcher(0.6, False).MatchBruteForce(A, B)
    D = np.array([[hd(A[i], B[j]) for j in range(nB)] for i in range(min(nA, 300))])
    eb = D.min(1); ei = D.argmin(1)
    es = np.array([np.sort(r)[1] if len(r) > 1 else 256 for r in D])
    n = len(eb)
    bad = np.nonzero((bd[:n] != eb) | (bi[:n] != ei) | (sd[:n] != es))[0]
    print(nA, nB, "bad rows", len(bad), bad[:10])
    for i in bad[:5]:
        print(i, "got", bi[i], bd[i], sd[i], "exp", ei[i], eb[i], es[i], "D at got", D[i, bi[i]] if bi[i] >= 0 else None)
