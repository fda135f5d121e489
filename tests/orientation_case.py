"""Shared inputs for the CheckOrientation tests (ORBmatcher.cc:249-309): query-indexed matches with
keypoint angles chosen so the 30-bin rotation histogram has many equal-size bins (the unstable
std::sort then decides which bins survive) and rotation differences on exact bin boundaries."""
import numpy as np

# rotation differences that land exactly on cvRound half-way points (15 deg -> 0.5 -> 0, 45 -> 1.5 -> 2,
# 345 -> 11.5 -> 12), near the wrap (359.99 -> 12) and negative differences (+360)
EDGE_DIFFS = np.array([0.0, 15.0, 45.0, 75.0, 345.0, 359.99, 14.999, 15.001, 30.0, 180.0, 195.0], np.float32)


def make_case(seed, nA=400, nB=500, match_frac=0.6):
    rng = np.random.default_rng(seed)
    match = np.where(rng.random(nA) < match_frac, rng.integers(0, nB, nA), -1).astype(np.int32)
    angA = rng.uniform(0, 360, nA).astype(np.float32)
    angB = np.zeros(nB, np.float32)
    # target rotation per match drawn from a few bins with tied populations
    mode = seed % 4
    if mode == 0:      # uniform: many small equal bins
        rot = rng.uniform(0, 360, nB).astype(np.float32)
    elif mode == 1:    # one dominant bin
        rot = np.where(rng.random(nB) < 0.9, 60.0, rng.uniform(0, 360, nB)).astype(np.float32)
    elif mode == 2:    # three bins of equal weight + noise
        rot = rng.choice(np.array([30.0, 90.0, 300.0], np.float32), nB)
        rot = np.where(rng.random(nB) < 0.2, rng.uniform(0, 360, nB), rot).astype(np.float32)
    else:              # exact boundary differences
        rot = rng.choice(EDGE_DIFFS, nB)
    # angB[j] - angA[i] = rot for the query that matches j (other B angles random)
    angB[:] = rng.uniform(0, 360, nB)
    for i in np.nonzero(match >= 0)[0]:
        j = match[i]
        v = np.float32(angA[i] + rot[j])
        if v >= 360:
            v = np.float32(v - 360)
        angB[j] = v
    return angA, angB, match


def reference_filter(angA, angB, match, std_sort_perm):
    """Literal Python restatement (bins as lists, std::sort order from libstdc++ via the oracle)."""
    factor = np.float32(1.0) / np.float32(30)
    hist = [[] for _ in range(30)]
    for i in range(len(match)):
        j = int(match[i])
        if j < 0:
            continue
        diff = np.float32(angB[j]) - np.float32(angA[i])
        if diff < 0:
            diff = np.float32(diff + np.float32(360))
        b = int(np.rint(np.float32(factor * diff)))
        if b == 30:
            b = 0
        hist[b].append(i)
    perm = std_sort_perm(np.array([len(h) for h in hist], np.int32))
    srt = [hist[k] for k in perm]
    m1, m2, m3 = len(srt[0]), len(srt[1]), len(srt[2])
    erase = 1 if m2 < 0.1 * m1 else (2 if m3 < 0.1 * m1 else 3)
    out = match.copy()
    red = 0
    for h in srt[erase:]:
        for i in h:
            out[i] = -1
            red += 1
    return out, int((match >= 0).sum()) - red
