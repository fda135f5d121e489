"""Price describe's LDS tap-read bank conflicts, and what a per-angle pair placement could save.

Offline model (no GPU): describe's sample stage (orbx.hip describe_kernel, `sample`) reads 7 vertical
taps of the horizontally blurred patch Hb (u16, row stride HBS) per sample point; lane L of round r
samples pair 64 r + L, first point then second point.  A ds_read_u16 is banked as two lane groups of 32
over 32 dword banks (MI355X_MICROARCH §LDS); identical dwords broadcast; each extra distinct dword on a
bank adds one cycle.  The 7 taps of one sample sit 20 k dwords apart, a constant bank shift, so every
tap instruction of a sample has the conflicts of its first tap.

It compares, over random keypoint angles:
  * today's placement (pair p in round p // 64, lane p % 64);
  * a per-angle-bucket placement: the 256 pairs re-assigned to the 8 (round, half) groups of 32 to
    balance the banks of both points, found by a greedy swap search at the bucket's centre angle and
    evaluated at random angles inside the bucket (the bits would be restored by one ds_bpermute per
    round);
  * the column-major blurred map (orbx.hip DESC_HBT=1): the 7 taps as 4 consecutive dwords.

usage: python tools/probe/desc_bank_price.py [buckets] [angles]
"""
import math
import pathlib
import re
import sys

import numpy as np

HBS = 40
ROOT = pathlib.Path(__file__).resolve().parents[2]


def pattern():
    txt = (ROOT / "orb_slam2_refactored_amd" / "csrc" / "orb_pattern31.inc").read_text()
    body = "\n".join(ln for ln in txt.splitlines() if not ln.lstrip().startswith("//"))
    v = np.array([int(t) for t in re.findall(r"-?\d+", body)], dtype=np.float32)
    assert v.size == 1024
    return v.reshape(256, 4)


def dwords(pat, deg):
    """Dword index of tap 0 of both sample points of every pair at keypoint angle `deg` (as describe)."""
    ang = np.float32(deg * np.float32(math.pi / 180.0))
    a = np.float32(math.cos(float(ang)))
    b = np.float32(math.sin(float(ang)))
    out = []
    for x, y in ((pat[:, 0], pat[:, 1]), (pat[:, 2], pat[:, 3])):
        dy = np.rint(x * b + y * a).astype(np.int64)
        dx = np.rint(x * a - y * b).astype(np.int64)
        ob = 2 * ((18 + dy) * HBS + 18 + dx)
        out.append(ob >> 2)
    return np.stack(out)   # [2, 256]


def group_cycles(dw):
    """LDS cycles of one 32-lane group: max over banks of distinct dwords."""
    u = np.unique(dw)
    return int(np.bincount(u % 32, minlength=32).max())


def cost(dw2, groups):
    """Cycles of both sample instructions (tap 0) over the 8 groups of 32 pairs."""
    return sum(group_cycles(dw2[s, g]) for g in groups for s in (0, 1))


def optimise(dw2, iters, rng):
    perm = np.arange(256)
    groups = [perm[32 * i:32 * (i + 1)].copy() for i in range(8)]
    cur = [sum(group_cycles(dw2[s, g]) for s in (0, 1)) for g in groups]
    for _ in range(iters):
        i, j = rng.choice(8, 2, replace=False)
        a, b = rng.integers(32), rng.integers(32)
        gi, gj = groups[i].copy(), groups[j].copy()
        gi[a], gj[b] = gj[b], gi[a]
        ci = sum(group_cycles(dw2[s, gi]) for s in (0, 1))
        cj = sum(group_cycles(dw2[s, gj]) for s in (0, 1))
        if ci + cj <= cur[i] + cur[j]:
            groups[i], groups[j], cur[i], cur[j] = gi, gj, ci, cj
    return groups


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 90
    na = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    pat = pattern()
    rng = np.random.default_rng(0)
    base_groups = [np.arange(32 * i, 32 * (i + 1)) for i in range(8)]
    plans = {}
    base, opt, ideal = [], [], 2 * 8   # ideal: one cycle per group per sample instruction
    for deg in rng.uniform(0, 360, na):
        bk = int(deg / 360 * nb) % nb
        if bk not in plans:
            plans[bk] = optimise(dwords(pat, (bk + 0.5) * 360 / nb), 3000, rng)
        dw2 = dwords(pat, deg)
        base.append(cost(dw2, base_groups))
        opt.append(cost(dw2, plans[bk]))
    base, opt = np.mean(base), np.mean(opt)
    print(f"tap-0 LDS cycles per keypoint (8 groups x 2 samples, conflict-free = {ideal}):")
    print(f"  today's placement      {base:.1f}  ({base / ideal:.2f}x)")
    print(f"  {nb}-bucket placement   {opt:.1f}  ({opt / ideal:.2f}x)")
    print(f"  x 7 taps: {7 * base:.0f} -> {7 * opt:.0f} LDS cycles per keypoint")
    # the column-major map (DESC_HBT): a sample's taps are u16 q .. q + 6 of column 18 + dx, read as
    # dwords q / 2 .. q / 2 + 3 (two ds_read2_b32, each banked as two ds_read_b32)
    hcs = 52
    col = []
    for deg in rng.uniform(0, 360, na):
        ang = np.float32(deg * np.float32(math.pi / 180.0))
        a, b = np.float32(math.cos(float(ang))), np.float32(math.sin(float(ang)))
        c = 0
        for x, y in ((pat[:, 0], pat[:, 1]), (pat[:, 2], pat[:, 3])):
            dy = np.rint(x * b + y * a).astype(np.int64)
            dx = np.rint(x * a - y * b).astype(np.int64)
            w = ((18 + dx) * hcs + 18 + dy) >> 1
            c += sum(group_cycles(w[g] + k) for g in base_groups for k in range(4))
        col.append(c)
    print(f"  column-major map, 4 dwords per sample: {np.mean(col):.0f} LDS cycles per keypoint "
          f"(conflict-free {2 * 8 * 4})")


if __name__ == "__main__":
    main()
