"""Where in the patch do the descriptor bits that differ between identical runs sample?

Reads the DET_DUMP json of tools/diag/desc_determinism.py (every differing row of run 1 against run
0: keypoint record, differing bit indices) and maps each differing bit (pattern pair k) to the two
blurred-patch positions describe reads for it, (18 + dy, 18 + dx) at the keypoint's angle, computed
as describe does (float32 products, no contraction, rint).  Prints histograms of the rows / columns
and of the 16x16 blur tiles the positions fall in, for the differing bits against all 256 bits of
the same keypoints: a position class over-represented among the differing bits is where the blurred
values (or the reads of them) differ.

usage: det_bits_positions.py dump.json
"""
import collections
import json
import math
import pathlib
import re
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]


def pattern():
    txt = (ROOT / "orb_slam2_refactored_amd" / "csrc" / "orb_pattern31.inc").read_text()
    body = "\n".join(ln for ln in txt.splitlines() if not ln.lstrip().startswith("//"))
    v = np.array([int(t) for t in re.findall(r"-?\d+", body)], dtype=np.float32)
    return v.reshape(256, 4)


def positions(pat, angle_deg):
    ang = np.float32(np.float32(angle_deg) * np.float32(math.pi / 180.0))
    a = np.float32(math.cos(float(ang)))
    b = np.float32(math.sin(float(ang)))
    out = []
    for x, y in ((pat[:, 0], pat[:, 1]), (pat[:, 2], pat[:, 3])):
        dy = np.rint(np.float32(x * b) + np.float32(y * a)).astype(np.int64)
        dx = np.rint(np.float32(x * a) - np.float32(y * b)).astype(np.int64)
        out.append((18 + dy, 18 + dx))
    return out   # [(rows[256], cols[256]) for point 0, point 1]


def main(path):
    rows = json.load(open(path))
    pat = pattern()
    diff_r, diff_c, all_r, all_c = collections.Counter(), collections.Counter(), collections.Counter(), collections.Counter()
    diff_t, all_t = collections.Counter(), collections.Counter()
    nbits = 0
    levels = collections.Counter()
    for r in rows:
        kp = np.array(r["kp"], dtype=np.int32)
        angle = float(kp[3:4].view(np.float32)[0])
        levels[int(kp[5])] += 1
        pos = positions(pat, angle)
        for k in range(256):
            for pr, pc in pos:
                all_r[int(pr[k])] += 1
                all_c[int(pc[k])] += 1
                all_t[(int(pr[k]) // 16, int(pc[k]) // 16)] += 1
        for k in r["bits"]:
            nbits += 1
            for pr, pc in pos:
                diff_r[int(pr[k])] += 1
                diff_c[int(pc[k])] += 1
                diff_t[(int(pr[k]) // 16, int(pc[k]) // 16)] += 1
    print(f"{len(rows)} differing rows, {nbits} differing bits; octaves {dict(sorted(levels.items()))}")
    tot_d, tot_a = sum(diff_r.values()), sum(all_r.values())

    def show(name, d, a):
        print(name)
        for key in sorted(a):
            fd, fa = d[key] / max(tot_d, 1), a[key] / tot_a
            print(f"  {key!s:>10}: differing {fd:6.3f}  all {fa:6.3f}  ratio {fd / fa if fa else 0:5.2f}")

    show("blurred row (18 + dy)", diff_r, all_r)
    show("blurred column (18 + dx)", diff_c, all_c)
    show("16x16 tile (row // 16, column // 16)", diff_t, all_t)


if __name__ == "__main__":
    main(sys.argv[1])
