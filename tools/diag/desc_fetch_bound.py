#!/usr/bin/env python3
"""Compulsory HBM fetch of describe_kernel per C2 frame (describe fetch <= 12 GB per
8192-frame launch).  Every kept keypoint reads its level's raw 43x43 neighbourhood (csrc/orbx.hip PATCH:
rBRIEF reach 18 + blur 3; ORBextractor.cc:74-140,799-806); the union of those neighbourhoods, in the
cache lines of the pyramid layout, is what a perfect cache would still fetch once.  Keypoints from the
oracle's Extract on pan frames (synth.pan_sequence, the bench's C2 workload) and on textured frames.
Prints bytes per frame and per 8192 frames next to the whole pyramid.  CPU only."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import oracle_api as O  # noqa: E402
from orb_slam2_refactored_amd.synth import pan_sequence, textured_image  # noqa: E402

R = 21      # patch half-width
LINE = 64   # bytes per cache line (L2 line on gfx950: 128 B; both printed)


def union_bytes(img, nf=2000, line=LINE):
    p = O.params(nf)
    kps, _, _ = O.extract(p, img)
    lv = O.pyramid(p, img)
    sc = O.scale_tables(p)["scale"]
    tot = pyr = 0
    for l, L in enumerate(lv):
        h, w = L.shape
        stride = w if l == 0 else (w + 15) // 16 * 16   # level 0: the frame itself; levels: 16-B aligned rows
        pyr += h * stride
        k = kps[kps["octave"] == l]
        mark = np.zeros((h, (stride + line - 1) // line + 1), bool)
        for x, y in zip(k["x"] / sc[l], k["y"] / sc[l]):
            cx, cy = int(round(x)), int(round(y))
            y0, y1 = max(0, cy - R), min(h - 1, cy + R)
            x0, x1 = max(0, cx - R), min(w - 1, cx + R)
            mark[y0:y1 + 1, x0 // line:x1 // line + 1] = True
        tot += int(mark.sum()) * line
    return tot, pyr, len(kps)


def main():
    frames = {"pan": pan_sequence(11, 1280, 720, 4), "textured": np.stack([textured_image(90 + i, 1280, 720) for i in range(2)])}
    for name, fr in frames.items():
        for line in (64, 128):
            u = [union_bytes(f, line=line) for f in fr]
            ub = np.mean([a for a, _, _ in u])
            pb = np.mean([b for _, b, _ in u])
            nk = np.mean([c for _, _, c in u])
            print(f"{name:9s} line {line:3d} B: {nk:7.1f} keypoints, union of patches {ub / 1e6:.3f} MB per frame "
                  f"({ub * 8192 / 1e9:.1f} GB per 8192 frames), pyramid {pb / 1e6:.3f} MB ({pb * 8192 / 1e9:.1f} GB)")


if __name__ == "__main__":
    main()
