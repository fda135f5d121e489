#!/usr/bin/env python3
"""How much the two OpenCV-build switches change Extract's output (CPU oracle only, no GPU).

The reference's keypoints / descriptors depend on two things its own source does not fix
(include/orbslam2_amd.h orbx_set_opencv_compat):
  * trig: `cos(angle)` at src/ORBextractor.cc:107 is ::cos(double) or std::cos(float) (cosf);
  * resize_simd V: where cv::resize's vertical SIMD loop stops and its scalar tail (different
    rounding) starts, per pyramid level (src/ORBextractor.cc:466-468).
For each mode against the default (double, V = 16) this counts, per 10^4 keypoints of the default:
  * keypoints of one output missing from the other (matched on (x, y, octave));
  * common keypoints whose angle or response differ;
  * common keypoints whose 32-byte descriptor differs, and the differing descriptor bits.
Frames: the golden C1 frames (synth_image seeds 0-3, 640x480, 1000 features), the bench's C2 pan
frames (pan_sequence(0, 1280, 720, 16), 2000 features) and textured C2 frames.

Usage: python tools/compat_sensitivity.py [--c2 N] [--json out.json]
"""
import argparse
import json
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import oracle_api as O  # noqa: E402
from orb_slam2_refactored_amd.synth import pan_sequence, synth_image, textured_image  # noqa: E402

MODES = [("double", 16), ("float", 16), ("double", 0), ("double", 1), ("double", 8), ("double", 32),
         ("double", 64), ("float", 0)]


def extract_all(frames, nfeat, trig, v):
    O.set_compat(trig, v)   # process-wide: set before the threads start, not changed while they run
    p = O.params(nfeat)
    with ThreadPoolExecutor(8) as ex:
        return list(ex.map(lambda im: O.extract(p, im, cap=16384)[:2], frames))


def compare(base, other):
    st = dict(kps=0, missing=0, extra=0, angle_or_response=0, desc_rows=0, desc_bits=0)
    for (k0, d0), (k1, d1) in zip(base, other):
        st["kps"] += len(k0)
        key = lambda k: list(zip(k["x"].tolist(), k["y"].tolist(), k["octave"].tolist()))
        m1 = {kk: i for i, kk in enumerate(key(k1))}
        common = 0
        for i, kk in enumerate(key(k0)):
            j = m1.pop(kk, None)
            if j is None:
                st["missing"] += 1
                continue
            common += 1
            if k0["angle"][i] != k1["angle"][j] or k0["response"][i] != k1["response"][j]:
                st["angle_or_response"] += 1
            x = np.bitwise_xor(d0[i], d1[j])
            if x.any():
                st["desc_rows"] += 1
                st["desc_bits"] += int(np.unpackbits(x).sum())
        st["extra"] += len(m1)
    per = 1e4 / max(st["kps"], 1)
    return {**st, **{f"{k}_per_1e4": round(v * per, 2) for k, v in st.items() if k != "kps"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c2", type=int, default=16, help="C2 pan frames (and as many textured ones)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    sets = {
        "C1 golden (seeds 0-3)": ([synth_image(s, 640, 480) for s in range(4)], 1000),
        f"C2 pan ({a.c2} frames)": (list(pan_sequence(0, 1280, 720, a.c2)), 2000),
        f"C2 textured ({a.c2} frames)": ([textured_image(s, 1280, 720) for s in range(a.c2)], 2000),
    }
    res = {}
    prev = O.set_compat()
    try:
        for name, (frames, nf) in sets.items():
            outs = {m: extract_all(frames, nf, *m) for m in MODES}
            base = outs[MODES[0]]
            res[name] = {f"trig={t} V={v}": compare(base, outs[(t, v)]) for (t, v) in MODES[1:]}
            print(f"== {name}: {sum(len(k) for k, _ in base)} keypoints in the default mode (double, V=16)")
            print(f"{'mode':22s} {'missing':>8s} {'extra':>8s} {'ang/resp':>9s} {'desc rows':>10s} {'desc bits':>10s}  (per 1e4 keypoints)")
            for m, st in res[name].items():
                print(f"{m:22s} {st['missing_per_1e4']:8.2f} {st['extra_per_1e4']:8.2f} {st['angle_or_response_per_1e4']:9.2f} "
                      f"{st['desc_rows_per_1e4']:10.2f} {st['desc_bits_per_1e4']:10.2f}")
    finally:
        O.set_compat(*prev)
    if a.json:
        Path(a.json).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
