#!/usr/bin/env python3
"""Kernel-level driver for profiling: runs the batched extractor (+ matcher) `--iters` times on
`--frames` synthetic 1280x720 frames resident in HBM, prints per-stage HIP-event times."""
import argparse
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=128)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--match", action="store_true")
    ap.add_argument("--pan", action="store_true", help="bench.py's frames: the §8d pan sequence (default: G frames)")
    ap.add_argument("--textured", action="store_true", help="texture-rich frames (bench.py c2_textured)")
    ap.add_argument("--no-profile", action="store_true", help="no per-stage event timing (wall time only)")
    a = ap.parse_args()
    import torch
    from orb_slam2_refactored_amd import ORBextractor, ORBmatcher
    from orb_slam2_refactored_amd.synth import pan_sequence, synth_image, textured_image
    if a.pan:
        pool = pan_sequence(0, a.width, a.height, min(16, a.frames))
    elif a.textured:
        pool = np.stack([textured_image(4000 + i, a.width, a.height) for i in range(min(16, a.frames))])
    else:
        pool = np.stack([synth_image(i, a.width, a.height) for i in range(min(16, a.frames))])
    frames = torch.from_numpy(np.concatenate([pool[i % len(pool)][None] for i in range(a.frames)])).cuda()
    ex = ORBextractor(ORBextractor.Parameters(nfeatures=a.nfeatures))
    kps, desc, cnt = ex.extract_batch_device(frames)
    m = ORBmatcher(0.6, False)
    prev = torch.tensor([(i - 1) % a.frames for i in range(a.frames)], dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ex.profile(not a.no_profile)
    t0 = time.perf_counter()
    for _ in range(a.iters):
        ex.extract_batch_device(frames, kps, desc, cnt)
        if a.match:
            m.match_batch_device(desc, cnt, desc, cnt, pair_b=prev)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = ex.profile_read()
    out = {k: round(v[0] / a.iters, 4) for k, v in st.items()}
    if a.match:   # the matcher alone, back to back (launch-bound gaps included)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            m.match_batch_device(desc, cnt, desc, cnt, pair_b=prev)
        e1.record()
        torch.cuda.synchronize()
        out["match"] = round(e0.elapsed_time(e1) / a.iters, 4)
    print(out, f"wall/iter {1e3 * dt / a.iters:.3f} ms", f"fps {a.frames * a.iters / dt:.0f}")


if __name__ == "__main__":
    main()
