#!/usr/bin/env python3
"""Probe: one extract + match step captured in a HIP graph (torch.cuda.CUDAGraph) against eager
launches, same stream, same buffers; prints ms per step for both and checks the outputs agree."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch
    from orb_slam2_refactored_amd import ORBextractor, ORBmatcher
    from orb_slam2_refactored_amd.synth import synth_image
    F = 128
    pool = np.stack([synth_image(i, 1280, 720) for i in range(16)])
    frames = torch.from_numpy(np.concatenate([pool[i % 16][None] for i in range(F)])).cuda()
    ex = ORBextractor(ORBextractor.Parameters(nfeatures=2000))
    m = ORBmatcher(0.6, False)
    kps, desc, cnt = ex.extract_batch_device(frames)
    prev = torch.tensor([(i - 1) % F for i in range(F)], dtype=torch.int32, device="cuda")
    cap = desc.shape[1]
    mout = torch.empty((4, F, cap), dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    torch.cuda.synchronize()

    def step():
        ex.extract_batch_device(frames, kps, desc, cnt, stream=s)
        m.match_batch_device(desc, cnt, desc, cnt, out=mout, stream=s, pair_b=prev)

    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.synchronize()
    ref = mout.clone()
    N = 50
    t0 = time.perf_counter()
    with torch.cuda.stream(s):
        for _ in range(N):
            step()
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / N * 1e3
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        step()
    torch.cuda.synchronize()
    mout.zero_()
    g.replay()
    torch.cuda.synchronize()
    same = bool(torch.equal(mout, ref))
    t0 = time.perf_counter()
    for _ in range(N):
        g.replay()
    torch.cuda.synchronize()
    graph = (time.perf_counter() - t0) / N * 1e3
    print(f"eager {eager:.3f} ms/step  graph {graph:.3f} ms/step  outputs equal: {same}")


if __name__ == "__main__":
    main()
