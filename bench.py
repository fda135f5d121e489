#!/usr/bin/env python3
"""Benchmark: ORB extract + brute-force Hamming match on 1280x720 frames (BASELINE.json configs[1],
"1280x720 mono, 8 levels, 2000 features, extract+brute-force Hamming match on 1 MI355X"), plus the
LocalBundleAdjustment LM-iteration rate on configs[3] (20 KF x 3000 MP).

One step = one batch of `--frames` synthetic frames already resident in HBM: ORBextractor::Extract on
every frame (one batched launch per stage) and a brute-force top-2 + ratio match of every frame
against its predecessor in the batch (frame 0 against the last frame).  With N > 1 GPUs each rank
processes its own batch (weak scaling: frames are independent) and the step ends with an RCCL
all-gather of the padded keypoint/descriptor slots (the loop-closure descriptor exchange of
BASELINE.json configs[4]).

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = json.loads((ROOT / "BASELINE.json").read_text())["metric"]   # verbatim
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec


def level_sizes(W, H, nlevels=8, scale=1.2):
    s = np.float32(1.0)
    out = []
    for _ in range(nlevels):
        inv = np.float32(1.0) / s
        out.append((int(np.rint(np.float32(inv * W))), int(np.rint(np.float32(inv * H)))))
        s = np.float32(s * np.float32(scale))
    return out


def algorithmic_bytes(W, H, n_kp, nlevels=8):
    """SURVEY §8d B_ext = P + (P - W*H) + 60*N: read every level once, write levels 1.. once,
    28-B keypoint + 32-B descriptor per feature."""
    P = sum(w * h for w, h in level_sizes(W, H, nlevels))
    return P + (P - W * H) + 60 * n_kp, P


STAGE_KERNEL = {"pyramid": "pyramid_level_kernel", "fast_cells": "fast_cells_kernel", "quadtree": "quadtree_kernel",
                "describe": "describe_kernel"}


def measured_traffic(stage, launches_per_step, frames, W, H, nfeat):
    """HBM bytes per launch of `stage` from the committed rocprofv3 FETCH_SIZE / WRITE_SIZE passes
    (profiles/*_traffic.json, tools/gpu_traffic.sh), corrected by the calibration measured in the same
    run (FETCH_SIZE counts half the bytes of streaming reads on gfx950; WRITE_SIZE exact).  Only
    reported when the profiled workload is this one; otherwise None."""
    files = sorted(ROOT.glob("profiles/*_traffic.json"))
    if not files or (frames, W, H, nfeat) != (128, 1280, 720, 2000):
        return None
    t = json.loads(files[-1].read_text())
    k = t["kernels_per_dispatch"].get(STAGE_KERNEL.get(stage, ""))
    if not k or k.get("fetch_bytes") is None:
        return None
    cal = t["calibration"]
    fetch = k["fetch_bytes"] / cal.get("fetch_ratio_8B", 0.5)
    write = (k.get("write_bytes") or 0.0) / cal.get("write_ratio_4B", 1.0)
    # the profile averages over dispatches; a stage with several launches per step (pyramid: one
    # per level) is reported per average launch, like `achieved`
    return fetch + write


def cpu_baseline(frames_np, nfeat, budget_s=12.0):
    """Oracle (single-threaded C++ restatement) extract + match on a bounded sample."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_api as O
    p = O.params(nfeat)
    done = 0
    prev = None
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s or done < 3:
        img = frames_np[done % len(frames_np)]
        _, d, _ = O.extract(p, img)
        if prev is not None:
            O.bf_match(d, prev)
        prev = d
        done += 1
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"{done} frames of 1280x720 (extract + bf match vs previous), oracle/orb_oracle.cpp, 1 thread"}


def cpu_ba_baseline(prob, budget_s=6.0):
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_api as O
    iters = 0
    calls = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s or calls < 2:
        r = O.local_ba(prob)
        iters += sum(r["iterations"])
        calls += 1
    dt = time.perf_counter() - t0
    return {"iters_per_s": iters / dt, "ms_per_call": 1e3 * dt / calls, "calls": calls, "cores": 1, "kind": "port"}


def stereo_leg(dev, local, pairs=64, steps=5):
    """configs[2]-shaped secondary measurement: 1242x375 stereo pairs (8 depth bands), both sides
    extracted in one batch each, then ComputeStereoMatches per pair on the on-device pyramids."""
    import torch
    from orb_slam2_refactored_amd import ORBextractor
    from orb_slam2_refactored_amd.matcher import stereo_matches_batch_device
    from orb_slam2_refactored_amd.synth import KITTI, stereo_pair
    pool = [stereo_pair(7000 + i) for i in range(8)]
    Ls = torch.from_numpy(np.stack([pool[i % 8][0] for i in range(pairs)])).to(dev)
    Rs = torch.from_numpy(np.stack([pool[i % 8][1] for i in range(pairs)])).to(dev)
    exl = ORBextractor(ORBextractor.Parameters(2000), device=local)
    exr = ORBextractor(ORBextractor.Parameters(2000), device=local)
    bf, base = KITTI["bf"], KITTI["bf"] / KITTI["fx"]
    outl = exl.extract_batch_device(Ls)
    outr = exr.extract_batch_device(Rs)
    out = stereo_matches_batch_device(exl, exr, outl, outr, bf, base)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        exl.extract_batch_device(Ls, *outl)
        exr.extract_batch_device(Rs, *outr)
        stereo_matches_batch_device(exl, exr, outl, outr, bf, base, out=out)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    t1 = time.perf_counter()
    for _ in range(steps):
        stereo_matches_batch_device(exl, exr, outl, outr, bf, base, out=out)
    torch.cuda.synchronize()
    dts = (time.perf_counter() - t1) / steps
    matched = float((out[1] > 0).sum().item()) / pairs
    return {"workload": "C3-shaped: 1242x375 stereo pairs, 2000 features, extract L+R + ComputeStereoMatches",
            "pairs_per_step": pairs, "pairs_per_s": pairs / dt, "stereo_match_ms_per_step": 1e3 * dts,
            "matched_per_pair": matched}


def pose_leg(dev, frames=1024, edges=1000, steps=10, cpu=True):
    """§8f row 3: batched PoseOptimization (Optimizer.cc:345-489), frames x edges map-point matches
    (KITTI-tracking sized), inputs resident in HBM, one launch per step; CPU oracle beside it."""
    import torch
    from orb_slam2_refactored_amd.optimizer import pose_optimization_device
    from orb_slam2_refactored_amd.synth import make_pose_batch
    b = make_pose_batch(12, n_frames=frames, n_edges=edges)
    d = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in b.items() if not k.startswith("gt_")}
    out = pose_optimization_device(d)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        pose_optimization_device(d, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    r = {"workload": f"{frames} frames x {edges} edges (40 % stereo, 10 % outliers), 4 x optimize(10), fp64",
         "frames_per_s": frames / (ms * 1e-3), "ms_per_step": ms,
         "mean_inliers": float(out["n_inliers"].double().mean().item())}
    if cpu:
        sys.path.insert(0, str(ROOT / "tests"))
        import oracle_api as O
        sub = make_pose_batch(13, n_frames=16, n_edges=edges)
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < 4.0 or n < 16:
            O.pose_optimization(sub)
            n += 16
        r["cpu_baseline"] = {"frames_per_s": n / (time.perf_counter() - t0), "cores": 1, "kind": "port",
                             "sample": f"16-frame batches of {edges} edges, oracle/orb_oracle.cpp, 1 thread"}
    return r


def projection_leg(dev, frames=256, steps=10, cpu=True):
    """§8f row 2: batched SearchByProjection + FeaturesGrid (ORBmatcher.cc:315-382, Frame.cc:71-145):
    per frame 2000 keypoints and 1500 local map points (th 1, nnratio 0.8), inputs in HBM."""
    import torch
    from orb_slam2_refactored_amd.matcher import search_by_projection_device
    from orb_slam2_refactored_amd.synth import make_proj_batch, tile_proj_batch
    base = make_proj_batch(21, n_frames=16, n_kp=2000, n_mp=1500)
    b = tile_proj_batch(base, frames // 16)
    d = {k: (torch.from_numpy(np.ascontiguousarray(v)).to(dev) if isinstance(v, np.ndarray) and k != "scale_factors"
             else v) for k, v in b.items()}
    km, nm = search_by_projection_device(d)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        search_by_projection_device(d, km, nm)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    r = {"workload": f"{frames} frames x (2000 keypoints, 1500 map points), th 1, grid + score + claim walk",
         "frames_per_s": frames / (ms * 1e-3), "ms_per_step": ms,
         "mean_matches": float(nm.double().mean().item())}
    if cpu:
        sys.path.insert(0, str(ROOT / "tests"))
        import oracle_api as O
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < 3.0 or n < 16:
            O.search_by_projection(base)
            n += 16
        r["cpu_baseline"] = {"frames_per_s": n / (time.perf_counter() - t0), "cores": 1, "kind": "port",
                             "sample": "16-frame batches, oracle/orb_oracle.cpp, 1 thread"}
    return r


def bow_leg(dev, local, frames=128, n=2000, steps=10, cpu=True):
    """§8f row 4: Frame::ComputeBoW = ORBVocabulary::transform(desc, BowVector, FeatureVector, 4)
    (TemplatedVocabulary.h:1130-1263) on an ORBvoc-shaped synthetic tree (k 10, L 6, 1.1 M nodes),
    `frames` descriptor sets of `n` rows resident in HBM."""
    import torch
    from orb_slam2_refactored_amd.synth import make_full_vocabulary
    from orb_slam2_refactored_amd.vocabulary import ORBVocabulary
    v = make_full_vocabulary(31)
    voc = ORBVocabulary.from_arrays(v["k"], v["L"], v["scoring"], v["weighting"], v["parent"], v["is_leaf"],
                                    v["desc"], v["weight"], device=local)
    rng = np.random.default_rng(32)
    X = rng.integers(0, 256, size=(frames, n, 32), dtype=np.uint8)
    desc = torch.from_numpy(X).to(dev)
    counts = torch.full((frames,), n, dtype=torch.int32, device=dev)
    out = voc.transform_batch_device(desc, counts)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        voc.transform_batch_device(desc, counts, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    r = {"workload": f"{frames} frames x {n} descriptors, vocabulary k 10 L 6 (1.11 M nodes), levelsup 4",
         "frames_per_s": frames / (ms * 1e-3), "ms_per_step": ms,
         "mean_words": float(out["n_words"].double().mean().item())}
    if cpu:
        sys.path.insert(0, str(ROOT / "tests"))
        import oracle_api as O
        o = O.Vocabulary(v)
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < 3.0 or k < 8:
            o.transform(X[k % frames], 4)
            k += 1
        r["cpu_baseline"] = {"frames_per_s": k / (time.perf_counter() - t0), "cores": 1, "kind": "port",
                             "sample": f"{n}-descriptor sets, oracle/orb_oracle.cpp, 1 thread"}
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=128, help="frames per step per GPU")
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ba", action="store_true")
    ap.add_argument("--no-stereo", action="store_true")
    ap.add_argument("--no-pose", action="store_true")
    ap.add_argument("--no-projection", action="store_true")
    ap.add_argument("--no-bow", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from orb_slam2_refactored_amd import ORBextractor, ORBmatcher
    from orb_slam2_refactored_amd.synth import synth_image
    from orb_slam2_refactored_amd.shard import SlotExchange, Slots, shard_range

    W, H, B = args.width, args.height, args.frames
    # synthetic frames: this rank's shard of world*B global frames (seed = global frame index);
    # a pool of 16 distinct images is tiled over the batch
    g0, _ = shard_range(world * B, world, rank)
    pool = min(B, 16)
    base = np.stack([synth_image(g0 + i, W, H) for i in range(pool)])
    frames_np = np.concatenate([base[i % pool][None] for i in range(B)])
    frames = torch.from_numpy(frames_np).to(dev)
    ex = ORBextractor(ORBextractor.Parameters(nfeatures=args.nfeatures), device=local)
    m = ORBmatcher(0.6, False)
    cap = ex.max_keypoints(H, W)
    prev_idx = torch.tensor([(i - 1) % B for i in range(B)], dtype=torch.int32, device=dev)
    match_out = torch.empty((4, B, cap), dtype=torch.int32, device=dev)
    # world > 1: double-buffered async all-gather of every rank's slots (shard.SlotExchange);
    # step k's collectives overlap step k+1's kernels.
    xchg = SlotExchange(B, cap, dev) if world > 1 else None
    single = Slots.empty(B, cap, dev)
    stream = torch.cuda.current_stream()
    last = [single]

    def step():
        local = xchg.acquire() if xchg else single
        ex.extract_batch_device(frames, local.kps, local.desc, local.counts, stream=stream)
        m.match_batch_device(local.desc, local.counts, local.desc, local.counts, out=match_out, stream=stream,
                             pair_b=prev_idx)
        if xchg:
            xchg.publish()
        last[0] = local

    for _ in range(args.warmup):
        step()
    if xchg:
        xchg.drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # inside the timed region only the dominant kernel (fast_cells) carries launch events (events on
    # every kernel cost ~3.5 % of the step); the other stages are timed in a separate pass below
    ex.profile(True, stages=["fast_cells"])
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    if xchg:
        xchg.drain()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ex.profile(False)
    timed = ex.profile_read()
    # per-stage breakdown: a separate short pass with events on every kernel (not the timed region)
    ex.profile(True)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    ex.profile(False)
    breakdown = ex.profile_read()
    brk_steps = 3
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    n_kp = float(last[0].counts.float().mean().item())
    matches = int((match_out[3] >= 0).sum().item())
    total_frames = world * B * args.steps
    value = total_frames / elapsed
    ms_per_step = 1e3 * elapsed / args.steps

    # roofline of the dominant kernel (per-launch algorithmic bytes / average launch time)
    bytes_frame, P = algorithmic_bytes(W, H, n_kp)
    stage_bytes = {
        "pyramid": (P - W * H) + (P - level_sizes(W, H)[-1][0] * level_sizes(W, H)[-1][1]),   # read l-1, write l
        "fast_cells": P + 4 * 0,    # every level read once (candidate lists are intermediates)
        "quadtree": 0,
        "describe": 60 * n_kp,      # keypoint + descriptor writes (neighbourhood reads are L2 re-reads)
    }
    dom = max(breakdown, key=lambda k: breakdown[k][0])
    if dom == "fast_cells":   # the live launch times of the timed region
        dom_ms, dom_launches = timed[dom]
        dom_steps = args.steps
    else:                     # another stage dominates: its times from the breakdown pass
        dom_ms, dom_launches = breakdown[dom]
        dom_steps = brk_steps
    traffic = measured_traffic(dom, dom_launches / max(dom_steps, 1), B, W, H, args.nfeatures)
    per_launch_ms = dom_ms / max(dom_launches, 1)
    launches_per_step = dom_launches / max(dom_steps, 1)
    # a stage may run as several launches per step (fast_cells: level 0 on the side stream, levels
    # 1..7 on the main stream): achieved = the step's algorithmic bytes / the step's summed launch
    # durations, i.e. per launch = bytes / launches_per_step over the average launch duration
    dom_bytes = stage_bytes[dom] * B / max(launches_per_step, 1)
    achieved = dom_bytes / (per_launch_ms * 1e-3) / 1e9 if per_launch_ms > 0 else 0.0
    extract_ms = sum(v[0] for v in breakdown.values()) / brk_steps
    pipeline_gbs = bytes_frame * B / (extract_ms * 1e-3) / 1e9 if extract_ms > 0 else 0.0

    result = {
        "metric": METRIC,
        "value": value,
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": f"C2: {W}x{H} mono, 8 levels, {args.nfeatures} features, extract + brute-force "
                               f"Hamming top-2/ratio match vs previous frame",
                   "frames_per_step_per_gpu": B, "width": W, "height": H, "nlevels": 8,
                   "nfeatures": args.nfeatures, "parallelism": f"frames sharded over {world} GPU(s)"
                   + (", RCCL all-gather of descriptor slots" if world > 1 else "")},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "algorithmic_bytes_per_launch": dom_bytes, "avg_launch_ms": per_launch_ms,
                     "launches_per_step": launches_per_step,
                     "timed_from": "timed region" if dom == "fast_cells" else "breakdown pass",
                     "stage_ms_per_step": {k: v[0] / brk_steps for k, v in breakdown.items()},
                     "stage_ms_source": "separate 3-step pass with launch events on every kernel",
                     "pipeline_algorithmic_GBs": pipeline_gbs, "pipeline_bytes_per_frame": bytes_frame},
        "keypoints_per_frame": n_kp,
        "matches_last_step": matches,
    }

    if rank == 0 and not args.no_ba:
        from orb_slam2_refactored_amd.optimizer import LocalBundleAdjustment
        from orb_slam2_refactored_amd.synth import make_ba_problem
        prob = make_ba_problem(0, n_kf=20, n_pts=3000, n_fixed=2)
        LocalBundleAdjustment(prob, device=local)   # warm-up
        iters = 0
        t1 = time.perf_counter()
        calls = 0
        while calls < 5:
            r = LocalBundleAdjustment(prob, device=local)
            iters += sum(r["iterations"])
            calls += 1
        dtb = time.perf_counter() - t1
        result["localba"] = {"workload": "C4: 20 KF x 3000 MP, optimize(5)+optimize(10), fp64",
                             "iters_per_s": iters / dtb, "ms_per_call": 1e3 * dtb / calls,
                             "edges": int(len(prob["edge_point"]))}
        if world == 1 and not args.no_cpu_baseline:
            result["localba"]["cpu_baseline"] = cpu_ba_baseline(prob)

    if rank == 0 and not args.no_stereo:
        result["stereo"] = stereo_leg(dev, local)

    if rank == 0 and not args.no_projection:
        result["search_by_projection"] = projection_leg(dev, cpu=world == 1 and not args.no_cpu_baseline)

    if rank == 0 and not args.no_bow:
        result["bow"] = bow_leg(dev, local, cpu=world == 1 and not args.no_cpu_baseline)

    if rank == 0 and not args.no_pose:
        result["pose_opt"] = pose_leg(dev, cpu=world == 1 and not args.no_cpu_baseline)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(frames_np[:4], args.nfeatures)
        result["cpu_baseline"]["host"] = os.uname().nodename
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
