#!/usr/bin/env python3
"""Benchmark of the ORB front end + LocalBA hot path (BASELINE.json).

Headline line (`value`): configs[1] / C2 — 1280x720 mono, 8 levels, 2000 features, extract + brute-force
Hamming top-2/ratio match of every frame against its predecessor.  One step = one batch of `--frames`
(default 8192) synthetic frames per GPU already resident in HBM: a camera-pan sequence (frame i = frame 0
shifted by i * (+3, +2) px with fresh noise: consecutive frames are the §8d C2 shifted pair), so frame i
is matched to i-1 as §8d C5 says (global frame 0 has no predecessor).  With N > 1 ranks the job is
N x 8192 frames (weak scaling): rank r extracts its contiguous shard, matches frames 1.. of the shard
locally, all-gathers the per-frame counts and then its Σn x 32 B descriptor block over RCCL (the
loop-closure descriptor exchange of configs[4]) and matches its first frame against rank r-1's last
frame read from the gathered descriptors (one step later, so the gather overlaps the next step's
kernels).

Secondary objects on the same JSON line, each with its own rate, roofline and CPU baseline:
  c1          configs[0]: 640x480, 1000 features — GPU batch throughput + the CPU plumbing median of 200
              single-frame Extract calls (seeds 0-15)
  c2_textured C2 on texture-rich frames (dense FAST candidates, deep quadtrees), per-stage times
  c3          configs[2]: stereo 1242x375, extract L+R + SearchForTriangulation (single BoW node)
  localba     configs[3]: 20 KF x 3000 MP, optimize(5) + optimize(10), fp64
  c5          configs[4] semantics at this N (cross-shard pairing, gather bytes); the scaling curve itself
              comes from the driver's N = 1, 2, 4, 8 runs
  stereo, search_by_projection, bow, pose_opt: the §8f rows

CPU baselines run the oracle (oracle/orb_oracle.cpp, the C++ restatement; the reference cannot be
built here) on the GPU box's host cores: one thread and 16 threads (one frame per thread) -- 16 is the
CPU share of a one-GPU box of this pool (its `nproc` reports the whole machine's CPUs, which the box
does not own) -- with the CPU model stated.  Prints ONE JSON line on rank 0.
"""
import argparse
import concurrent.futures as cf
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = json.loads((ROOT / "BASELINE.json").read_text())["metric"]   # verbatim
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_PEAK_TFLOPS = 78.6    # MI355X spec, FP64 vector (BASELINE.md / SURVEY §8d honest ceiling)
FP4_PEAK_TFLOPS = 10000.0  # MI355X_MICROARCH.md: FP4 / FP6 MFMA ~10 PF dense


# ------------------------------------------------------------------------------------------ helpers
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


def stage_bytes(W, H, n_kp):
    sz = level_sizes(W, H)
    P = sum(w * h for w, h in sz)
    return {"pyramid": (P - sz[-1][0] * sz[-1][1]) + (P - W * H),   # read l-1, write l
            "fast_cells": P,                                          # every level read once
            "quadtree": 0,                                            # intermediates only
            "describe": 60 * n_kp}                                    # keypoint + descriptor writes


def stage_kernels(nlevels=8):
    """Kernels per extractor stage and their launches per step: levels 1+2, 3+4, 5+6 are one
    pyramid_pair_kernel launch each, an odd last level one pyramid_level_kernel (the bench's frames are
    16-byte aligned, so pairing starts at level 1)."""
    n = nlevels - 1
    return {"pyramid": [("pyramid_pair_kernel", n // 2), ("pyramid_level_kernel", n % 2)],
            "fast_cells": [("fast_cells_kernel", 1)], "quadtree": [("quadtree_kernel", 1)],
            "describe": [("describe_kernel", 1)]}


STAGE_KERNELS = stage_kernels()


def traffic_profile(frames, W, H, nfeat):
    """The newest committed rocprofv3 FETCH_SIZE / WRITE_SIZE profile (profiles/*_traffic.json,
    tools/gpu_traffic.sh) of this exact workload, or None."""
    for f in sorted(ROOT.glob("profiles/*_traffic.json"), reverse=True):
        t = json.loads(f.read_text())
        wl = t.get("workload")
        if not isinstance(wl, dict):   # r01 files: the 128-frame C2 workload
            wl = {"frames": 128, "width": 1280, "height": 720, "nfeatures": 2000}
        if (wl.get("frames"), wl.get("width"), wl.get("height"), wl.get("nfeatures")) == (frames, W, H, nfeat):
            return t
    return None


def kernel_traffic(t, kernel):
    """HBM bytes per dispatch of `kernel` in profile `t`, corrected by the calibration measured in the same
    run (FETCH_SIZE counts half the bytes of streaming reads on gfx950; WRITE_SIZE exact); None if absent.
    A kernel launched several times per step (pyramid_pair_kernel) is the average over its dispatches."""
    k = t["kernels_per_dispatch"].get(kernel)
    if not k or k.get("fetch_bytes") is None:
        return None
    cal = t["calibration"]
    return k["fetch_bytes"] / cal.get("fetch_ratio_8B", 0.5) + (k.get("write_bytes") or 0.0) / cal.get("write_ratio_4B", 1.0)


def measured_traffic(stage, frames, W, H, nfeat):
    """HBM bytes per launch of a single-kernel stage (the roofline's dominant kernel), or None."""
    t = traffic_profile(frames, W, H, nfeat)
    ks = STAGE_KERNELS.get(stage, [])
    if t is None or len(ks) != 1:
        return None
    return kernel_traffic(t, ks[0][0])


def measured_traffic_step(frames, W, H, nfeat, nlevels=8, profile=None):
    """Measured HBM bytes per step of the whole extractor: every kernel's per-dispatch traffic x its
    launches per step (3 pyramid_pair_kernel + 1 pyramid_level_kernel at 8 levels), or None when a kernel
    of this workload has no committed profile (`profile`: a loaded *_traffic.json instead of the newest)."""
    t = profile if profile is not None else traffic_profile(frames, W, H, nfeat)
    if t is None:
        return None
    tot = 0.0
    for ks in stage_kernels(nlevels).values():
        for kernel, launches in ks:
            if not launches:
                continue
            b = kernel_traffic(t, kernel)
            if b is None:
                return None
            tot += b * launches
    return tot


# Issue roofline (VERDICT r05 "Next round" 5): the extractor kernels are bound by instruction issue, not
# HBM, so each stage's committed PMC instruction counts (profiles/rNN_pmc_inst_summary_{pan,textured}.txt,
# tools/gpu_pmc_round.sh: SQ_INSTS_VALU / SQ_INSTS_SALU per dispatch at 1024 frames, scaled to this
# launch's frames) are priced against the chip's issue slots over the stage's live time:
#   VALU: 1024 SIMDs x CLK_GHZ; a wave64 vector instruction holds its SIMD 4 cycles for the packed u16,
#         permute, compare and 64-bit forms the extractor is built from (tools/probe/issue_probe3; it is also
#         the rate rocprof's VALUBusy assumes) and 2 cycles for plain 32-bit ALU forms (SIMD-32 dual pass,
#         MI355X_MICROARCH constants table), so valu_frac_4cyc is the upper and valu_frac_2cyc the lower
#         bound of the VALU pipe's occupancy;
#   SALU: one scalar instruction per cycle per CU (256 CUs x CLK_GHZ; the rate SALUBusy assumes).
CLK_GHZ = 2.4
ISSUE_MODEL = ("VALU: 4 cycles (upper) / 2 cycles (lower) per wave64 instruction per SIMD, 1024 SIMDs; SALU: 1 "
               "instruction per cycle per CU, 256 CUs; clock 2.4 GHz; instruction counts from the committed PMC "
               "pass at 1024 frames scaled to the launch")


def pmc_inst_profile(kind):
    """The newest committed PMC instruction summary of the pan or textured C2 workload: (file, {kernel:
    {counter: per-dispatch value}}), or (None, None)."""
    for f in sorted(ROOT.glob(f"profiles/*_pmc_inst_summary_{kind}.txt"), reverse=True):
        d, cur = {}, None
        for line in f.read_text().splitlines():
            if not line.strip():
                continue
            if not line.startswith(" "):
                cur = line.strip()
                d[cur] = {}
            elif cur is not None:
                parts = line.split()
                try:
                    d[cur][parts[0]] = float(parts[-1])
                except ValueError:
                    pass
        return f.name, d
    return None, None


def issue_roofline(kind, stage_ms, frames, nlevels=8, pmc_frames=1024):
    """Per-stage VALU / SALU issue fractions (see ISSUE_MODEL) from `stage_ms` (ms per step of each stage)."""
    src, d = pmc_inst_profile(kind)
    if d is None:
        return None
    out = {}
    for stage, ks in stage_kernels(nlevels).items():
        t = (stage_ms.get(stage) or 0.0) * 1e-3
        valu = salu = 0.0
        ok = t > 0
        for kernel, launches in ks:
            c = d.get(kernel)
            if launches and (not c or "SQ_INSTS_VALU" not in c or "SQ_INSTS_SALU" not in c):
                ok = False
                break
            if launches:
                valu += c["SQ_INSTS_VALU"] * launches
                salu += c["SQ_INSTS_SALU"] * launches
        if not ok:
            continue
        valu *= frames / pmc_frames
        salu *= frames / pmc_frames
        simd_slots = 1024 * CLK_GHZ * 1e9 * t
        out[stage] = {"ms_per_step": 1e3 * t, "valu_insts": valu, "salu_insts": salu,
                      "valu_frac_4cyc": 4 * valu / simd_slots, "valu_frac_2cyc": 2 * valu / simd_slots,
                      "salu_frac": salu / (256 * CLK_GHZ * 1e9 * t)}
    return {"source": f"profiles/{src}", "workload": kind, "model": ISSUE_MODEL, "stages": out}


def cpu_info():
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    return {"cpu_model": model, "nproc": os.cpu_count(), "usable_cpus": usable,
            "threads_all": max(1, min(16, usable))}


def run_threads(work, threads, budget_s):
    """work(stop_time) -> units done; run on `threads` Python threads (the oracle is called through
    ctypes, which releases the GIL), return (units/s, units)."""
    t0 = time.perf_counter()
    stop = t0 + budget_s
    with cf.ThreadPoolExecutor(threads) as pool:
        done = sum(pool.map(lambda _: work(stop), range(threads)))
    return done / (time.perf_counter() - t0), done


def oracle():
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_api as O
    O.lib()
    return O


def cpu_extract_match(frames_np, nfeat, threads, budget_s):
    """Oracle extract + brute-force match vs the previous frame, one frame per thread at a time."""
    O = oracle()
    p = O.params(nfeat)

    def work(stop):
        prev, n, i = None, 0, int.from_bytes(os.urandom(2), "little")
        while time.perf_counter() < stop or n < 2:
            _, d, _ = O.extract(p, frames_np[i % len(frames_np)])
            if prev is not None:
                O.bf_match(d, prev)
            prev = d
            n += 1
            i += 1
        return n

    return run_threads(work, threads, budget_s)


def cpu_baseline_block(unit, sample, single, multi, info):
    v1, n1 = single
    vN, nN = multi
    return {"value": vN, "unit": unit, "cores": info["threads_all"], "kind": "port",
            "sample": f"{sample}; {nN} units on {info['threads_all']} threads, oracle/orb_oracle.cpp (-O3)",
            "single_thread": {"value": v1, "cores": 1, "units": n1}, "cpu_model": info["cpu_model"],
            "nproc": info["nproc"], "usable_cpus": info["usable_cpus"],
            "cores_note": "16 threads = the CPU share of this pool's one-GPU box: the box runs one GPU of an 8-GPU "
                          "host and sets OMP_NUM_THREADS / MAX_JOBS to 16; nproc / affinity report the whole "
                          "host's CPUs, shared with the other GPUs' jobs, so an all-cores run would measure "
                          "contention, not this port"}


def event_ms(fn, steps, stream):
    import torch
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def extract_match_gpu_leg(dev, local, frames_np, nfeat, steps=10, reps=None, issue_kind=None):
    """Batched extract + match-vs-predecessor on `frames_np` tiled to `reps` frames; returns the rate,
    per-stage times and the fast_cells roofline."""
    import torch
    from orb_slam2_refactored_amd import ORBextractor, ORBmatcher
    F = reps or len(frames_np)
    H, W = frames_np.shape[1:]
    idx = torch.arange(F) % len(frames_np)
    frames = torch.from_numpy(frames_np).to(dev)[idx.to(dev)].contiguous()
    ex = ORBextractor(ORBextractor.Parameters(nfeatures=nfeat), device=local)
    m = ORBmatcher(0.6, False)
    prev = torch.tensor([(i - 1) % F for i in range(F)], dtype=torch.int32, device=dev)
    kps, desc, cnt = ex.extract_batch_device(frames)
    out = m.match_batch_device(desc, cnt, desc, cnt, pair_b=prev)
    st = torch.cuda.current_stream()

    def step():
        ex.extract_batch_device(frames, kps, desc, cnt, stream=st)
        m.match_batch_device(desc, cnt, desc, cnt, out=out, pair_b=prev, stream=st)

    step()
    torch.cuda.synchronize()
    ms = event_ms(step, steps, st)
    ex.profile(True)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    ex.profile(False)
    brk = ex.profile_read()
    ex.batch_status()
    n_kp = float(cnt.float().mean().item())
    stg = {k: v[0] / 3 for k, v in brk.items()}
    fb = stage_bytes(W, H, n_kp)["fast_cells"] * F
    fms = brk["fast_cells"][0] / max(brk["fast_cells"][1], 1)
    bytes_frame, _ = algorithmic_bytes(W, H, n_kp)
    return {"frames_per_step": F, "frames_per_s": F / (ms * 1e-3), "ms_per_step": ms,
            "keypoints_per_frame": n_kp, "matches_per_frame": float((out[3] >= 0).sum().item()) / F,
            "stage_ms_per_step": stg,
            "roofline": {"bound": "hbm", "kernel": "fast_cells", "achieved": fb / (fms * 1e-3) / 1e9 if fms else 0.0,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": (fb / (fms * 1e-3) / 1e9 / HBM_PEAK_GBS) if fms else 0.0,
                         "algorithmic_bytes_per_launch": fb, "avg_launch_ms": fms,
                         "pipeline_algorithmic_GBs": bytes_frame * F / (sum(stg.values()) * 1e-3) / 1e9,
                         "issue": issue_roofline(issue_kind, stg, F) if issue_kind else None}}


# ------------------------------------------------------------------------------------------ legs
def c1_leg(dev, local, frames=1024, cpu=True, info=None):
    """configs[0]: 640x480, 8 levels, 1000 features.  GPU: batched extract + match throughput (north
    star "synthetic 640x480 pyramids ... fps and fraction of HBM roofline").  CPU: the plumbing
    measurement of BASELINE.md — median of 200 single-frame oracle Extract calls over seeds 0-15 after
    10 warm-ups, one thread (the reference's Extract is single-threaded)."""
    from orb_slam2_refactored_amd import ORBextractor
    from orb_slam2_refactored_amd.synth import pan_sequence
    seq = pan_sequence(0, 640, 480, 16)
    r = {"workload": "C1: 640x480 mono, 8 levels, 1000 features (GPU: batch of pan-sequence frames, extract + "
                     "match vs previous frame)"}
    r.update(extract_match_gpu_leg(dev, local, seq, 1000, reps=frames))
    # single-frame host API (H2D + extract + D2H, synchronous): the reference's calling convention
    ex = ORBextractor(ORBextractor.Parameters(1000), device=local)
    imgs = [seq[i] for i in range(16)]
    for i in range(10):
        ex.Extract(imgs[i % 16])
    lat = []
    for i in range(200):
        t0 = time.perf_counter()
        ex.Extract(imgs[i % 16])
        lat.append(time.perf_counter() - t0)
    r["gpu_single_frame_extract_ms_median"] = 1e3 * float(np.median(lat))
    if cpu:
        from orb_slam2_refactored_amd.synth import synth_image
        O = oracle()
        p = O.params(1000)
        cimgs = [synth_image(s, 640, 480) for s in range(16)]
        for i in range(10):
            O.extract(p, cimgs[i % 16])
        t = []
        for i in range(200):
            t0 = time.perf_counter()
            O.extract(p, cimgs[i % 16])
            t.append(time.perf_counter() - t0)
        med = float(np.median(t))
        r["cpu_baseline"] = {"value": 1.0 / med, "unit": "frames/s", "cores": 1, "kind": "port",
                             "median_ms": 1e3 * med, "p90_ms": 1e3 * float(np.percentile(t, 90)),
                             "sample": "median of 200 single-frame Extract calls, seeds 0-15, 10 warm-ups, "
                                       "oracle/orb_oracle.cpp, 1 thread", "cpu_model": (info or {}).get("cpu_model")}
    return r


def c2_textured_leg(dev, local, frames=1024, cpu=True, info=None):
    """C2 on texture-rich frames: FAST fires almost everywhere, thousands of quadtree candidates per
    level (the LDS-resident path holds 2048; beyond it the global-memory fallback runs)."""
    from orb_slam2_refactored_amd.synth import textured_image
    seq = np.stack([textured_image(4000 + i, 1280, 720) for i in range(16)])
    r = {"workload": "C2 on textured 1280x720 frames (value noise + sigma-12 pixel noise), 2000 features, "
                     "extract + match vs previous frame"}
    r.update(extract_match_gpu_leg(dev, local, seq, 2000, reps=frames, issue_kind="textured"))
    if cpu:
        r["cpu_baseline"] = cpu_baseline_block("frames/s", "textured 1280x720 frames, extract + match vs previous",
                                               cpu_extract_match(seq[:4], 2000, 1, 4.0),
                                               cpu_extract_match(seq[:8], 2000, info["threads_all"], 4.0), info)
    return r


def c2_1000_leg(dev, local, frames=1024, cpu=True, info=None):
    """The metric string's feature count: C2's pan sequence at 1000 features (the headline line runs
    configs[1] at 2000, the larger configuration)."""
    from orb_slam2_refactored_amd.synth import pan_sequence
    seq = pan_sequence(0, 1280, 720, 16)
    r = {"workload": "C2 pan sequence at 1000 features (the metric's feature count), 1280x720, 8 levels, "
                     "extract + match vs previous frame"}
    r.update(extract_match_gpu_leg(dev, local, seq, 1000, reps=frames))
    if cpu:
        r["cpu_baseline"] = cpu_baseline_block("frames/s", "1280x720 pan-sequence frames at 1000 features, "
                                               "extract + match vs previous",
                                               cpu_extract_match(seq[:4], 1000, 1, 4.0),
                                               cpu_extract_match(seq[:8], 1000, info["threads_all"], 4.0), info)
    return r


def c3_leg(dev, local, pairs=128, steps=10, cpu=True, info=None):
    """configs[2]: stereo 1242x375 (8 depth bands, KITTI bf), extract L and R (one batched launch set of
    2 x pairs frames) + SearchForTriangulation(KF1 = L @ [I|0], KF2 = R @ [I|(-bf/fx,0,0)], F12 from
    ComputeF12, onlyStereo false, uright -1, no MapPoints, a single BoW node) per pair, all on the
    device (orbm_search_for_triangulation_batch_device on the extractor's slots)."""
    import torch
    from orb_slam2_refactored_amd import ORBextractor
    from orb_slam2_refactored_amd.matcher import search_for_triangulation_batch_device
    from orb_slam2_refactored_amd.synth import stereo_pair, stereo_tri_geometry
    pool = [stereo_pair(7000 + i)[:2] for i in range(8)]
    Lh = np.stack([pool[i % 8][0] for i in range(pairs)])
    Rh = np.stack([pool[i % 8][1] for i in range(pairs)])
    frames = torch.from_numpy(np.concatenate([Lh, Rh])).to(dev)
    ex = ORBextractor(ORBextractor.Parameters(2000), device=local)
    F12, ep2 = stereo_tri_geometry()
    Ft = torch.from_numpy(np.tile(F12, (pairs, 1))).to(dev)
    Et = torch.from_numpy(np.tile(ep2, (pairs, 1))).to(dev)
    f1 = torch.arange(pairs, dtype=torch.int32, device=dev)
    f2 = f1 + pairs
    scale, sigma2 = ex.GetScaleFactors(), ex.GetScaleSigmaSquares()
    kps, desc, cnt = ex.extract_batch_device(frames)
    tri = search_for_triangulation_batch_device(kps, desc, cnt, kps, desc, cnt, Ft, Et, scale, sigma2,
                                                frame1=f1, frame2=f2)
    st = torch.cuda.current_stream()

    def do_tri():
        search_for_triangulation_batch_device(kps, desc, cnt, kps, desc, cnt, Ft, Et, scale, sigma2, frame1=f1,
                                              frame2=f2, out=tri, stream=st)

    def step():
        ex.extract_batch_device(frames, kps, desc, cnt, stream=st)
        do_tri()

    step()
    torch.cuda.synchronize()
    ms = event_ms(step, steps, st)
    tri_ms = event_ms(do_tri, steps, st)
    ex.profile(True)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    ex.profile(False)
    brk = ex.profile_read()
    ex.batch_status()
    n = cnt.cpu().numpy().astype(np.float64)
    cand = float((n[:pairs] * n[pairs:]).sum())   # query x candidate pairs scanned per step
    W, H = 1242, 375
    n_kp = float(n.mean())
    fb = stage_bytes(W, H, n_kp)["fast_cells"] * 2 * pairs
    fms = brk["fast_cells"][0] / max(brk["fast_cells"][1], 1)
    bytes_pair = 2 * algorithmic_bytes(W, H, n_kp)[0]
    r = {"workload": "C3: stereo 1242x375 (KITTI-shaped synthetic, 8 depth bands), 2000 features, extract L+R + "
                     "SearchForTriangulation (single BoW node), per stereo pair",
         "pairs_per_step": pairs, "pairs_per_s": pairs / (ms * 1e-3), "ms_per_step": ms,
         "triangulation_ms_per_step": tri_ms, "extract_stage_ms_per_step": {k: v[0] / 3 for k, v in brk.items()},
         "keypoints_per_frame": n_kp, "matches_per_pair": float(tri[1].double().mean().item()),
         "roofline": {"bound": "hbm", "kernel": "fast_cells", "achieved": fb / (fms * 1e-3) / 1e9 if fms else 0.0,
                      "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": fb / (fms * 1e-3) / 1e9 / HBM_PEAK_GBS if fms else 0.0,
                      "algorithmic_bytes_per_launch": fb, "avg_launch_ms": fms,
                      "pipeline_algorithmic_GBs": bytes_pair * pairs / (ms * 1e-3) / 1e9},
         # tri_mm_kernel: a query x candidate pair is a 256-bit dot product on the FP4 matrix path
         # (2 x 256 = 512 flops of v_mfma_scale_f32_16x16x128_f8f6f4), plus the d <= TH_LOW events
         "triangulation_roofline": {"bound": "mfma", "kernel": "tri_mm_kernel",
                                    "achieved": 512 * cand / (tri_ms * 1e-3) / 1e12, "peak": FP4_PEAK_TFLOPS,
                                    "unit": "TFLOP/s (FP4)", "frac": 512 * cand / (tri_ms * 1e-3) / 1e12 / FP4_PEAK_TFLOPS,
                                    "ops": "512 FP4 MFMA flops per query x candidate (256 bits)",
                                    "pairs_per_launch": cand}}
    if cpu:
        O = oracle()
        p = O.params(2000)

        def work(stop):
            k = 0
            i = int.from_bytes(os.urandom(1), "little")
            while time.perf_counter() < stop or k < 1:
                L, R = pool[i % 8]
                kl, dl, _ = O.extract(p, L)
                kr, dr, _ = O.extract(p, R)
                keep = O._Keep()
                one = lambda kk, dd: O.tri_frame(keep, np.ascontiguousarray(np.stack([kk["x"], kk["y"]], 1)),  # noqa
                                                 kk["octave"], np.full(len(kk), -1, np.float32),
                                                 np.zeros(len(kk), np.uint8), dd, np.array([0], np.uint32),
                                                 np.array([0, len(kk)], np.int32), np.arange(len(kk), dtype=np.int32))
                O.search_for_triangulation(one(kl, dl), one(kr, dr), F12, ep2, scale, sigma2, False)
                k += 1
                i += 1
            return k

        r["cpu_baseline"] = cpu_baseline_block("pairs/s", "stereo pairs (extract L + R + SearchForTriangulation)",
                                               run_threads(work, 1, 6.0), run_threads(work, info["threads_all"], 6.0),
                                               info)
    return r


def ba_flops_per_iter(prob):
    """SURVEY §8d F_iter = 380 E_mono + 520 E_stereo + sum_pts (45 + 144k + 108 k(k+1)) + (6P)^3/3 +
    4 (6P)^2 + sum_pts (36k + 18), P = free keyframes, k = observations per point."""
    st = prob["edge_obs"][:, 2] >= 0
    k = np.bincount(prob["edge_point"], minlength=len(prob["points"])).astype(np.float64)
    k = k[k > 0]
    P = int((prob["pose_fixed"] == 0).sum())
    D = 6.0 * P
    return (380.0 * (~st).sum() + 520.0 * st.sum() + (45 + 144 * k + 108 * k * (k + 1)).sum() + D ** 3 / 3 +
            4 * D ** 2 + (36 * k + 18).sum())


def localba_leg(local, calls=20, cpu=True, info=None):
    from orb_slam2_refactored_amd.optimizer import LocalBundleAdjustment
    from orb_slam2_refactored_amd.synth import make_ba_problem
    prob = make_ba_problem(0, n_kf=20, n_pts=3000, n_fixed=2)
    for _ in range(2):   # warm-up (device buffers grown, kernels loaded)
        LocalBundleAdjustment(prob, device=local)
    iters = 0
    lat = []
    for _ in range(calls):
        t0 = time.perf_counter()
        r = LocalBundleAdjustment(prob, device=local)
        lat.append(time.perf_counter() - t0)
        iters += sum(r["iterations"])
    dt = sum(lat)
    f_iter = ba_flops_per_iter(prob)
    ips = iters / dt
    out = {"workload": "C4: 20 KF x 3000 MP (KF0 + 2 fixed cameras), optimize(5) + optimize(10), fp64",
           "iters_per_s": ips, "ms_per_call": 1e3 * dt / calls, "ms_per_call_median": 1e3 * float(np.median(lat)),
           "edges": int(len(prob["edge_point"])), "iterations_per_call": iters / calls,
           "roofline": {"bound": "fp64", "achieved": f_iter * ips / 1e12, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": f_iter * ips / 1e12 / FP64_PEAK_TFLOPS, "flops_per_iter": f_iter,
                        "note": "latency-bound: one 114x114 LDL^T + 5 small launches per LM trial"}}
    if cpu:
        O = oracle()
        it = 0
        n = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 5.0 or n < 2:
            it += sum(O.local_ba(prob)["iterations"])
            n += 1
        d = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": it / d, "unit": "LM iterations/s", "ms_per_call": 1e3 * d / n, "calls": n,
                               "cores": 1, "kind": "port",
                               "sample": "oracle g2o restatement (Eigen-free), 1 thread as g2o without OpenMP",
                               "cpu_model": (info or {}).get("cpu_model")}
    return out


def stereo_leg(dev, local, pairs=64, steps=5):
    """§8f row 1 (ComputeStereoMatches) on C3-shaped pairs, both sides extracted in one batch each."""
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
    st = torch.cuda.current_stream()
    torch.cuda.synchronize()
    ms = event_ms(lambda: stereo_matches_batch_device(exl, exr, outl, outr, bf, base, out=out, stream=st), steps, st)
    matched = float((out[1] > 0).sum().item()) / pairs
    return {"workload": "ComputeStereoMatches on 1242x375 stereo pairs (extracted on the device), 2000 features",
            "pairs_per_step": pairs, "pairs_per_s": pairs / (ms * 1e-3), "stereo_match_ms_per_step": ms,
            "matched_per_pair": matched}


def latency_leg(dev, local, cpu=True, calls=100):
    """Single-call latency at the reference's own call shape (VERDICT r05 "Next round" 5):
    * C2: one 1280x720 frame through the host API `orbx_extract` (ORBextractor::Extract, H2D + extract +
      D2H, synchronous), as Tracking::GrabImageMonocular calls it (System.cc:449-452 for the stereo
      case; one frame per call);
    * C3: one 1242x375 stereo pair as Frame's stereo constructor does it (Frame.cc: the two Extract calls
      on two threads, then ComputeStereoMatches, System.cc:449-461): two handles, two host threads, then
      the host-pyramid `orbm_compute_stereo_matches` on the handles' GetImagePyramid() levels;
    each with the single-thread oracle doing the same work beside it (median of the calls)."""
    import threading
    import torch
    from orb_slam2_refactored_amd import ComputeStereoMatches, ORBextractor
    from orb_slam2_refactored_amd.matcher import ComputeStereoMatchesLast
    from orb_slam2_refactored_amd.synth import KITTI, pan_sequence, stereo_pair
    torch.cuda.synchronize()
    seq = pan_sequence(0, 1280, 720, 16)
    ex = ORBextractor(ORBextractor.Parameters(2000), device=local)
    for i in range(10):
        ex.Extract(seq[i % 16])
    lat = []
    for i in range(calls):
        t0 = time.perf_counter()
        ex.Extract(seq[i % 16])
        lat.append(time.perf_counter() - t0)
    r = {"c2_extract": {"workload": "C2 single frame through orbx_extract (host image in, keypoints + descriptors out)",
                        "calls": calls, "median_ms": 1e3 * float(np.median(lat)), "p90_ms": 1e3 * float(np.percentile(lat, 90))}}
    pairs = [stereo_pair(7000 + i) for i in range(8)]
    bf, base = KITTI["bf"], KITTI["bf"] / KITTI["fx"]
    exl = ORBextractor(ORBextractor.Parameters(2000), device=local)
    exr = ORBextractor(ORBextractor.Parameters(2000), device=local)
    scale = np.asarray(exl.GetScaleFactors(), np.float32)
    inv = np.asarray(exl.GetInverseScaleFactors(), np.float32)
    res = {}

    def side(name, e, img):
        res[name] = e.Extract(img)

    def pair_call(L, R):
        ta = threading.Thread(target=side, args=("L", exl, L))
        tb = threading.Thread(target=side, args=("R", exr, R))
        t0 = time.perf_counter()
        ta.start(); tb.start(); ta.join(); tb.join()
        t1 = time.perf_counter()
        (kl, dl), (kr, dr) = res["L"], res["R"]
        ur, dp = ComputeStereoMatchesLast(exl, exr, len(kl), bf, base)   # the extractors' device-resident data
        t2 = time.perf_counter()
        return t1 - t0, t2 - t1, t2 - t0, float((dp > 0).sum())

    def pair_call_host(L, R):   # the host-pyramid entry point (GetImagePyramid + orbm_compute_stereo_matches)
        t0 = time.perf_counter()
        kl, dl = exl.Extract(L)
        kr, dr = exr.Extract(R)
        t1 = time.perf_counter()
        pl, pr = exl.GetImagePyramid(), exr.GetImagePyramid()
        t2 = time.perf_counter()
        ComputeStereoMatches(kl, dl, pl, kr, dr, pr, scale, inv, bf, base)
        t3 = time.perf_counter()
        return t1 - t0, t2 - t1, t3 - t2, t3 - t0
    for i in range(5):
        pair_call(pairs[i % 8][0], pairs[i % 8][1])
        pair_call_host(pairs[i % 8][0], pairs[i % 8][1])
    rows = [pair_call(pairs[i % 8][0], pairs[i % 8][1]) for i in range(calls // 2)]
    hrows = [pair_call_host(pairs[i % 8][0], pairs[i % 8][1]) for i in range(calls // 4)]
    a, ha = np.array(rows), np.array(hrows)
    r["c3_stereo_pair"] = {
        "workload": "C3 stereo pair 1242x375, 2000 features: Extract L and R on two host threads (two handles), "
                    "then orbx_stereo_matches_last on the extractors' device-resident keypoints / descriptors / "
                    "pyramids (uright / depth back to the host)",
        "calls": len(rows), "median_ms": 1e3 * float(np.median(a[:, 2])),
        "extract_two_threads_median_ms": 1e3 * float(np.median(a[:, 0])),
        "stereo_match_median_ms": 1e3 * float(np.median(a[:, 1])), "matched_per_pair": float(np.mean(a[:, 3])),
        "host_pyramid_path": {
            "workload": "Extract L then R on one thread, GetImagePyramid of both, orbm_compute_stereo_matches on "
                        "the host pyramids (the API for pyramids that are not an extractor's)",
            "calls": len(hrows), "median_ms": 1e3 * float(np.median(ha[:, 3])),
            "extract_sequential_median_ms": 1e3 * float(np.median(ha[:, 0])),
            "get_pyramids_median_ms": 1e3 * float(np.median(ha[:, 1])),
            "stereo_match_median_ms": 1e3 * float(np.median(ha[:, 2]))}}
    if cpu:
        O = oracle()
        p = O.params(2000)
        t = []
        for i in range(12):
            t0 = time.perf_counter()
            O.extract(p, seq[i % 16])
            t.append(time.perf_counter() - t0)
        r["c2_extract"]["cpu_baseline"] = {"median_ms": 1e3 * float(np.median(t[2:])), "cores": 1, "kind": "port",
                                           "sample": "10 single-frame oracle Extract calls after 2 warm-ups, 1 thread"}
        tt = O.scale_tables(p)
        t = []
        for i in range(8):
            L, R = pairs[i % 8][0], pairs[i % 8][1]
            t0 = time.perf_counter()
            kl, dl, _ = O.extract(p, L)
            kr, dr, _ = O.extract(p, R)
            pl, pr = O.pyramid(p, L), O.pyramid(p, R)
            O.compute_stereo_matches(kl, dl, pl, kr, dr, pr, tt["scale"], tt["inv_scale"], bf, base)
            t.append(time.perf_counter() - t0)
        r["c3_stereo_pair"]["cpu_baseline"] = {
            "median_ms": 1e3 * float(np.median(t[2:])), "cores": 1, "kind": "port",
            "sample": "6 stereo pairs after 2 warm-ups, oracle Extract L then R + ComputeStereoMatches on one thread "
                      "(the pyramid recomputed for the matcher is included)"}
    return r


def pose_leg(dev, frames=1024, edges=1000, steps=10, cpu=True):
    """§8f row 3: batched PoseOptimization (Optimizer.cc:345-489), inputs resident in HBM."""
    import torch
    from orb_slam2_refactored_amd.optimizer import pose_optimization_device
    from orb_slam2_refactored_amd.synth import make_pose_batch
    b = make_pose_batch(12, n_frames=frames, n_edges=edges)
    d = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in b.items() if not k.startswith("gt_")}
    out = pose_optimization_device(d)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    ms = event_ms(lambda: pose_optimization_device(d, out=out), steps, st)
    r = {"workload": f"{frames} frames x {edges} edges (40 % stereo, 10 % outliers), 4 x optimize(10), fp64",
         "frames_per_s": frames / (ms * 1e-3), "ms_per_step": ms,
         "mean_inliers": float(out["n_inliers"].double().mean().item())}
    if cpu:
        O = oracle()
        sub = make_pose_batch(13, n_frames=16, n_edges=edges)
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < 3.0 or n < 16:
            O.pose_optimization(sub)
            n += 16
        r["cpu_baseline"] = {"frames_per_s": n / (time.perf_counter() - t0), "cores": 1, "kind": "port",
                             "sample": f"16-frame batches of {edges} edges, oracle/orb_oracle.cpp, 1 thread"}
    return r


def projection_leg(dev, frames=256, steps=10, cpu=True):
    """§8f row 2: batched SearchByProjection + FeaturesGrid: 2000 keypoints / 1500 map points per frame."""
    import torch
    from orb_slam2_refactored_amd.matcher import search_by_projection_device
    from orb_slam2_refactored_amd.synth import make_proj_batch, tile_proj_batch
    base = make_proj_batch(21, n_frames=16, n_kp=2000, n_mp=1500)
    b = tile_proj_batch(base, frames // 16)
    d = {k: (torch.from_numpy(np.ascontiguousarray(v)).to(dev) if isinstance(v, np.ndarray) and k != "scale_factors"
             else v) for k, v in b.items()}
    km, nm = search_by_projection_device(d)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    ms = event_ms(lambda: search_by_projection_device(d, km, nm), steps, st)
    r = {"workload": f"{frames} frames x (2000 keypoints, 1500 map points), th 1, grid + score + claim walk",
         "frames_per_s": frames / (ms * 1e-3), "ms_per_step": ms, "mean_matches": float(nm.double().mean().item())}
    if cpu:
        O = oracle()
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < 3.0 or n < 16:
            O.search_by_projection(base)
            n += 16
        r["cpu_baseline"] = {"frames_per_s": n / (time.perf_counter() - t0), "cores": 1, "kind": "port",
                             "sample": "16-frame batches, oracle/orb_oracle.cpp, 1 thread"}
    r["motion_model"] = motion_projection_leg(dev, base, b, frames, steps, cpu)
    return r


def motion_projection_leg(dev, base, b, frames, steps, cpu):
    """SearchByProjection(Frame&, const Frame&, th 7, stereo) (ORBmatcher.cc:1279-1362) on the same
    frames: the 1500 points play the last frame's (octave = trackScaleLevel), CheckOrientation on."""
    import torch
    from orb_slam2_refactored_amd.matcher import search_by_projection_motion_device

    def motion(src, seed):
        rng = np.random.default_rng(seed)
        K, M = int(src["kp_begin"][-1]), int(src["mp_begin"][-1])
        F = len(src["kp_begin"]) - 1
        return dict(kp_begin=src["kp_begin"], kp_xy=src["kp_xy"], kp_octave=src["kp_octave"],
                    kp_uright=src["kp_uright"], kp_desc=src["kp_desc"],
                    kp_angle=((40 + rng.normal(0, 4, K)) % 360).astype(np.float32), kp_claimed=None,
                    bounds=src["bounds"], mp_begin=src["mp_begin"], mp_valid=src["mp_valid"], mp_proj=src["mp_proj"],
                    mp_octave=np.minimum(src["mp_level"], 7).astype(np.int32), mp_desc=src["mp_desc"],
                    mp_has_obs=src["mp_has_obs"], mp_angle=((45 + rng.normal(0, 4, M)) % 360).astype(np.float32),
                    motion=(np.arange(F) % 3).astype(np.int32), scale_factors=src["scale_factors"], th=7.0,
                    check_orientation=1)
    mb = motion(b, 5)
    d = {k: (torch.from_numpy(np.ascontiguousarray(v)).to(dev) if isinstance(v, np.ndarray) and k != "scale_factors"
             else v) for k, v in mb.items()}
    km, nm = search_by_projection_motion_device(d)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    ms = event_ms(lambda: search_by_projection_motion_device(d, km, nm), steps, st)
    r = {"workload": f"{frames} frames x (2000 keypoints, 1500 last-frame points), th 7, forward / backward / "
                     "neither level windows, CheckOrientation on",
         "frames_per_s": frames / (ms * 1e-3), "ms_per_step": ms, "mean_matches": float(nm.double().mean().item())}
    if cpu:
        O = oracle()
        mb0 = motion(base, 6)
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < 3.0 or n < 16:
            O.search_by_projection_motion(mb0)
            n += 16
        r["cpu_baseline"] = {"frames_per_s": n / (time.perf_counter() - t0), "cores": 1, "kind": "port",
                             "sample": "16-frame batches, oracle/orb_oracle.cpp, 1 thread"}
    return r


def reloc_leg(dev, frames=256, steps=10, cpu=True):
    """Relocalisation SearchByProjection(Frame&, KeyFrame*, alreadyFound, th 10, ORBdist 100)
    (ORBmatcher.cc:1364-1445, Tracking.cc:403): 256 (frame, candidate keyframe) pairs, 2000 keypoints and
    600 keyframe points each, CheckOrientation on."""
    import torch
    from orb_slam2_refactored_amd.matcher import search_by_projection_reloc_device
    from orb_slam2_refactored_amd.synth import make_reloc_batch, tile_ragged_batch
    b = tile_ragged_batch(make_reloc_batch(41, n_frames=16, n_kp=2000, n_mp=600), frames // 16)
    d = {k: (torch.from_numpy(np.ascontiguousarray(v)).to(dev) if isinstance(v, np.ndarray) and k != "scale_factors"
             else v) for k, v in b.items()}
    km, nm = search_by_projection_reloc_device(d)
    torch.cuda.synchronize()
    ms = event_ms(lambda: search_by_projection_reloc_device(d, km, nm), steps, torch.cuda.current_stream())
    r = {"workload": f"{frames} (frame, keyframe) pairs x (2000 keypoints, 600 keyframe points), th 10, ORBdist 100, "
                     "projection + invariance gate + PredictScale + claim walk, CheckOrientation on",
         "pairs_per_s": frames / (ms * 1e-3), "ms_per_step": ms, "mean_matches": float(nm.double().mean().item())}
    if cpu:
        O = oracle()
        b8 = make_reloc_batch(42, n_frames=8, n_kp=2000, n_mp=600)
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < 3.0 or n < 8:
            O.search_by_projection_reloc(b8)
            n += 8
        r["cpu_baseline"] = {"pairs_per_s": n / (time.perf_counter() - t0), "cores": 1, "kind": "port",
                             "sample": "8-pair batches, oracle/orb_oracle.cpp, 1 thread"}
    return r


def init_leg(dev, pairs=64, steps=10, cpu=True):
    """SearchForInitialization(F1, F2, prevMatched, matches12, windowSize 100) with ORBmatcher(0.9, true)
    (ORBmatcher.cc:614-694, Tracking.cc:1050-1052): 64 pairs of 4000-keypoint frames.  prevMatched is
    updated in place by each call, so every timed call first restores it (one 2 x 4 B x 256k device copy,
    inside the timing)."""
    import torch
    from orb_slam2_refactored_amd.matcher import search_for_initialization_device
    from orb_slam2_refactored_amd.synth import make_init_batch, tile_ragged_batch
    b = tile_ragged_batch(make_init_batch(43, n_pairs=8), pairs // 8)
    d = {k: (torch.from_numpy(np.ascontiguousarray(v)).to(dev) if isinstance(v, np.ndarray) else v)
         for k, v in b.items()}
    pm0 = d["prev_matched"].clone()
    m12, nm = search_for_initialization_device(d)
    torch.cuda.synchronize()

    def call():
        d["prev_matched"].copy_(pm0)
        search_for_initialization_device(d, m12, nm)
    ms = event_ms(call, steps, torch.cuda.current_stream())
    r = {"workload": f"{pairs} pairs x (4000 + 4000 keypoints), window 100, nnratio 0.9, CheckOrientation on",
         "pairs_per_s": pairs / (ms * 1e-3), "ms_per_step": ms, "mean_matches": float(nm.double().mean().item())}
    if cpu:
        O = oracle()
        b4 = make_init_batch(44, n_pairs=4)
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < 3.0 or n < 4:
            O.search_for_initialization(b4)
            n += 4
        r["cpu_baseline"] = {"pairs_per_s": n / (time.perf_counter() - t0), "cores": 1, "kind": "port",
                             "sample": "4-pair batches, oracle/orb_oracle.cpp, 1 thread"}
    return r


def bow_leg(dev, local, frames=128, n=2000, steps=10, cpu=True):
    """§8f row 4: ORBVocabulary::transform(desc, BowVector, FeatureVector, 4) on an ORBvoc-shaped
    synthetic tree (k 10, L 6, 1.1 M nodes)."""
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
    st = torch.cuda.current_stream()
    ms = event_ms(lambda: voc.transform_batch_device(desc, counts, out=out), steps, st)
    r = {"workload": f"{frames} frames x {n} descriptors, vocabulary k 10 L 6 (1.11 M nodes), levelsup 4",
         "frames_per_s": frames / (ms * 1e-3), "ms_per_step": ms, "mean_words": float(out["n_words"].double().mean().item())}
    if cpu:
        O = oracle()
        o = O.Vocabulary(v)
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < 3.0 or k < 8:
            o.transform(X[k % frames], 4)
            k += 1
        r["cpu_baseline"] = {"frames_per_s": k / (time.perf_counter() - t0), "cores": 1, "kind": "port",
                             "sample": f"{n}-descriptor sets, oracle/orb_oracle.cpp, 1 thread"}
    r["search_by_bow"] = search_by_bow_leg(dev, X, out, voc, steps, cpu)
    return r


def search_by_bow_leg(dev, X, fv1_out, voc, steps, cpu):
    """SearchByBoW(KeyFrame*, Frame&) (ORBmatcher.cc:452-516): pair p = keyframe p (the bow leg's
    descriptors) against a frame holding the same features with 8 of 256 bits flipped, both
    FeatureVectors from the device transform (levelsup 4), CheckOrientation on (random angles)."""
    import torch
    from orb_slam2_refactored_amd.matcher import search_by_bow_batch_device
    frames, n = X.shape[0], X.shape[1]
    rng = np.random.default_rng(33)
    flip = np.zeros((frames, n, 256), np.uint8)
    pos = rng.integers(0, 256, size=(frames, n, 8))
    np.put_along_axis(flip, pos, 1, axis=2)
    X2 = X ^ np.packbits(flip, axis=2)
    desc1 = torch.from_numpy(X).to(dev)
    desc2 = torch.from_numpy(X2).to(dev)
    counts = torch.full((frames,), n, dtype=torch.int32, device=dev)
    fv2_out = voc.transform_batch_device(desc2, counts)
    kp = np.zeros((frames, n, 7), np.float32)
    kp[:, :, 3] = rng.random((frames, n)) * 360
    kp2 = kp.copy()
    kp2[:, :, 3] = (kp[:, :, 3] + rng.normal(0, 3, (frames, n))) % 360
    kps1 = torch.from_numpy(kp.view(np.int32)).to(dev)
    kps2 = torch.from_numpy(kp2.view(np.int32)).to(dev)
    fv = lambda o: (o["fv_node"], o["fv_off"], o["fv_idx"], o["n_nodes"])   # noqa: E731
    out = search_by_bow_batch_device(kps1, desc1, fv(fv1_out), kps2, desc2, counts, fv(fv2_out), checkOri=True)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    ms = event_ms(lambda: search_by_bow_batch_device(kps1, desc1, fv(fv1_out), kps2, desc2, counts, fv(fv2_out),
                                                     checkOri=True, out=out), steps, st)
    r = {"workload": f"{frames} (keyframe, frame) pairs x {n} features, FeatureVectors at levelsup 4 of the "
                     "k 10 L 6 vocabulary, 8-bit-flipped frame descriptors, CheckOrientation on",
         "pairs_per_s": frames / (ms * 1e-3), "ms_per_step": ms,
         "mean_matches": float(out[1].double().mean().item())}
    if cpu:
        O = oracle()
        h1 = [t.cpu().numpy() for t in fv(fv1_out)]
        h2 = [t.cpu().numpy() for t in fv(fv2_out)]

        def frame(keep, h, D, p, mp):
            node, off, idx, nn = h
            k = int(nn[p])
            o = off[p, :k + 1]
            z = np.zeros(n, np.float32)
            return O.tri_frame(keep, np.zeros((n, 2), np.float32), np.zeros(n, np.int32), z, mp, D[p],
                               node[p, :k].astype(np.uint32), o, idx[p, :o[-1]])

        ones = np.ones(n, np.uint8)
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < 3.0 or k < 8:
            p = k % frames
            keep = O._Keep()
            O.search_by_bow(frame(keep, h1, X, p, ones), frame(keep, h2, X2, p, ones), kp[p, :, 3], kp2[p, :, 3],
                            0.6, True)
            k += 1
        r["cpu_baseline"] = {"pairs_per_s": k / (time.perf_counter() - t0), "cores": 1, "kind": "port",
                             "sample": "single pairs, oracle/orb_oracle.cpp, 1 thread (FeatureVectors given)"}
    return r


# ------------------------------------------------------------------------------------------ ranks
class _StubExtractor:
    """CPU stand-in used ONLY by `--stub` (tests/test_bench_launcher.py drives the N > 1 launcher and the
    exchange over gloo without a GPU).  Fills the slots deterministically from the frame index; a stub
    run says so in its JSON line ("stub": true) and is never a measurement."""

    def __init__(self, nfeat):
        self.cap = 48
        self._on, self._launches = False, 0

    def max_keypoints(self, rows, cols):
        return self.cap

    def extract_batch_device(self, frames, kps, desc, counts, stream=None):
        import torch
        g = frames.to(torch.int64)                         # global frame indices of this shard
        counts.copy_(((g * 7 + 3) % (self.cap + 1)).to(torch.int32))
        r = torch.arange(self.cap, dtype=torch.int64)
        desc.copy_(((g[:, None, None] * 131 + r[None, :, None] * 17 + torch.arange(32)[None, None, :]) % 251)
                   .to(torch.uint8))
        kps.zero_()
        if self._on:
            self._launches += 1

    def profile(self, enable=True, stages=None):
        self._on, self._launches = enable, (0 if enable else self._launches)

    def profile_read(self):
        n = self._launches
        return {"pyramid": (0.0, 4 * n), "fast_cells": (0.0, n), "quadtree": (0.0, n), "describe": (0.0, n)}

    def batch_status(self, stream=None):
        return 0


class _StubMatcher:
    def match_batch_device(self, descA, nA, descB, nB, out=None, stream=None, pair_b=None):
        out.fill_(-1)
        return out


class Ranks:
    """One process per GPU (torch.distributed over RCCL) or, with `stub`, CPU processes over gloo."""

    def __init__(self, stub: bool):
        import torch
        import torch.distributed as dist
        self.stub = stub
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if stub:
            self.dev = torch.device("cpu")
        else:
            torch.cuda.set_device(self.local)
            self.dev = torch.device("cuda", self.local)
        if self.world > 1:
            if stub:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=self.dev)
            if dist.get_world_size() != self.world:
                raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, WORLD_SIZE {self.world}")

    def sync(self):
        if not self.stub:
            import torch
            torch.cuda.synchronize()

    def barrier(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.barrier()

    def stream(self):
        if self.stub:
            return None
        import torch
        return torch.cuda.current_stream()

    def max(self, x: float) -> float:
        if self.world == 1:
            return x
        import torch
        import torch.distributed as dist
        t = torch.tensor([x], dtype=torch.float64, device=self.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x: float) -> float:
        if self.world == 1:
            return x
        import torch
        import torch.distributed as dist
        t = torch.tensor([x], dtype=torch.float64, device=self.dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()


def count_gpus_kfd() -> int:
    """GPUs visible to this process, counted from the KFD topology in sysfs (a node with SIMDs is a GPU),
    restricted by HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES when set.  No HIP
    or torch call: the launcher never initialises the GPU runtime before it starts the rank processes."""
    n = 0
    nodes = Path("/sys/class/kfd/kfd/topology/nodes")
    try:
        for d in nodes.iterdir():
            try:
                props = (d / "properties").read_text()
            except OSError:
                continue
            for line in props.splitlines():
                k, _, v = line.partition(" ")
                if k == "simd_count" and int(v or 0) > 0:
                    n += 1
    except OSError:
        return 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        vis = os.environ.get(var)
        if vis is not None:
            n = min(n, len([x for x in vis.split(",") if x.strip() != ""]))
    return n


def launch_ranks(args) -> int:
    """`bench.py --gpus N` without a launcher: start N fresh rank processes, rank 0's stdout is the JSON line.
    This process never touches the GPU runtime: it counts GPUs from sysfs (count_gpus_kfd, no HIP / torch
    call) and starts children rather than exec'ing.  The driver's own form -- torch.distributed.run
    setting WORLD_SIZE / RANK / LOCAL_RANK -- runs the same rank code directly."""
    import socket
    import subprocess
    n = args.gpus
    if not args.stub:
        have = count_gpus_kfd()
        if have < n:
            print(f"bench.py: --gpus {n} but only {have} GPU(s) visible", file=sys.stderr, flush=True)
            return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, WORLD_SIZE=str(n), RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in pending:      # one rank failed: the others would wait in a collective forever
                        q.terminate()
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


# ------------------------------------------------------------------------------------------ sharded steps
class ShardedRun:
    """The C2 / C5 step on this rank: extract B frames of the global pan sequence (rank r holds global frames
    r*B .. r*B+B-1), match frames 1.. of the shard against their in-shard predecessor, and -- with the
    exchange -- all-gather per-frame counts and the Σn x 32 B descriptor block, matching the shard's first
    frame against rank r-1's last frame from the gathered block one step later."""

    def __init__(self, ranks, ex, m, base, B, exchange):
        import torch
        from orb_slam2_refactored_amd.shard import CompactExchange, Slots, cross_shard_predecessor, shard_range
        self.ranks, self.ex, self.m, self.B = ranks, ex, m, B
        world, rank, dev = ranks.world, ranks.rank, ranks.dev
        H, W = base.shape[1:]
        self.g0, _ = shard_range(B * world, world, rank)
        gidx = torch.arange(self.g0, self.g0 + B)
        if ranks.stub:
            self.frames = gidx                      # the stub extractor derives its output from the index
        else:
            # frame g = base[g % 16]; every frame its own buffer in HBM (8192 x 0.92 MB >> the 256 MB MALL)
            self.frames = torch.from_numpy(base).to(dev)[(gidx % len(base)).to(dev)].contiguous()
        self.cap = ex.max_keypoints(H, W)
        self.match_out = torch.empty((4, B, self.cap), dtype=torch.int32, device=dev)
        self.prev_idx = torch.arange(0, B - 1, dtype=torch.int32, device=dev)
        self.pred = cross_shard_predecessor(rank, world, B) if world > 1 else -1
        if exchange:
            self.xchg = CompactExchange(B, self.cap, dev)
            self.cross_out = torch.full((4, 1, self.cap), -1, dtype=torch.int32, device=dev)
            self.single = None
        else:
            self.xchg = None
            self.single = Slots.empty(B, self.cap, dev)
        self.k = 0
        self.cross = 0          # cross-shard matches run
        self.matched = -1       # last step whose cross-shard match ran (each step's runs once)
        self.stream = ranks.stream()

    def slots(self):
        return self.single if self.xchg is None else self.xchg.local(max(self.k - 1, 0))

    def _cross_match(self, j):
        import torch
        if j == self.matched:
            return
        self.matched = j
        self.xchg.wait(j)
        if self.ranks.rank == 0:
            return
        pb = self.xchg.frame(j, self.ranks.rank - 1, self.B - 1)
        n = int(pb.shape[0])
        if n == 0:
            return
        loc = self.xchg.local(j)
        nb = torch.full((1,), n, dtype=torch.int32, device=self.ranks.dev)
        self.m.match_batch_device(loc.desc[0:1], loc.counts[0:1], pb.reshape(1, n, 32), nb, out=self.cross_out,
                                  stream=self.stream)
        self.cross += 1

    def step(self):
        B, st = self.B, self.stream
        if self.xchg is None:
            s = self.single
            self.ex.extract_batch_device(self.frames, s.kps, s.desc, s.counts, stream=st)
            if B > 1:
                self.m.match_batch_device(s.desc[1:], s.counts[1:], s.desc, s.counts, out=self.match_out[:, 1:],
                                          stream=st, pair_b=self.prev_idx)
            self.k += 1
            return
        k = self.k
        loc = self.xchg.local(k)
        self.ex.extract_batch_device(self.frames, loc.kps, loc.desc, loc.counts, stream=st)
        if B > 1:
            self.m.match_batch_device(loc.desc[1:], loc.counts[1:], loc.desc, loc.counts, out=self.match_out[:, 1:],
                                      stream=st, pair_b=self.prev_idx)
        had = self.xchg.pending
        self.xchg.publish(k)
        if had is not None:
            self._cross_match(had)
        self.k = k + 1

    def finish(self):
        if self.xchg is not None and self.xchg.pending is not None:
            j = self.xchg.pending
            self.xchg.drain()
            self._cross_match(j)

    def timed(self, steps, warmup, profile_stage=None):
        """W untimed steps, then exactly `steps` steps between barrier + synchronize on both sides;
        returns the max over ranks of the timed region (s) and, with `profile_stage`, the live HIP-event
        launch times of that stage inside the timed region."""
        for _ in range(warmup):
            self.step()
        self.finish()
        self.ranks.sync()
        self.ranks.barrier()
        self.ranks.sync()
        if profile_stage:
            self.ex.profile(True, stages=[profile_stage])
        t0 = time.perf_counter()
        for _ in range(steps):
            self.step()
        self.finish()
        self.ranks.sync()
        self.ranks.barrier()
        self.ranks.sync()
        elapsed = time.perf_counter() - t0
        prof = None
        if profile_stage:
            self.ex.profile(False)
            prof = self.ex.profile_read()
        self.fault = self.ex.batch_status()   # raises if a device capacity check tripped in the timed steps
        return self.ranks.max(elapsed), prof

    def exchange_block(self, steps):
        """The exchange's numbers over the last `steps` steps (gathered bytes, gather time, xGMI bounds)."""
        import numpy as np
        x, world = self.xchg, self.ranks.world
        if not self.ranks.stub:
            x.collect_gather_times()
        pay = x.payload_bytes[-steps:] if x.payload_bytes else [0]
        gms = x.gather_ms[-steps:] if x.gather_ms else [0.0]
        per_step = float(np.mean(pay)) + world * self.B * 4   # payload + counts
        recv = per_step * (world - 1) / world                  # bytes each rank receives
        g = float(np.mean(gms))
        return {"gather_bytes_per_step": per_step, "received_bytes_per_rank_per_step": recv,
                "padded_slot_gather_bytes_per_step": (self.cap * (28 + 32) + 4) * self.B * world,
                "gather_ms_per_step": g, "gather_ms_max_over_ranks": self.ranks.max(g),
                "gather_GBs_received_per_rank": recv / (g * 1e-3) / 1e9 if g else None,
                "xgmi_bound_ms": {"all_7_links": recv / (7 * 153e9) * 1e3, "single_link": recv / 153e9 * 1e3},
                "cross_shard_predecessor": self.pred,
                "cross_match_first_frame_matches": (int((self.cross_out[3] >= 0).sum().item())
                                                    if self.ranks.rank > 0 else None),
                "cross_matches_run": self.cross,
                "cross_shard_matches_all_ranks": int(self.ranks.sum(
                    float((self.cross_out[3] >= 0).sum().item()) if self.ranks.rank > 0 else 0.0)),
                "cross_matches_run_all_ranks": int(self.ranks.sum(float(self.cross)))}


def c5_leg(ranks, ex, m, base, total=1024, steps=20, warmup=3, nfeat=2000):
    """configs[4]: 1024 independent 1280x720 frames per step in total, sharded over the N ranks (1024/N per
    rank: the fixed-size job of C5, i.e. strong scaling), extract + match vs predecessor + the counts /
    descriptor all-gather and the cross-shard predecessor match.  Runs on every rank (collectives); at N = 1
    it runs the same exchange path as the curve's first point."""
    if total % ranks.world:
        raise SystemExit(f"bench.py: C5's {total} frames do not split over {ranks.world} ranks")
    B = total // ranks.world
    run = ShardedRun(ranks, ex, m, base, B, exchange=True)
    elapsed, _ = run.timed(steps, warmup)
    H, W = base.shape[1:]
    ms = 1e3 * elapsed / steps
    # the extractor's algorithmic bytes (SURVEY §8d B_ext) of all ranks' frames over the whole step, against
    # N x the per-GPU HBM peak: the north star's "fraction of HBM roofline" at this N
    n_kp = ranks.sum(float(run.slots().counts.float().sum().item())) / total
    bytes_frame, _ = algorithmic_bytes(W, H, n_kp)
    gbs = bytes_frame * total / (ms * 1e-3) / 1e9
    out = {"workload": f"C5 (configs[4]): {total} {W}x{H} frames per step in total, {B} per rank on "
                       f"{ranks.world} rank(s), extract + match vs predecessor, RCCL counts + descriptor "
                       "all-gather, cross-shard predecessor match",
           "frames_per_step": total, "frames_per_rank": B, "n_ranks": ranks.world, "scaling": "strong",
           "steps": steps, "warmup": warmup, "frames_per_s": total * steps / elapsed,
           "ms_per_step": ms, "keypoints_per_frame": n_kp, "keypoint_quota": nfeat,
           "hbm_frac": gbs / (HBM_PEAK_GBS * ranks.world),
           "hbm": {"algorithmic_bytes_per_frame": bytes_frame, "GBs_all_ranks": gbs,
                   "peak_GBs_all_ranks": HBM_PEAK_GBS * ranks.world,
                   "note": "extractor algorithmic bytes (SURVEY §8d B_ext) x frames / ms_per_step over N x peak"}}
    out.update(run.exchange_block(steps))
    return out


def c5_per_rank_leg(ranks, ex, m, base, per_rank=128, n_project=8, steps=20, warmup=3):
    """C5 (configs[4]) as ONE rank of the N = 8 job sees it, measured on this one GPU (VERDICT r05 "Next
    round" 5): 1024 / 8 = 128 frames per step through the exchange path (pack, counts / payload gather,
    cross-shard match; the same code as N > 1, with a world of 1), next to the xGMI time of the gather the
    eight ranks would do: each rank receives 7/8 of 8 x this rank's measured payload.  The projection
    assumes the gather overlaps the next step's kernels (it runs on the process group's stream) or, as a
    bound, that it serialises behind one link."""
    run = ShardedRun(ranks, ex, m, base, per_rank, exchange=True)
    elapsed, _ = run.timed(steps, warmup)
    ms = 1e3 * elapsed / steps
    blk = run.exchange_block(steps)
    payload_rank = blk["gather_bytes_per_step"] - ranks.world * per_rank * 4   # this rank's descriptor block
    gathered = n_project * (payload_rank + per_rank * 4)
    recv = gathered * (n_project - 1) / n_project
    x7, x1 = recv / (7 * 153e9) * 1e3, recv / 153e9 * 1e3
    return {"workload": f"C5 per-rank share at N = {n_project}: {per_rank} 1280x720 frames per step on this GPU, "
                        "extract + match vs predecessor + the exchange path (world of 1)",
            "frames_per_rank": per_rank, "steps": steps, "warmup": warmup, "ms_per_step": ms,
            "frames_per_s_this_rank": per_rank * steps / elapsed,
            "payload_bytes_per_rank_per_step": payload_rank,
            "projected_n": n_project, "projected_gather_bytes_per_step": gathered,
            "projected_received_bytes_per_rank": recv,
            "xgmi_bound_ms": {"all_7_links": x7, "single_link": x1},
            "projected_job_frames_per_s": {
                "gather_overlapped": n_project * per_rank / (max(ms, x7) * 1e-3),
                "gather_serial_single_link": n_project * per_rank / ((ms + x1) * 1e-3)},
            "gather_ms_local": blk["gather_ms_per_step"]}


# ------------------------------------------------------------------------------------------ main
def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks, one per GPU: started here when no launcher set WORLD_SIZE; must equal WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=8192, help="frames per step per GPU (weak scaling: the job is frames x world)")
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--force-exchange", action="store_true",
                    help="run the N > 1 exchange path (pack, counts / payload gather, cross-shard match) at N = 1 too")
    ap.add_argument("--no-legs", action="store_true", help="only the headline C2 measurement (and C5)")
    ap.add_argument("--c5-frames", type=int, default=1024, help="C5's total frames per step (configs[4]: 1024)")
    ap.add_argument("--stub", action="store_true",
                    help="CPU test of the launcher / exchange only: gloo, stub extraction, no GPU, no measurement")
    for leg in ("c1", "textured", "c3", "ba", "stereo", "pose", "projection", "bow", "c5", "latency", "c5n8"):
        ap.add_argument(f"--no-{leg}", action="store_true")
    return ap.parse_args(argv)


def main():
    args = parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)", file=sys.stderr, flush=True)
        sys.exit(2)
    if not args.stub:
        import torch
        have = torch.cuda.device_count()
        if int(os.environ.get("LOCAL_RANK", "0")) >= have:
            print(f"bench.py: LOCAL_RANK {os.environ.get('LOCAL_RANK')} but {have} GPU(s) visible", file=sys.stderr,
                  flush=True)
            sys.exit(2)
    ranks = Ranks(args.stub)
    rank = ranks.rank

    from orb_slam2_refactored_amd.synth import pan_sequence

    W, H = args.width, args.height
    B = args.frames                      # frames per GPU per step (weak scaling)
    total = B * world
    base = pan_sequence(0, W, H, 16)     # the global job: frame g = base[g % 16]
    if args.stub:
        ex, m = _StubExtractor(args.nfeatures), _StubMatcher()
    else:
        from orb_slam2_refactored_amd import ORBextractor, ORBmatcher
        ex = ORBextractor(ORBextractor.Parameters(nfeatures=args.nfeatures), device=ranks.local)
        m = ORBmatcher(0.6, False)
    run = ShardedRun(ranks, ex, m, base, B, exchange=world > 1 or args.force_exchange)
    # inside the timed region only the dominant kernel (fast_cells) carries launch events (events on every
    # kernel cost ~3.5 %); the other stages are timed in a separate pass below
    elapsed, timed = run.timed(args.steps, args.warmup, profile_stage="fast_cells")
    ex.profile(True)
    for _ in range(3):
        run.step()
    run.finish()
    ranks.sync()
    ex.profile(False)
    breakdown = ex.profile_read()
    brk_steps = 3
    # the matcher alone (3 calls on the last step's descriptors), for its FP4 roofline
    match_ms = 0.0
    sl = run.slots()
    if B > 1 and not args.stub:
        import torch
        st = run.stream
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(3):
            m.match_batch_device(sl.desc[1:], sl.counts[1:], sl.desc, sl.counts, out=run.match_out[:, 1:], stream=st,
                                 pair_b=run.prev_idx)
        e1.record(st)
        e1.synchronize()
        match_ms = e0.elapsed_time(e1) / 3

    n_kp = float(sl.counts.float().mean().item())
    matches = int((run.match_out[3] >= 0).sum().item())
    value = total * args.steps / elapsed
    ms_per_step = 1e3 * elapsed / args.steps
    bytes_frame, P = algorithmic_bytes(W, H, n_kp)
    sb = stage_bytes(W, H, n_kp)
    dom = max(breakdown, key=lambda k: breakdown[k][0])
    if dom == "fast_cells":
        dom_ms, dom_launches, dom_steps = timed[dom][0], timed[dom][1], args.steps
    else:
        dom_ms, dom_launches, dom_steps = breakdown[dom][0], breakdown[dom][1], brk_steps
    per_launch_ms = dom_ms / max(dom_launches, 1)
    launches_per_step = dom_launches / max(dom_steps, 1)
    dom_bytes = sb[dom] * B / max(launches_per_step, 1)
    achieved = dom_bytes / (per_launch_ms * 1e-3) / 1e9 if per_launch_ms > 0 else 0.0
    traffic = measured_traffic(dom, B, W, H, args.nfeatures)
    extract_ms = sum(v[0] for k, v in breakdown.items() if k in STAGE_KERNELS) / brk_steps
    pipe_traffic = measured_traffic_step(B, W, H, args.nfeatures)
    match_tflops = 512.0 * n_kp * n_kp * (B - 1) / (match_ms * 1e-3) / 1e12 if match_ms else 0.0

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
        "data": ("STUB (CPU launcher test, no extraction)" if args.stub else
                 "synthetic (pan sequence of §8d G frames, shifted (+3,+2) px per frame)"),
        "config": {"workload": f"C2: {W}x{H} mono, 8 levels, {args.nfeatures} features, extract + brute-force "
                               f"Hamming top-2/ratio match of every frame vs its predecessor",
                   "frames_per_step": total, "frames_per_step_per_gpu": B, "width": W, "height": H, "nlevels": 8,
                   "nfeatures": args.nfeatures, "parallelism": f"{total}-frame job sharded over {world} GPU(s), "
                   f"{B} frames per GPU" + (", RCCL all-gather of the descriptor blocks, cross-shard predecessor match"
                                          if world > 1 else "")},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "algorithmic_bytes_per_launch": dom_bytes, "avg_launch_ms": per_launch_ms,
                     "launches_per_step": launches_per_step,
                     "timed_from": "timed region" if dom == "fast_cells" else "breakdown pass",
                     "stage_ms_per_step": {k: v[0] / brk_steps for k, v in breakdown.items()},
                     "stage_ms_source": "separate 3-step pass with launch events on every kernel",
                     "pipeline_algorithmic_GBs": bytes_frame * B / (extract_ms * 1e-3) / 1e9 if extract_ms else 0.0,
                     "pipeline_bytes_per_frame": bytes_frame,
                     # the whole step (extract + match + host plumbing) against the extractor's algorithmic bytes
                     "pipeline_GBs_from_ms_per_step": bytes_frame * B / (ms_per_step * 1e-3) / 1e9,
                     "pipeline_frac": bytes_frame * B / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "pipeline_traffic_per_step": pipe_traffic,
                     "pipeline_traffic_over_algorithmic": pipe_traffic / (bytes_frame * B) if pipe_traffic else None,
                     # what actually binds the extractor kernels: instruction issue (ISSUE_MODEL); the
                     # dominant kernel's fractions use its live timed-region launch time
                     "issue": issue_roofline("pan", dict({k: v[0] / brk_steps for k, v in breakdown.items()},
                                                         **({"fast_cells": per_launch_ms * launches_per_step}
                                                            if dom == "fast_cells" else {})), B)},
        # the brute-force matcher's FP4 MFMA path: every query x candidate pair is a 256-bit dot product
        "match_roofline": {"bound": "mfma", "kernel": "match (FP4 tiles)", "achieved": match_tflops,
                           "peak": FP4_PEAK_TFLOPS, "unit": "TFLOP/s (FP4)", "frac": match_tflops / FP4_PEAK_TFLOPS,
                           "ops": "512 FP4 flops per query x candidate pair, n_kp^2 pairs per matched frame (B - 1 per step)",
                           "match_ms_per_step": match_ms},
        "keypoints_per_frame": n_kp,
        "keypoint_quota": args.nfeatures,
        "keypoints_over_quota": n_kp / args.nfeatures if args.nfeatures else None,
        "matches_last_step": matches,
        "device_fault_mask": run.fault,
        "timed_region_s": elapsed,
    }
    if args.stub:
        result["stub"] = True
    if run.xchg is not None:
        result["exchange"] = dict(run.exchange_block(args.steps),
                                  workload="the headline's exchange (weak scaling, frames_per_step_per_gpu per rank)")
    # C5 (configs[4]) on every rank: it has collectives, so it runs before the rank-0-only legs
    if not args.no_c5:
        result["c5"] = c5_leg(ranks, ex, m, base, total=args.c5_frames, steps=args.steps, warmup=args.warmup,
                              nfeat=args.nfeatures)

    if world == 1 and not args.stub and not args.no_c5n8 and not args.no_legs:
        result["c5_n8_per_rank"] = c5_per_rank_leg(ranks, ex, m, base, per_rank=max(1, args.c5_frames // 8),
                                                   steps=args.steps, warmup=args.warmup)
    legs = rank == 0 and not args.no_legs and not args.stub
    cpu = world == 1 and not args.no_cpu_baseline and rank == 0 and not args.stub
    info = cpu_info()
    local = ranks.local
    dev = ranks.dev
    # LocalBA first: its host loop polls the device, so it is timed before any leg's CPU-baseline
    # thread pool has run in this process
    if legs and not args.no_ba:
        result["localba"] = localba_leg(local, cpu=cpu, info=info)
    if legs and not args.no_c1:
        result["c1"] = c1_leg(dev, local, cpu=cpu, info=info)
    if legs and not args.no_textured:
        result["c2_textured"] = c2_textured_leg(dev, local, cpu=cpu, info=info)
    if legs and not args.no_c1:
        result["c2_1000"] = c2_1000_leg(dev, local, cpu=cpu, info=info)
    if legs and not args.no_c3:
        result["c3"] = c3_leg(dev, local, cpu=cpu, info=info)
    if legs and not args.no_stereo:
        result["stereo"] = stereo_leg(dev, local)
    if legs and not args.no_latency:
        result["latency"] = latency_leg(dev, local, cpu=cpu)
    if legs and not args.no_projection:
        result["search_by_projection"] = projection_leg(dev, cpu=cpu)
        result["search_by_projection"]["relocalisation"] = reloc_leg(dev, cpu=cpu)
        result["search_for_initialization"] = init_leg(dev, cpu=cpu)
    if legs and not args.no_bow:
        result["bow"] = bow_leg(dev, local, cpu=cpu)
    if legs and not args.no_pose:
        result["pose_opt"] = pose_leg(dev, cpu=cpu)
    if cpu:
        result["cpu_baseline"] = cpu_baseline_block(
            "frames/s", f"{W}x{H} pan-sequence frames, extract + brute-force match vs previous",
            cpu_extract_match(base[:4], args.nfeatures, 1, 8.0),
            cpu_extract_match(base[:8], args.nfeatures, info["threads_all"], 8.0), info)
    # the headline's actual load next to it (inside config, which the driver's record keeps whole): the pan
    # frames fill ~70 % of the quota; the full-quota textured frames run at about half the rate
    result["config"]["load"] = {
        "keypoints_per_frame": n_kp, "keypoint_quota": args.nfeatures,
        "keypoints_over_quota": n_kp / args.nfeatures if args.nfeatures else None,
        "c2_textured_frames_per_s": (result.get("c2_textured") or {}).get("frames_per_s"),
        "c2_textured_keypoints_per_frame": (result.get("c2_textured") or {}).get("keypoints_per_frame"),
        "c2_1000_frames_per_s": (result.get("c2_1000") or {}).get("frames_per_s")}
    # the metric's other halves, flat and last on the line (a record that keeps only the tail of stdout
    # still holds them)
    result["summary"] = summary(result)
    if rank == 0:
        print(json.dumps(result), flush=True)
    ranks.close()


def summary(r):
    def g(*path):
        v = r
        for p in path:
            if not isinstance(v, dict) or p not in v:
                return None
            v = v[p]
        return round(v, 4) if isinstance(v, float) else v
    return {"c2_frames_per_s": g("value"), "c2_ms_per_step": g("ms_per_step"), "n_gpus": g("n_gpus"),
            "c2_keypoints_per_frame": g("keypoints_per_frame"), "c2_keypoint_quota": g("keypoint_quota"),
            "c2_textured_keypoints_per_frame": g("c2_textured", "keypoints_per_frame"),
            "fast_cells_frac": g("roofline", "frac"), "fast_cells_ms": g("roofline", "avg_launch_ms"),
            "pipeline_traffic_over_algorithmic": g("roofline", "pipeline_traffic_over_algorithmic"),
            "localba_iters_per_s": g("localba", "iters_per_s"), "localba_ms_per_call": g("localba", "ms_per_call"),
            "localba_cpu_iters_per_s": g("localba", "cpu_baseline", "value"),
            "c1_frames_per_s": g("c1", "frames_per_s"), "c1_cpu_median_ms": g("c1", "cpu_baseline", "median_ms"),
            "c2_1000_frames_per_s": g("c2_1000", "frames_per_s"),
            "c2_1000_cpu_frames_per_s": g("c2_1000", "cpu_baseline", "value"),
            "c2_textured_frames_per_s": g("c2_textured", "frames_per_s"),
            "c3_pairs_per_s": g("c3", "pairs_per_s"),
            "c5_frames_per_s": g("c5", "frames_per_s"), "c5_n_ranks": g("c5", "n_ranks"),
            "c5_gather_ms": g("c5", "gather_ms_max_over_ranks"), "c5_hbm_frac": g("c5", "hbm_frac"),
            "cpu_frames_per_s": g("cpu_baseline", "value")}


if __name__ == "__main__":
    main()
