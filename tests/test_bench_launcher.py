"""bench.py's multi-rank launcher and the traffic accounting, on CPU.

* `--gpus N` without a launcher starts N rank processes (VERDICT r03 "Next round" 1): driven here at N = 2
  with `--stub` (gloo, a deterministic stand-in for the extraction: the launcher, the rank bookkeeping,
  the C5 leg's exchange and cross-shard pairing are what is tested, not the kernels).
* `--gpus N` must fail loudly when N GPUs are not there or the launcher started a different world.
* `pipeline_traffic_over_algorithmic` recomputed from the committed round-3 profile (every pyramid kernel
  counted: 3 pyramid_pair_kernel launches + 1 pyramid_level_kernel per step)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                          "MASTER_PORT")}
    env.update(kw)
    return env


def _run(args, env, timeout=240):
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, cwd=ROOT, env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_launcher_starts_n_ranks_stub():
    p = _run(["--gpus", "2", "--stub", "--steps", "3", "--warmup", "1", "--frames", "8", "--c5-frames", "16"], _env())
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout        # one JSON line, from rank 0 only
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["stub"] is True
    assert r["config"]["frames_per_step"] == 16 and r["config"]["frames_per_step_per_gpu"] == 8
    # headline exchange: rank 1's first frame is matched against rank 0's last frame once per step
    x = r["exchange"]
    assert x["cross_shard_predecessor"] == -1            # rank 0 prints: global frame 0 has no predecessor
    assert x["gather_bytes_per_step"] > 0
    c5 = r["c5"]
    assert c5["n_ranks"] == 2 and c5["frames_per_rank"] == 8 and c5["frames_per_step"] == 16
    # each of warmup + steps (C5 takes --steps / --warmup) matched exactly once on rank 1 (no duplicate match
    # of the warm-up's last step)
    assert c5["cross_matches_run_all_ranks"] == 1 + 3
    assert c5["steps"] == 3 and c5["warmup"] == 1
    assert 0 < c5["hbm_frac"] < 1 and c5["keypoint_quota"] == 2000
    assert r["config"]["load"]["keypoint_quota"] == 2000
    assert r["summary"]["n_gpus"] == 2 and r["summary"]["c5_n_ranks"] == 2


def test_launcher_single_rank_stub_has_c5():
    p = _run(["--stub", "--steps", "2", "--warmup", "1", "--frames", "4", "--c5-frames", "8"], _env())
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert r["n_gpus"] == 1 and "exchange" not in r
    assert r["c5"]["n_ranks"] == 1 and r["c5"]["frames_per_rank"] == 8 and r["c5"]["cross_matches_run"] == 0


def test_count_gpus_kfd_without_hip(monkeypatch):
    """The launcher counts GPUs from sysfs, never through torch / HIP (a parent that initialised HIP and then
    started the ranks is what this pool forbids); visibility variables cap the count."""
    n = bench.count_gpus_kfd()
    assert n >= 0
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert bench.count_gpus_kfd() == 0
    src = (ROOT / "bench.py").read_text()
    body = src[src.index("def launch_ranks"):src.index("# ----", src.index("def launch_ranks"))]
    assert "import torch" not in body and "device_count(" not in body and "hipGetDeviceCount" not in body


def test_gpus_without_devices_fails_loudly():
    if bench.count_gpus_kfd() >= 2:
        pytest.skip("GPUs present")
    p = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"], _env(), timeout=120)
    assert p.returncode == 2
    assert "GPU(s) visible" in p.stderr


def test_gpus_world_mismatch_fails_loudly():
    p = _run(["--gpus", "2", "--stub"], _env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), timeout=120)
    assert p.returncode == 2
    assert "started 1 rank" in p.stderr


def test_pipeline_traffic_from_r03_profile():
    """VERDICT r03 What's weak 3: the r03 profile gives 82.2 GB per 8192-frame step = 2.06x the 39.9 GB
    algorithmic, not 58.1 GB = 1.46x."""
    t = json.loads((ROOT / "profiles" / "r03_traffic.json").read_text())
    tot = bench.measured_traffic_step(8192, 1280, 720, 2000, profile=t)
    assert tot == pytest.approx(82.2e9, rel=2e-3)
    alg = 4868261.0 * 8192          # r03 bench: pipeline_bytes_per_frame at 1994.2 keypoints
    assert tot / alg == pytest.approx(2.06, abs=0.005)
    # the pair kernel's average dispatch counts three times, the level kernel once
    assert [k for k, n in bench.stage_kernels(8)["pyramid"]] == ["pyramid_pair_kernel", "pyramid_level_kernel"]
    assert [n for k, n in bench.stage_kernels(8)["pyramid"]] == [3, 1]


def test_stage_kernels_by_level_count():
    # levels 1+2, 3+4, ... as pair launches, an odd last level as one level launch
    assert bench.stage_kernels(8)["pyramid"] == [("pyramid_pair_kernel", 3), ("pyramid_level_kernel", 1)]
    assert bench.stage_kernels(7)["pyramid"] == [("pyramid_pair_kernel", 3), ("pyramid_level_kernel", 0)]
    assert bench.stage_kernels(2)["pyramid"] == [("pyramid_pair_kernel", 0), ("pyramid_level_kernel", 1)]


def test_summary_is_flat_and_survives_missing_legs():
    r = {"value": 1.5, "ms_per_step": 2.0, "n_gpus": 1, "roofline": {"frac": 0.2, "avg_launch_ms": 3.0},
         "localba": {"iters_per_s": 9000.123456, "cpu_baseline": {"value": 500.0}}, "c5": {"frames_per_s": 7.0}}
    s = bench.summary(r)
    assert s["c2_frames_per_s"] == 1.5 and s["fast_cells_frac"] == 0.2 and s["localba_iters_per_s"] == 9000.1235
    assert s["localba_cpu_iters_per_s"] == 500.0 and s["c5_frames_per_s"] == 7.0
    assert s["c3_pairs_per_s"] is None and s["c1_frames_per_s"] is None
    assert all(not isinstance(v, dict) for v in s.values())
