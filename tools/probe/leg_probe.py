"""One bench.py leg alone (no CPU baseline): python tools/leg_probe.py projection|pose|bow|stereo."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import bench  # noqa: E402

name = sys.argv[1]
fn = {"projection": lambda: bench.projection_leg("cuda:0", cpu=False),
      "pose": lambda: bench.pose_leg("cuda:0", cpu=False),
      "bow": lambda: bench.bow_leg("cuda:0", 0, cpu=False),
      "stereo": lambda: bench.stereo_leg("cuda:0", 0)}[name]
r = fn()
print(json.dumps({k: v for k, v in r.items() if not isinstance(v, dict)}))
