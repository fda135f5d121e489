"""C3 leg alone (extract L+R + batched SearchForTriangulation): per-step and triangulation-only times."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import bench  # noqa: E402

r = bench.c3_leg("cuda:0", 0, cpu=False)
print(json.dumps({k: r[k] for k in ("pairs_per_s", "ms_per_step", "triangulation_ms_per_step", "matches_per_pair")}))
