"""The bench's LocalBA leg alone (8 and 30 calls), without the CPU baseline."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import bench  # noqa: E402

print(json.dumps({k: v for k, v in bench.localba_leg(0, calls=8, cpu=False).items() if k != 'roofline'}))
print(json.dumps({k: v for k, v in bench.localba_leg(0, calls=30, cpu=False).items() if k != 'roofline'}))
