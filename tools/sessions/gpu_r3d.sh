#!/bin/bash
# describe parity + determinism, the new matcher legs and the headline fields on a short bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/diag/desc_determinism.py 2>&1 | tail -1 || exit 2
timeout -k 10 500 python -u -m pytest tests/test_extractor_gpu.py tests/test_init_gpu.py tests/test_projection_reloc_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r3d_t.log 2>&1 || { tail -20 gpurun_out/r3d_t.log; exit 3; }
tail -1 gpurun_out/r3d_t.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --frames 1024 --no-ba --no-c1 --no-textured --no-c3 --no-stereo --no-pose --no-bow > gpurun_out/r3d_bench.json 2> gpurun_out/r3d_bench.err || { tail -20 gpurun_out/r3d_bench.err; exit 4; }
python - <<'PY'
import json
r = json.loads(open("gpurun_out/r3d_bench.json").read().strip().splitlines()[-1])
print(r["value"], r["ms_per_step"])
print({k: r["roofline"][k] for k in ("pipeline_frac", "pipeline_GBs_from_ms_per_step", "pipeline_traffic_per_step", "pipeline_traffic_over_algorithmic")})
print(r["match_roofline"])
print(json.dumps(r["search_by_projection"]["relocalisation"]))
print(json.dumps(r["search_for_initialization"]))
PY
timeout -k 10 120 python tools/diag/ba_stamps.py 2>&1 | tail -14
bash tools/ba_tl.sh 2>&1 | tail -16
