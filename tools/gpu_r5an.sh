#!/bin/bash
# Round-5 session AN: the final library once more -- every GPU test, smoke, and a short bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_an.log 2>&1 || { tail -30 gpurun_out/pytest_an.log; exit 2; }
tail -1 gpurun_out/pytest_an.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_an.log 2>&1 || { tail -20 gpurun_out/smoke_an.log; exit 3; }
tail -1 gpurun_out/smoke_an.log
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-legs --no-c5 --no-cpu-baseline > gpurun_out/bench_an.log 2>&1 || { tail -20 gpurun_out/bench_an.log; exit 5; }
grep '^{' gpurun_out/bench_an.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['stage_ms_per_step'])"
echo "session done"
