#!/bin/bash
# Round-5 session A: GPU suite, then the resize-tail cost (ORBX_RESIZE_TAIL 0 vs 16) on the pan workload,
# then a short bench.  Each GPU step under its own limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 2; }
tail -2 gpurun_out/pytest_gpu.log
for i in 1 2; do
  for v in 0 16; do
    ORBX_RESIZE_TAIL=$v timeout -k 10 120 python tools/kbench.py --frames 2048 --iters 5 --pan > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
    sed "s/^/tail=$v: /" gpurun_out/kb.log | tail -1
  done
done
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 7; }
grep '^{' gpurun_out/bench.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step']); print(json.dumps(r['summary']))"
echo "session done"
