#!/bin/bash
# One GPU session: parity tests, smoke, short bench.  Every GPU step has its own time limit and
# the chain stops at the first failure (no retries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 -ra > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
if [ -f tools/diag/liborbslam2_amd_pjk1.so ]; then
  # SearchByProjection with K = 1 kept candidate: every claim conflict goes through the rescan path
  ORBSLAM2_AMD_LIB=$PWD/tools/diag/liborbslam2_amd_pjk1.so timeout -k 10 300 python -m pytest tests/test_projection_gpu.py -q \
    -p no:cacheprovider --timeout 200 > gpurun_out/pytest_pjk1.log 2>&1 || { echo "K=1 projection run failed"; tail -20 gpurun_out/pytest_pjk1.log; exit 5; }
  tail -1 gpurun_out/pytest_pjk1.log
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 3; }
tail -3 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 4; }
tail -3 gpurun_out/bench.log
exit $rc
