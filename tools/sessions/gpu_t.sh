#!/bin/bash
# Run a subset of GPU tests: TESTS="tests/a.py tests/b.py" bash tools/gpu_t.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${TLIM:-500} python -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -ra > gpurun_out/t.log 2>&1
rc=$?
tail -25 gpurun_out/t.log
exit $rc
