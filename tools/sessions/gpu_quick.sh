#!/bin/bash
# Quick GPU iteration: extractor/matcher parity tests + kernel stage timings (kbench).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-"tests/test_extractor_gpu.py tests/test_matcher_gpu.py"}
timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/quick_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/quick_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/kbench.py --iters 20 --match $KB_ARGS > gpurun_out/quick_kbench.log 2>&1 || { tail -20 gpurun_out/quick_kbench.log; exit 4; }
cat gpurun_out/quick_kbench.log | grep -v amdgpu.ids
