#!/bin/bash
# LocalBA change: BA parity tests, then babench A/B over
# tools/ab/lib_*.so and the in-tree build (alternating)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PT="python -u -m pytest -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 600 $PT tests/test_ba_gpu.py tests/test_cpp_dropin_gpu.py > gpurun_out/ba3_pytest.log 2>&1 || { tail -30 gpurun_out/ba3_pytest.log; exit 3; }
tail -1 gpurun_out/ba3_pytest.log
for i in 1 2 3; do
  for lib in tools/ab/lib_*.so; do
    ORBSLAM2_AMD_LIB=$PWD/$lib timeout -k 10 120 python3 tools/babench.py 50 | sed "s#^#$(basename $lib .so): #" || exit 4
  done
  timeout -k 10 120 python3 tools/babench.py 50 | sed 's/^/new: /' || exit 5
done
