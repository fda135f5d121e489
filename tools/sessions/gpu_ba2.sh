#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py tests/test_cpp_dropin_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ba2.log 2>&1 || { tail -20 gpurun_out/ba2.log; exit 3; }
tail -1 gpurun_out/ba2.log
for i in 1 2; do
  echo "head: $(ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_head.so timeout -k 10 60 python tools/babench.py 40 2>&1 | grep LocalBA)"
  echo "new:  $(timeout -k 10 60 python tools/babench.py 40 2>&1 | grep LocalBA)"
done
bash tools/ba_tl.sh 2>&1 | tail -12
