#!/bin/bash
# LocalBA A/B: BA parity tests of the in-tree build, then babench alternating base / new.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py tests/test_cpp_dropin_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/abba_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/abba_pytest.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_head.so timeout -k 10 60 python tools/babench.py 40 2>&1 | grep LocalBA | sed 's/^/base: /'
  timeout -k 10 60 python tools/babench.py 40 2>&1 | grep LocalBA | sed 's/^/new:  /'
  if [ -f tools/ab/lib_c.so ]; then
    ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_c.so timeout -k 10 60 python tools/babench.py 40 2>&1 | grep LocalBA | sed 's/^/c:    /'
  fi
done
ORBBA_DEBUG_TIMING=1 timeout -k 10 60 python tools/babench.py 2 2>&1 | grep orbba | tail -11
