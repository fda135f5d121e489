#!/bin/bash
# Round-5 session AK: parity of the in-tree build (whole-block split from 512 points), then the
# sub-phase stamps of one phase-1 pass of a small level (level 6, pass 5) on pan and textured frames.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_extractor_gpu.py tests/test_cpp_dropin_gpu.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_ak.log 2>&1 || { tail -30 gpurun_out/pytest_ak.log; exit 2; }
tail -1 gpurun_out/pytest_ak.log
for kind in pan textured; do
  a=""; [ $kind = textured ] && a=textured
  QT_STAMPS_LIB=$PWD/tools/diag/liborbslam2_amd_stamps6s.so QT_SUB_ITER=5 timeout -k 10 180 python tools/diag/qt_stamps.py 1024 $a \
    > gpurun_out/qt6s_$kind.log 2>&1 || { tail gpurun_out/qt6s_$kind.log; exit 9; }
  echo "== $kind level 6"; grep -v amdgpu.ids gpurun_out/qt6s_$kind.log
done
echo "session done"
