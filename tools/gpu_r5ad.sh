#!/bin/bash
# Round-5 session AD: quadtree phase stamps of a small level (level 6, frame 0), pan and textured.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for kind in pan textured; do
  a=""; [ $kind = textured ] && a=textured
  QT_STAMPS_LIB=$PWD/tools/diag/liborbslam2_amd_stamps6.so timeout -k 10 180 python tools/diag/qt_stamps.py 1024 $a \
    > gpurun_out/qt6_$kind.log 2>&1 || { tail gpurun_out/qt6_$kind.log; exit 9; }
  echo "== $kind level 6"; cat gpurun_out/qt6_$kind.log | grep -v amdgpu.ids | head -30
done
bash tools/gpu_r5ae.sh
