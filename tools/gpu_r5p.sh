#!/bin/bash
# Round-5 session P: A/B of the VALU pyramid's inline 24-bit multiply (lib_premulhi = commit d2d10ac) and of
# the FAST first-cell speculation on the same box; quadtree phase stamps (textured and pan, level 0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for kind in pan textured; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for i in 1 2 3; do
    ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_premulhi.so timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
    sed "s/^/$kind premulhi: /" gpurun_out/kb.log | tail -1
    ORBX_FAST_SPEC_FIRST=0 timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
    sed "s/^/$kind head first=0: /" gpurun_out/kb.log | tail -1
    timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
    sed "s/^/$kind head: /" gpurun_out/kb.log | tail -1
  done
done
timeout -k 10 180 python tools/diag/qt_stamps.py 1024 textured > gpurun_out/qt_tex.log 2>&1 || { tail gpurun_out/qt_tex.log; exit 9; }
cat gpurun_out/qt_tex.log | head -40
timeout -k 10 180 python tools/diag/qt_stamps.py 1024 > gpurun_out/qt_pan.log 2>&1 || { tail gpurun_out/qt_pan.log; exit 9; }
cat gpurun_out/qt_pan.log | head -40
echo "session done"
