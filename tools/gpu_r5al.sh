#!/bin/bash
# Round-5 session AL: level-0 quadtree stamps (current build, pass 1 sub-phases), then the gather with
# the cells' points past 8 loaded for all of a thread's cells together (tools/ab/lib_df.so): parity
# through it, then the in-tree build against it on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for kind in pan textured; do
  a=""; [ $kind = textured ] && a=textured
  QT_SUB_ITER=1 timeout -k 10 180 python tools/diag/qt_stamps.py 1024 $a > gpurun_out/qt0_$kind.log 2>&1 || { tail gpurun_out/qt0_$kind.log; exit 9; }
  echo "== $kind level 0"; grep -v amdgpu.ids gpurun_out/qt0_$kind.log
done
ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_df.so timeout -k 10 300 python -u -m pytest tests/test_extractor_gpu.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_al.log 2>&1 || { tail -30 gpurun_out/pytest_al.log; exit 2; }
tail -1 gpurun_out/pytest_al.log
for kind in textured pan; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for i in 1 2 3; do
    for v in tree df; do
      unset ORBSLAM2_AMD_LIB
      [ $v = df ] && export ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_df.so
      timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
      sed "s/^/$kind $v: /" gpurun_out/kb.log | tail -1
    done
  done
done
echo "session done"
