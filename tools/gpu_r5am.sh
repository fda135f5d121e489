#!/bin/bash
# Round-5 session AM: the whole-block split counting 8 or 16 points per thread per round instead of 4 (bs8, bs16), and its scatter loading the next tile before the barrier (bspf)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in bs8 bs16 bspf; do
  ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_extractor_gpu.py -m gpu -x -q \
    -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_am_$v.log 2>&1 || { tail -30 gpurun_out/pytest_am_$v.log; exit 2; }
  echo "$v: $(tail -1 gpurun_out/pytest_am_$v.log)"
done
for kind in textured pan; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for i in 1 2 3; do
    for v in tree bs8 bs16 bspf; do
      unset ORBSLAM2_AMD_LIB
      [ $v != tree ] && export ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_$v.so
      timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
      sed "s/^/$kind $v: /" gpurun_out/kb.log | tail -1
    done
  done
done
echo "session done"
