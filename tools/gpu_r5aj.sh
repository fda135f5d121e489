#!/bin/bash
# Round-5 session AJ: quadtree gather with ceil(cells / blockDim) cells per thread (lib_c3), and on top
# of it the whole-block split for phase-1 nodes above 512 / 256 points instead of 2048 (lib_b512,
# lib_b256) -- parity through each library, then the in-tree build against them on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in c3 b512 b256; do
  ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_extractor_gpu.py -m gpu -x -q \
    -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_aj_$v.log 2>&1 || { tail -30 gpurun_out/pytest_aj_$v.log; exit 2; }
  echo "$v: $(tail -1 gpurun_out/pytest_aj_$v.log)"
done
for kind in textured pan; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for i in 1 2 3; do
    for v in tree c3 b512 b256; do
      unset ORBSLAM2_AMD_LIB
      [ $v != tree ] && export ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_$v.so
      timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
      sed "s/^/$kind $v: /" gpurun_out/kb.log | tail -1
    done
  done
done
echo "session done"
