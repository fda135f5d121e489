#!/bin/bash
# Round-5 session AI: the partitioned gather with cells as runs of 8 points (tools/ab/lib_vc.so)
# -- parity through that library, then the in-tree build against it on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_vc.so timeout -k 10 600 python -u -m pytest tests/test_extractor_gpu.py tests/test_cpp_dropin_gpu.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_ai.log 2>&1 || { tail -30 gpurun_out/pytest_ai.log; exit 2; }
tail -1 gpurun_out/pytest_ai.log
for kind in textured pan; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for i in 1 2 3; do
    for v in tree vc; do
      unset ORBSLAM2_AMD_LIB
      [ $v = vc ] && export ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_vc.so
      timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
      sed "s/^/$kind $v: /" gpurun_out/kb.log | tail -1
    done
  done
done
echo "session done"
