#!/bin/bash
# Round-5 session AE: quadtree packed ne/dv scan without the separate total pass (one chunk) --
# parity, then the previous build (lib_head) against this build on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_extractor_gpu.py tests/test_cpp_dropin_gpu.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_ae.log 2>&1 || { tail -30 gpurun_out/pytest_ae.log; exit 2; }
tail -2 gpurun_out/pytest_ae.log
for kind in pan textured; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for i in 1 2 3; do
    for v in head pack new; do
      if [ $v = new ]; then unset ORBSLAM2_AMD_LIB; else export ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_$v.so; fi
      timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
      sed "s/^/$kind $v: /" gpurun_out/kb.log | tail -1
    done
  done
done
echo "session done"
