#!/bin/bash
# Round-5 session AF: quadtree small-level instance (quadtree_kernel<true>, 5 workgroups per CU) --
# parity, then head / packed scans / this build without and with the small instance on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_extractor_gpu.py tests/test_cpp_dropin_gpu.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_af.log 2>&1 || { tail -30 gpurun_out/pytest_af.log; exit 2; }
tail -2 gpurun_out/pytest_af.log
ORBX_QT_SMALL=0 timeout -k 10 300 python -u -m pytest tests/test_extractor_gpu.py -m gpu -x -q -p no:cacheprovider -k "quadtree or bit_exact or batch" \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_af0.log 2>&1 || { tail -30 gpurun_out/pytest_af0.log; exit 3; }
tail -1 gpurun_out/pytest_af0.log
for kind in pan textured; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for i in 1 2 3; do
    for v in head pack s0 s1; do
      unset ORBSLAM2_AMD_LIB ORBX_QT_SMALL
      case $v in head|pack) export ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_$v.so;; s0) export ORBX_QT_SMALL=0;; esac
      timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
      sed "s/^/$kind $v: /" gpurun_out/kb.log | tail -1
    done
  done
done
echo "session done"
