#!/bin/bash
# Round-5 session AC: small pyramid levels' quadtrees in 64- / 128-thread workgroups (ORBX_QT_SMALL) --
# parity with it on, then A/B against the single 256-thread launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ORBX_QT_SMALL=64 timeout -k 10 600 python -u -m pytest tests/test_extractor_gpu.py tests/test_cpp_dropin_gpu.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_ac.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ac.log; [ $rc -gt 1 ] && exit 2
for kind in pan textured; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for i in 1 2; do
    for v in 0 64 128; do
      ORBX_QT_SMALL=$v timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
      sed "s/^/$kind qt_small=$v: /" gpurun_out/kb.log | tail -1
    done
  done
done
echo "session done"
