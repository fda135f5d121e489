#!/bin/bash
# Round-5 session O: FAST speculation on a strip's first cell (ORBX_FAST_SPEC_FIRST) -- exactness and A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ORBX_FAST_SPEC_FIRST=1 timeout -k 10 600 python -u -m pytest tests/test_extractor_gpu.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_o.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_o.log; [ $rc -gt 1 ] && exit 2
for kind in pan textured; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for i in 1 2; do
    for v in 0 1; do
      ORBX_FAST_SPEC_FIRST=$v timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
      sed "s/^/$kind spec_first=$v: /" gpurun_out/kb.log | tail -1
    done
  done
done
for kind in pan textured; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for sp in 4 2; do
    ORBX_FAST_SPEC=$sp ORBX_FAST_SPEC_FIRST=1 timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
    sed "s/^/$kind spec=$sp first=1: /" gpurun_out/kb.log | tail -1
  done
done
echo "session done"
