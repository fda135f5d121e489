#!/bin/bash
# Round-5 session R: FAST speculation of every cell from its hint (ORBX_FAST_SPEC_FIRST=2) against the first-cell hint (1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ORBX_FAST_SPEC_FIRST=2 timeout -k 10 600 python -u -m pytest tests/test_extractor_gpu.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_q.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_q.log; [ $rc -gt 1 ] && exit 2
timeout -k 10 120 python tools/diag/desc_determinism.py > gpurun_out/det.log 2>&1; rc=$?
[ $rc -gt 1 ] && { tail -5 gpurun_out/det.log; exit 4; }
echo "determinism: $(tail -1 gpurun_out/det.log)"
for kind in pan textured; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for i in 1 2 3; do
    for v in 1 2; do
      ORBX_FAST_SPEC_FIRST=$v timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
      sed "s/^/$kind hint=$v: /" gpurun_out/kb.log | tail -1
    done
  done
done
echo "session done"
