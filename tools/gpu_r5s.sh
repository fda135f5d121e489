#!/bin/bash
# Round-5 session S: the matrix-core pyramid's GPU tests; round 4's final library against this round's on
# one box (kbench, pan and textured); the round's PMC evidence (profiles/r05_pmc_*).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_pyramid_mfma_gpu.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_s.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_s.log; [ $rc -gt 1 ] && exit 2
for kind in pan textured; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for i in 1 2 3; do
    ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_r04.so timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
    sed "s/^/$kind r04: /" gpurun_out/kb.log | tail -1
    timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
    sed "s/^/$kind r05: /" gpurun_out/kb.log | tail -1
  done
done
bash tools/gpu_pmc_round.sh r05 > gpurun_out/pmc_round.log 2>&1 || { tail -20 gpurun_out/pmc_round.log; exit 5; }
tail -30 gpurun_out/pmc_round.log
echo "session done"
