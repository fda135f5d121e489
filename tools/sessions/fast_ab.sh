#!/bin/bash
# Extractor tuning sweep: parity tests, then kbench over knobs (and the previous commit's library).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_extractor_gpu.py -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_ab.log 2>&1 || { tail -30 gpurun_out/pytest_ab.log; exit 1; }
tail -2 gpurun_out/pytest_ab.log
if [ -f tools/diag/liborbslam2_amd_prev.so ]; then
  echo "previous library"
  ORBSLAM2_AMD_LIB=tools/diag/liborbslam2_amd_prev.so timeout -k 10 120 python tools/kbench.py --iters 20 || exit 2
fi
for n in ${NSUBS:-1 2}; do
for c in ${CPWS:-1 2 4}; do
  echo "nsub $n cpw $c"
  ORBX_NSUB=$n ORBX_FAST_CPW=$c timeout -k 10 120 python tools/kbench.py --iters 20 || exit 2
done
done
