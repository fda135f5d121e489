#!/bin/bash
# Round-5 session I: pyramid pair kernel with the horizontal pass on the matrix cores -- parity,
# determinism, A/B against the VALU pair kernel; the angold determinism dump (differing bits).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_extractor_gpu.py tests/test_compat_gpu.py tests/test_cpp_dropin_gpu.py \
  tests/test_stereo_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_i.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_i.log; [ $rc -gt 1 ] && exit 2
timeout -k 10 120 python tools/diag/desc_determinism.py > gpurun_out/det.log 2>&1; rc=$?
[ $rc -gt 1 ] && { tail -5 gpurun_out/det.log; exit 4; }
echo "determinism (head): $(tail -1 gpurun_out/det.log)"
for kind in pan textured; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for i in 1 2; do
    for v in 0 1; do
      ORBX_PYR_MFMA=$v timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
      sed "s/^/$kind pyr_mfma=$v: /" gpurun_out/kb.log | tail -1
    done
  done
done
DET_FRAMES=64 DET_W=640 DET_H=480 DET_DUMP=gpurun_out/det_angold_dump.json ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_angold.so \
  timeout -k 10 180 python tools/diag/desc_determinism.py > gpurun_out/det_angold_i.log 2>&1; rc=$?
[ $rc -gt 1 ] && { tail -5 gpurun_out/det_angold_i.log; exit 4; }
echo "angold: $(tail -1 gpurun_out/det_angold_i.log)"
echo "session done"
