#!/bin/bash
# Round-5 session N: pyramid MFMA pair kernel v3 (vertical taps in source-row space through DPP, no LDS
# ring: 22.5 KiB, 7 workgroups per CU) -- parity, determinism, A/B, busy counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ORBX_PYR_MFMA=1 timeout -k 10 600 python -u -m pytest tests/test_extractor_gpu.py tests/test_compat_gpu.py tests/test_stereo_gpu.py \
  -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_n.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_n.log; [ $rc -gt 1 ] && exit 2
ORBX_PYR_MFMA=1 timeout -k 10 120 python tools/diag/desc_determinism.py > gpurun_out/det.log 2>&1; rc=$?
[ $rc -gt 1 ] && { tail -5 gpurun_out/det.log; exit 4; }
echo "determinism (mfma pyramid): $(tail -1 gpurun_out/det.log)"
for kind in pan textured; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for i in 1 2; do
    for v in 0 1; do
      ORBX_PYR_MFMA=$v timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
      sed "s/^/$kind pyr_mfma=$v: /" gpurun_out/kb.log | tail -1
    done
  done
done
PMC_GROUPS=tools/pmc_groups_busy.txt ORBX_PYR_MFMA=1 bash tools/gpu_pmc.sh pmcb_pyr1 --pan --frames 1024 || exit 6
grep -A3 "^pyramid_pair" gpurun_out/pmcb_pyr1/summary.txt
echo "session done"
