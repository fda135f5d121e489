#!/bin/bash
# Round-5 session M: pyramid MFMA pair kernel v2 (fixed store column) parity + A/B + PMC; the i8 matcher
# (LDS-load-over-MFMA-source pattern in its listing) against the FP4 matcher.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ORBX_PYR_MFMA=1 timeout -k 10 600 python -u -m pytest tests/test_extractor_gpu.py tests/test_compat_gpu.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_m.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_m.log; [ $rc -gt 1 ] && exit 2
ORBX_PYR_MFMA=1 timeout -k 10 120 python tools/diag/desc_determinism.py > gpurun_out/det.log 2>&1; rc=$?
[ $rc -gt 1 ] && { tail -5 gpurun_out/det.log; exit 4; }
echo "determinism (head): $(tail -1 gpurun_out/det.log)"
for i in 1 2; do
  for v in 0 1; do
    ORBX_PYR_MFMA=$v timeout -k 10 120 python tools/kbench.py --frames 2048 --iters 5 --pan > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
    sed "s/^/pan pyr_mfma=$v: /" gpurun_out/kb.log | tail -1
  done
done
ORBX_PYR_MFMA=1 bash tools/gpu_pmc.sh pmc_pyr1b --pan --frames 1024 || exit 5
grep -A16 "^pyramid_pair" gpurun_out/pmc_pyr1b/summary.txt
PMC_GROUPS=tools/pmc_groups_busy.txt ORBX_PYR_MFMA=1 bash tools/gpu_pmc.sh pmcb_pyr1 --pan --frames 1024 || exit 6
PMC_GROUPS=tools/pmc_groups_busy.txt ORBX_PYR_MFMA=0 bash tools/gpu_pmc.sh pmcb_pyr0 --pan --frames 1024 || exit 6
grep -A3 "^pyramid_pair" gpurun_out/pmcb_pyr1/summary.txt gpurun_out/pmcb_pyr0/summary.txt
timeout -k 10 300 python tools/diag/matcher_i8_war.py > gpurun_out/mi8.log 2>&1; rc=$?
tail -14 gpurun_out/mi8.log; [ $rc -gt 1 ] && exit 7
echo "session done"
