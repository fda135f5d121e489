#!/bin/bash
# Round-5 session K: T12 (the angold MFMA / LDS-load sequence) on the hardware; the determinism probe on
# builds of today's describe the LDS-WAR rule calls clean (keep-alive, fused sincos) or not (angle first,
# angold); PMC passes of the pyramid with and without the matrix-core pair kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 tools/probe/hazard_probe 200 > gpurun_out/hazard_probe.log 2>&1 || { tail gpurun_out/hazard_probe.log; exit 9; }
grep "T12\|T10\|T4" gpurun_out/hazard_probe.log
for v in angold keep fma af; do
  DET_FRAMES=64 DET_W=640 DET_H=480 ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_$v.so \
    timeout -k 10 180 python tools/diag/desc_determinism.py > gpurun_out/det_$v.log 2>&1; rc=$?
  [ $rc -gt 1 ] && { tail -5 gpurun_out/det_$v.log; exit 4; }
  echo "$v: $(tail -1 gpurun_out/det_$v.log)"
done
for v in 0 1; do
  ORBX_PYR_MFMA=$v bash tools/gpu_pmc.sh pmc_pyr$v --pan --frames 1024 || exit 5
  grep -i "pyramid" gpurun_out/pmc_pyr$v/summary.txt | head -20
done
echo "session done"
