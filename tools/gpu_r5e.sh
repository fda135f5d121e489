#!/bin/bash
# Round-5 session E: is the DESC_ANGLE_MFMA=0 build's nondeterminism the MFMA whose D partially overlaps
# its SrcA?  Hazard probe T8 / T9 (partial D-over-source), then the determinism probe on the head and the
# angold builds.  (Exit codes other than 3: tools/gpurun_retry.sh reserves 3.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 90 tools/probe/hazard_probe 200 > gpurun_out/hazard_probe.log 2>&1 || { tail gpurun_out/hazard_probe.log; exit 9; }
grep "T8\|T9\|T3\|T4" gpurun_out/hazard_probe.log
for v in head angold; do
  if [ $v = head ]; then unset ORBSLAM2_AMD_LIB; else export ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_$v.so; fi
  DET_FRAMES=64 DET_W=640 DET_H=480 timeout -k 10 180 python tools/diag/desc_determinism.py > gpurun_out/det_$v.log 2>&1
  rc=$?
  [ $rc -gt 1 ] && { tail -20 gpurun_out/det_$v.log; exit 5; }
  echo "$v: $(tail -1 gpurun_out/det_$v.log)"
done
echo "session done"
