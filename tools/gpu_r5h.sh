#!/bin/bash
# Round-5 session H: bisect the DESC_ANGLE_MFMA=0 (angold) descriptor nondeterminism -- the same build with
# MFMA results in AGPRs, and with a drain (waitcnt + nops) before / after the blur products.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp DET_FRAMES=64 DET_W=640 DET_H=480
mkdir -p gpurun_out
for v in angold angold_agpr angold_nop1 angold_nop2 head; do
  if [ $v = head ]; then unset ORBSLAM2_AMD_LIB; else export ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_$v.so; fi
  timeout -k 10 180 python tools/diag/desc_determinism.py > gpurun_out/det_$v.log 2>&1; rc=$?
  [ $rc -gt 1 ] && { tail -5 gpurun_out/det_$v.log; exit 4; }
  echo "$v: $(grep -c 'descriptor rows differ' gpurun_out/det_$v.log) pairs, $(tail -1 gpurun_out/det_$v.log)"
  grep "rows differ" gpurun_out/det_$v.log | head -3
done
unset ORBSLAM2_AMD_LIB
for i in 1 2; do
  timeout -k 10 120 python tools/kbench.py --frames 2048 --iters 5 --pan > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
  sed "s/^/head pan: /" gpurun_out/kb.log | tail -1
done
echo "session done"
