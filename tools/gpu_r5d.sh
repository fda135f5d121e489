#!/bin/bash
# Round-5 session D: the round-4 nondeterministic describe builds rebuilt on the current code (LDS IC_Angle,
# empty-asm keep-alives, fused sincos) against the shipped build, each through the determinism probe
# (tools/diag/desc_determinism.py, 5 runs, larger frames), to reproduce the effect before naming a cause.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in head angold keep sfma; do
  if [ $v = head ]; then unset ORBSLAM2_AMD_LIB; else export ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_$v.so; fi
  for sz in "24 320 240" "64 640 480"; do
    set -- $sz
    DET_FRAMES=$1 DET_W=$2 DET_H=$3 timeout -k 10 180 python tools/diag/desc_determinism.py > gpurun_out/det_$v.log 2>&1 || { tail -20 gpurun_out/det_$v.log; exit 3; }
    echo "$v ${1}x${2}x${3}: $(grep -c 'rows differ' gpurun_out/det_$v.log) pairs, $(tail -1 gpurun_out/det_$v.log)"
    grep "rows differ" gpurun_out/det_$v.log | grep -v " 0 descriptor" | head -3
  done
done
echo "session done"
