#!/bin/bash
# Round-5 session AA: where the remaining pyramid difference against round 4 comes from -- builds without
# the resize tail's instantiation (diagnostic) and with the masked compiler multiply.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in r04 head notail mask; do
    if [ $v = head ]; then unset ORBSLAM2_AMD_LIB; else export ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_$v.so; fi
    timeout -k 10 120 python tools/kbench.py --frames 2048 --iters 5 --pan > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
    sed "s/^/pan $v: /" gpurun_out/kb.log | tail -1
  done
done
unset ORBSLAM2_AMD_LIB
echo "session done"
