#!/bin/bash
# Round-5 session W: fast_cells against round 4 with the resize tail off (ORBX_RESIZE_TAIL=0: round 4's pyramid output).
#
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_r04.so timeout -k 10 120 python tools/kbench.py --frames 2048 --iters 5 --pan > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
  sed "s/^/pan r04: /" gpurun_out/kb.log | tail -1
  timeout -k 10 120 python tools/kbench.py --frames 2048 --iters 5 --pan > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
  sed "s/^/pan r05: /" gpurun_out/kb.log | tail -1
  ORBX_RESIZE_TAIL=0 timeout -k 10 120 python tools/kbench.py --frames 2048 --iters 5 --pan > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
  sed "s/^/pan r05 tail off: /" gpurun_out/kb.log | tail -1
done
echo "session done"
