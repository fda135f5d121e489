#!/bin/bash
# Round-5 session AO: the scheduling knobs again on the final kernels -- sub-batches on side streams
# (ORBX_NSUB) and the level-0 side-stream overlap (ORBX_LEVEL_OVERLAP), pan and textured, one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for kind in pan textured; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for i in 1 2; do
    for v in "1 0" "2 0" "1 1" "2 1"; do
      set -- $v
      ORBX_NSUB=$1 ORBX_LEVEL_OVERLAP=$2 timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
      sed "s/^/$kind nsub $1 overlap $2: /" gpurun_out/kb.log | tail -1
    done
  done
done
echo "session done"
