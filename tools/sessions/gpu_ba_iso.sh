#!/bin/bash
# which LocalBA build fails the oracle comparison (tools/ab/lib_*.so via ORBSLAM2_AMD_LIB, then in-tree)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PT="python -u -m pytest -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread"
for lib in tools/ab/lib_*.so; do
  ORBSLAM2_AMD_LIB=$PWD/$lib timeout -k 10 300 $PT tests/test_ba_gpu.py -k matches_oracle > gpurun_out/iso.log 2>&1; echo "$(basename $lib): rc $? $(tail -1 gpurun_out/iso.log)"
done
ORBBA_SNAP_SIDE=0 timeout -k 10 300 $PT tests/test_ba_gpu.py -k matches_oracle > gpurun_out/iso.log 2>&1; echo "new snap0: rc $? $(tail -1 gpurun_out/iso.log)"
timeout -k 10 300 $PT tests/test_ba_gpu.py -k matches_oracle > gpurun_out/iso.log 2>&1; echo "new: rc $? $(tail -1 gpurun_out/iso.log)"
