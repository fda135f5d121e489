#!/bin/bash
# LocalBA per-kernel floor: babench with the default kernel-argument placement and with
# HIP_FORCE_DEV_KERNARG=1, then a kernel trace of the latter (ba_timeline)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 120 python3 tools/babench.py 50 || exit 1
  HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 python3 tools/babench.py 50 || exit 2
  HIP_FORCE_DEV_KERNARG=0 timeout -k 10 120 python3 tools/babench.py 50 || exit 3
done
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ba_tl_dk -o run -- python3 tools/babench.py > gpurun_out/ba_tl_dk.log 2>&1 || { tail -5 gpurun_out/ba_tl_dk.log; exit 4; }
python3 tools/ba_timeline.py gpurun_out/ba_tl_dk v | tail -14
