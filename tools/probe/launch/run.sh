#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 tools/probe/launch/launch_floor || exit 1
exit 0
cat gpurun_out/lf/run_kernel_stats.csv | cut -d, -f1-8
