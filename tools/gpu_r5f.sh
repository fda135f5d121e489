#!/bin/bash
# Round-5 session F: the queued-MFMA WAR hypothesis (T10 / T11 of the hazard probe).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 tools/probe/hazard_probe 200 > gpurun_out/hazard_probe.log 2>&1 || { tail gpurun_out/hazard_probe.log; exit 9; }
cat gpurun_out/hazard_probe.log
echo "session done"
