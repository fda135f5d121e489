#!/bin/bash
# Round-5 session B: persistent describe.  Extractor parity (persistent default), determinism probe, then
# describe A/B: slot kernel (ORBX_DESC_PERSIST=0) vs persistent at KPI 4 / 8 / 16, pan and textured.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_extractor_gpu.py tests/test_compat_gpu.py tests/test_cpp_dropin_gpu.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_x.log 2>&1 || { tail -40 gpurun_out/pytest_x.log; exit 2; }
tail -2 gpurun_out/pytest_x.log
timeout -k 10 120 python tools/diag/desc_determinism.py > gpurun_out/det.log 2>&1 || { tail -20 gpurun_out/det.log; exit 3; }
tail -12 gpurun_out/det.log
for kind in pan textured; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for i in 1 2; do
    for cfg in "0 8" "1 4" "1 8" "1 16"; do
      set -- $cfg
      ORBX_DESC_PERSIST=$1 ORBX_DESC_KPI=$2 timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
      sed "s/^/$kind persist=$1 kpi=$2: /" gpurun_out/kb.log | tail -1
    done
  done
done
timeout -k 10 60 tools/probe/hazard_probe 200 > gpurun_out/hazard_probe.log 2>&1 || { tail gpurun_out/hazard_probe.log; exit 9; }
cat gpurun_out/hazard_probe.log
echo "session done"
