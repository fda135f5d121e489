#!/bin/bash
# Round-5 session C: persistent describe with dynamic group counters.  Parity + determinism, then describe
# A/B (slot kernel vs persistent 8-wave / 7-wave builds, KPI 4 / 8 / 16), pan and textured; hazard probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_extractor_gpu.py tests/test_compat_gpu.py tests/test_cpp_dropin_gpu.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_x.log 2>&1 || { tail -40 gpurun_out/pytest_x.log; exit 2; }
tail -2 gpurun_out/pytest_x.log
timeout -k 10 120 python tools/diag/desc_determinism.py > gpurun_out/det.log 2>&1 || { tail -20 gpurun_out/det.log; exit 3; }
tail -2 gpurun_out/det.log
for kind in pan textured; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for i in 1 2; do
    for cfg in "head 0 8" "head 1 4" "head 1 8" "head 1 16" "w7 1 8"; do
      set -- $cfg
      if [ $1 = w7 ]; then export ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_w7.so; else unset ORBSLAM2_AMD_LIB; fi
      ORBX_DESC_PERSIST=$2 ORBX_DESC_KPI=$3 timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
      sed "s/^/$kind lib=$1 persist=$2 kpi=$3: /" gpurun_out/kb.log | tail -1
    done
  done
done
timeout -k 10 90 tools/probe/hazard_probe 200 > gpurun_out/hazard_probe.log 2>&1 || { tail gpurun_out/hazard_probe.log; exit 9; }
cat gpurun_out/hazard_probe.log
echo "session done"
