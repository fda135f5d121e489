#!/bin/bash
# Round-5 session G: hazard probe (queued-MFMA WAR), quadtree root-partitioned gather parity, quadtree A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 tools/probe/hazard_probe 200 > gpurun_out/hazard_probe.log 2>&1 || { tail gpurun_out/hazard_probe.log; exit 9; }
grep "T10\|T11\|T4" gpurun_out/hazard_probe.log
timeout -k 10 600 python -u -m pytest tests/test_extractor_gpu.py tests/test_compat_gpu.py tests/test_cpp_dropin_gpu.py tests/test_stereo_gpu.py \
  tests/test_triangulation_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_x.log 2>&1 \
  || { tail -40 gpurun_out/pytest_x.log; exit 2; }
tail -2 gpurun_out/pytest_x.log
timeout -k 10 120 python tools/diag/desc_determinism.py > gpurun_out/det.log 2>&1 || { tail -5 gpurun_out/det.log; exit 4; }
tail -1 gpurun_out/det.log
for kind in pan textured; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for i in 1 2; do
    for v in base new; do
      if [ $v = base ]; then export ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_base.so; else unset ORBSLAM2_AMD_LIB; fi
      timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
      sed "s/^/$kind $v: /" gpurun_out/kb.log | tail -1
    done
  done
done
for i in 1 2; do
  for v in new cheapsc; do
    if [ $v = cheapsc ]; then export ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_cheapsc.so; else unset ORBSLAM2_AMD_LIB; fi
    timeout -k 10 120 python tools/kbench.py --frames 2048 --iters 5 --pan > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
    sed "s/^/sincos-cost pan $v: /" gpurun_out/kb.log | tail -1
  done
done
unset ORBSLAM2_AMD_LIB
for kind in pan textured; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for i in 1 2; do
    for sp in 8 1 -1; do
      ORBX_FAST_SPEC=$sp timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
      sed "s/^/fast-spec $kind $sp: /" gpurun_out/kb.log | tail -1
    done
  done
done
echo "session done"
