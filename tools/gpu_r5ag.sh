#!/bin/bash
# Round-5 session AG: the partitioned gather's boundary cells with batched loads (the in-tree build)
# -- parity, then the packed-scan build without it (tools/ab/lib_pack.so) against it on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_extractor_gpu.py tests/test_cpp_dropin_gpu.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_ag.log 2>&1 || { tail -30 gpurun_out/pytest_ag.log; exit 2; }
tail -1 gpurun_out/pytest_ag.log
for kind in textured pan; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for i in 1 2 3; do
    for v in pack tree; do
      unset ORBSLAM2_AMD_LIB
      [ $v = pack ] && export ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_pack.so
      timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
      sed "s/^/$kind $v: /" gpurun_out/kb.log | tail -1
    done
  done
done
QT_STAMPS_LIB=$PWD/tools/diag/liborbslam2_amd_stamps6g.so timeout -k 10 180 python tools/diag/qt_stamps.py 1024 textured \
  > gpurun_out/qt6g_textured.log 2>&1 || { tail gpurun_out/qt6g_textured.log; exit 9; }
grep -v amdgpu.ids gpurun_out/qt6g_textured.log | head -24
echo "session done"
