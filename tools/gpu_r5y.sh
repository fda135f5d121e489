#!/bin/bash
# Round-5 session Y: the first-cell hint as an iniThFAST bit in cell_cnt -- round 4 against this build, with the FAST
# first-cell hint on / compiled out; parity of the extractor tests first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_extractor_gpu.py tests/test_compat_gpu.py tests/test_stereo_gpu.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_x.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_x.log; [ $rc -gt 1 ] && exit 2
for kind in pan textured; do
  args="--frames 2048 --iters 5 --pan"; [ $kind = textured ] && args="--frames 1024 --iters 5 --textured"
  for i in 1 2 3; do
    ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_r04.so timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
    sed "s/^/$kind r04: /" gpurun_out/kb.log | tail -1
    timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
    sed "s/^/$kind r05: /" gpurun_out/kb.log | tail -1
    ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_nohint.so timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
    sed "s/^/$kind r05 no hint code: /" gpurun_out/kb.log | tail -1
  done
done
echo "session done"
