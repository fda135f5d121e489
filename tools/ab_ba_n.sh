#!/bin/bash
# LocalBA A/B/n: BA parity tests and babench for every tools/ab/lib_*.so and the in-tree library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in tools/ab/lib_*.so new; do
  if [ $lib = new ]; then unset ORBSLAM2_AMD_LIB; v=new; else export ORBSLAM2_AMD_LIB=$PWD/$lib; v=$(basename $lib .so); fi
  timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/abban_$v.log 2>&1
  echo "$v tests: $(tail -1 gpurun_out/abban_$v.log)"
done
for i in 1 2; do
  for lib in tools/ab/lib_*.so new; do
    if [ $lib = new ]; then unset ORBSLAM2_AMD_LIB; v=new; else export ORBSLAM2_AMD_LIB=$PWD/$lib; v=$(basename $lib .so); fi
    echo "$v: $(timeout -k 10 60 python tools/babench.py 40 2>&1 | grep LocalBA)"
  done
done
