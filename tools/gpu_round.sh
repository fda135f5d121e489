#!/bin/bash
# One GPU session of the round: the -m gpu suite, then optional A/B and bench steps named on the command
# line (tests | xtests | ba_ab | bench | kb_pan | kb_tex).  A/B steps compare tools/ab/lib_$BASE.so
# (default head) with the in-tree library.  Every GPU step has its own time limit; the chain stops at the
# first failure and nothing runs on the GPU after it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for step in "$@"; do
  case $step in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
      > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 2; }
    tail -2 gpurun_out/pytest_gpu.log ;;
  xtests)
    timeout -k 10 600 python -u -m pytest tests/test_extractor_gpu.py tests/test_cpp_dropin_gpu.py tests/test_matcher_gpu.py \
      -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_x.log 2>&1 \
      || { tail -30 gpurun_out/pytest_x.log; exit 2; }
    tail -2 gpurun_out/pytest_x.log ;;
  ba_ab)
    for i in 1 2 3; do
      ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_${BASE:-head}.so timeout -k 10 60 python tools/babench.py 40 > gpurun_out/babench.log 2>&1 || exit 5
      grep LocalBA gpurun_out/babench.log | sed "s/^/base: /"
      timeout -k 10 60 python tools/babench.py 40 > gpurun_out/babench.log 2>&1 || exit 6
      grep LocalBA gpurun_out/babench.log | sed "s/^/new:  /"
    done ;;
  bench)
    timeout -k 10 600 python -u bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 7; }
    grep '^{' gpurun_out/bench.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(json.dumps(r['summary'])); print(json.dumps(r.get('c5')))" ;;
  kb_pan|kb_tex)
    args="--frames 2048 --iters 5 --pan"; [ $step = kb_tex ] && args="--frames 1024 --iters 5 --textured"
    for i in 1 2; do
      ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_${BASE:-head}.so timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 8; }
      sed "s/^/$step base: /" gpurun_out/kb.log | tail -1
      timeout -k 10 120 python tools/kbench.py $args > gpurun_out/kb.log 2>&1 || { tail gpurun_out/kb.log; exit 9; }
      sed "s/^/$step new:  /" gpurun_out/kb.log | tail -1
    done ;;
  *) echo "unknown step $step"; exit 1 ;;
  esac
done
echo "session done"
