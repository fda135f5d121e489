#!/bin/bash
# A/B on one GPU box: tools/ab/lib_base.so (a build of the base commit) against the in-tree library,
# alternating, after the GPU parity tests of the in-tree build.  KB_ARGS is passed to kbench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-"tests/test_extractor_gpu.py tests/test_matcher_gpu.py"}
timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1
rc=$?
tail -2 gpurun_out/ab_pytest.log
[ $rc -ne 0 ] && exit $rc
VARIANTS="base new"
[ -f tools/ab/lib_c.so ] && VARIANTS="base new c"
for i in 1 2 3; do
  for v in $VARIANTS; do
    case $v in
      base) export ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_base.so ;;
      c) export ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_c.so ;;
      *) unset ORBSLAM2_AMD_LIB ;;
    esac
    timeout -k 10 120 python tools/kbench.py --iters 20 --match $KB_ARGS > gpurun_out/ab_$v$i.log 2>&1 || { tail -5 gpurun_out/ab_$v$i.log; exit 5; }
    echo "$v: $(grep wall gpurun_out/ab_$v$i.log)"
  done
done
