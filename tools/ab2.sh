#!/bin/bash
# A/B on one GPU box over several frame sets: tools/ab/lib_base.so (a build of the base commit)
# against the in-tree library (and tools/ab/lib_c.so when present), alternating, after the GPU
# parity tests of the in-tree build.  SETS: kbench argument sets separated by ';'.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-"tests/test_extractor_gpu.py tests/test_matcher_gpu.py"}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1
  rc=$?
  tail -2 gpurun_out/ab_pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
VARIANTS="base new"
[ -f tools/ab/lib_c.so ] && VARIANTS="base new c"
# extra variants of the in-tree library under an environment setting: ENVV="NAME=VALUE ..."
for e in $ENVV; do VARIANTS="$VARIANTS env:$e"; done
SETS=${SETS:-"--pan --frames 1024;--textured --frames 1024"}
IFS=';' read -ra SETA <<< "$SETS"
for set in "${SETA[@]}"; do
  echo "== $set"
  for i in 1 2; do
    for v in $VARIANTS; do
      unset ORBSLAM2_AMD_LIB
      case $v in
        env:*) ;;
        base) export ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_base.so ;;
        c) export ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_c.so ;;
        *) unset ORBSLAM2_AMD_LIB ;;
      esac
      ev=""; [[ $v == env:* ]] && ev=${v#env:}
      lg=gpurun_out/ab_${v//[:=]/_}$i.log
      env $ev timeout -k 10 120 python tools/kbench.py --iters 10 --match $set > $lg 2>&1 || { tail -5 $lg; exit 5; }
      echo "$v: $(grep wall $lg)"
    done
  done
done
