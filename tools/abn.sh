#!/bin/bash
# A/B/n on one GPU box: every tools/ab/lib_*.so (ORBSLAM2_AMD_LIB) and the in-tree library ("new"),
# and the in-tree library under each ENVV setting ("NAME=VALUE ..."), alternating, REPS rounds, over SETS (kbench argument sets separated by ';').  Optional parity tests
# of the in-tree build first (TESTS, "none" to skip).  Each GPU step is time-limited; stops on failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-none}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/abn_pytest.log 2>&1
  rc=$?
  tail -2 gpurun_out/abn_pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
SETS=${SETS:-"--pan --frames 1024;--textured --frames 1024"}
REPS=${REPS:-2}
IFS=';' read -ra SETA <<< "$SETS"
for set in "${SETA[@]}"; do
  echo "== $set"
  for i in $(seq 1 $REPS); do
    for lib in tools/ab/lib_*.so new $ENVV; do
      ev=""
      [[ "$lib" == *.so && ! -e "$lib" ]] && continue   # no tools/ab libraries: the glob stays literal
      if [ "$lib" = new ]; then unset ORBSLAM2_AMD_LIB; v=new;
      elif [[ "$lib" == *=* ]]; then unset ORBSLAM2_AMD_LIB; v=env_${lib//=/_}; ev=$lib;
      else export ORBSLAM2_AMD_LIB=$PWD/$lib; v=$(basename $lib .so); fi
      lg=gpurun_out/abn_${v}_$i.log
      env $ev timeout -k 10 120 python tools/kbench.py --iters 10 --match $set > $lg 2>&1 || { tail -5 $lg; exit 5; }
      echo "$v: $(grep wall $lg)"
    done
  done
done
