#!/bin/bash
# Baseline session: the whole -m gpu suite, then kernel stage times on pan / textured / G frames.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/base_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/base_pytest.log
[ $rc -ne 0 ] && exit $rc
for m in --pan --textured ""; do
  timeout -k 10 120 python tools/kbench.py --frames 1024 --iters 10 --match $m > gpurun_out/base_kb.log 2>&1 || { tail -5 gpurun_out/base_kb.log; exit 4; }
  echo "kbench $m: $(grep wall gpurun_out/base_kb.log)"
done
