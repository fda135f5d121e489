#!/bin/bash
# Round-3 check: extractor + BA parity of the in-tree build, then extractor A/B (abn) and LocalBA A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/diag/desc_determinism.py 2>&1 | tail -2 || exit 2
timeout -k 10 500 python -u -m pytest tests/test_extractor_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r3b_ext.log 2>&1 || { tail -20 gpurun_out/r3b_ext.log; exit 3; }
tail -1 gpurun_out/r3b_ext.log
TESTS=none REPS=2 bash tools/abn.sh || exit 4
bash tools/ab_ba.sh
