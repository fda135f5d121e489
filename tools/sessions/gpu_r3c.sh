#!/bin/bash
# extractor parity + determinism of the in-tree build, then describe A/B (kbench) over tools/ab/lib_*.so
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/diag/desc_determinism.py 2>&1 | tail -1 || exit 2
timeout -k 10 500 python -u -m pytest tests/test_extractor_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r3c_ext.log 2>&1 || { tail -20 gpurun_out/r3c_ext.log; exit 3; }
tail -1 gpurun_out/r3c_ext.log
SETS="--pan --frames 1024;--textured --frames 1024" REPS=${REPS:-2} TESTS=none bash tools/abn.sh || exit 4
