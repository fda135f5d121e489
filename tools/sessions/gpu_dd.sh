#!/bin/bash
# describe determinism (repeated identical extractions) of the in-tree build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 120 python tools/diag/desc_determinism.py 2>&1 | tail -3
