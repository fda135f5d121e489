#!/bin/bash
# A round's PMC evidence (TAG, e.g. r04): instruction and busy counters per kernel (kbench, 1024 pan and
# 1024 textured C2 frames), summaries + per-cell / per-wavefront counts under gpurun_out/profiles_pmc_TAG/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04}
O=gpurun_out/profiles_pmc_$TAG
mkdir -p $O
for w in pan textured; do
  PMC_GROUPS=tools/pmc_groups_inst.txt bash tools/gpu_pmc.sh pmci_$w --$w --frames 1024 || exit 1
  PMC_GROUPS=tools/pmc_groups_busy.txt bash tools/gpu_pmc.sh pmcb_$w --$w --frames 1024 || exit 2
  cp gpurun_out/pmci_$w/summary.txt $O/${TAG}_pmc_inst_summary_$w.txt
  cp gpurun_out/pmcb_$w/summary.txt $O/${TAG}_pmc_busy_summary_$w.txt
  python3 tools/pmc_percell.py gpurun_out/pmci_$w 1024 > $O/${TAG}_pmc_percell_$w.txt || exit 3
  cat $O/${TAG}_pmc_percell_$w.txt
done
