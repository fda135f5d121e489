#!/bin/bash
# r03 PMC evidence: instruction and busy counters per kernel (kbench, 1024 pan and 1024 textured C2
# frames), summaries + per-cell / per-wavefront counts under gpurun_out/profiles_pmc_r03/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/profiles_pmc_r03
mkdir -p $O
for w in pan textured; do
  PMC_GROUPS=tools/pmc_groups_inst.txt bash tools/gpu_pmc.sh pmci_$w --$w --frames 1024 || exit 1
  PMC_GROUPS=tools/pmc_groups_busy.txt bash tools/gpu_pmc.sh pmcb_$w --$w --frames 1024 || exit 2
  cp gpurun_out/pmci_$w/summary.txt $O/r03_pmc_inst_summary_$w.txt
  cp gpurun_out/pmcb_$w/summary.txt $O/r03_pmc_busy_summary_$w.txt
  python3 tools/pmc_percell.py gpurun_out/pmci_$w 1024 > $O/r03_pmc_percell_$w.txt || exit 3
  cat $O/r03_pmc_percell_$w.txt
done
