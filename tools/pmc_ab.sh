#!/bin/bash
# PMC passes (tools/pmc_groups_fast.txt or PMC_GROUPS) for the in-tree library and tools/ab/lib_base.so
# on one kbench workload (ARGS); summaries under gpurun_out/pmc_{new,base}/summary.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ARGS=${ARGS:-"--pan --frames 1024"}
for v in new base; do
  if [ $v = base ]; then export ORBSLAM2_AMD_LIB=$PWD/tools/ab/lib_base.so; else unset ORBSLAM2_AMD_LIB; fi
  PMC_GROUPS=${PMC_GROUPS:-tools/pmc_groups_fast.txt} bash tools/gpu_pmc.sh pmc_$v $ARGS || exit 1
done
