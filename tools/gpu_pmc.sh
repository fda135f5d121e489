#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, --kernel-trace only, no trace domains).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-pmc}
shift
ARGS="$@"
mkdir -p gpurun_out/$TAG
i=0
GROUPS_FILE=${PMC_GROUPS:-}
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc $group -d gpurun_out/$TAG/p$i -o run -- \
      python3 tools/kbench.py --iters 2 $ARGS > gpurun_out/$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/$TAG/p$i.log; exit 1; }
done < <(if [ -n "$GROUPS_FILE" ]; then cat "$GROUPS_FILE"; else cat << 'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM
SQ_WAIT_INST_LDS SQ_IFETCH SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE
FETCH_SIZE
WRITE_SIZE
GROUPS
fi)
python3 tools/pmc_summary.py gpurun_out/$TAG > gpurun_out/$TAG/summary.txt
echo done $i passes
