#!/bin/bash
# describe A/B: kbench timing (abn over tools/ab/lib_*.so + in-tree) and instruction / LDS PMC
# for each library on the pan workload; summaries under gpurun_out/pmcd_<lib>/summary.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
SETS="--pan --frames 1024;--textured --frames 1024" REPS=${REPS:-2} TESTS=none bash tools/abn.sh || exit 4
printf '%s\n' "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVES" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" > /tmp/pmcd_groups.txt
for lib in tools/ab/lib_*.so new; do
  if [ $lib = new ]; then unset ORBSLAM2_AMD_LIB; v=new; else export ORBSLAM2_AMD_LIB=$PWD/$lib; v=$(basename $lib .so); fi
  PMC_GROUPS=/tmp/pmcd_groups.txt bash tools/gpu_pmc.sh pmcd_$v --pan --frames 1024 || exit 5
  echo "== $v"; grep -A14 "^describe_kernel" gpurun_out/pmcd_$v/summary.txt
done
