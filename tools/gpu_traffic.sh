#!/bin/bash
# HBM traffic evidence: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes (--kernel-trace only,
# no trace domains), for (1) the calibration program (known bytes per access width) and (2) the
# extractor at the bench workload.  tools/pmc_traffic.py turns them into profiles/<tag>_traffic.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r02}
FRAMES=${FRAMES:-8192}
OUT=gpurun_out/traffic_$TAG
mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc $c -d $OUT/calib_$c -o run -- \
      tools/calib/fetch_calib > $OUT/calib_$c.log 2>&1 || { echo "calib $c failed"; tail -5 $OUT/calib_$c.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc $c -d $OUT/kb_$c -o run -- \
      python3 tools/kbench.py --iters 2 --frames $FRAMES --pan > $OUT/kb_$c.log 2>&1 || { echo "kbench $c failed"; tail -5 $OUT/kb_$c.log; exit 1; }
done
python3 tools/pmc_traffic.py $OUT $OUT/${TAG}_traffic.json $FRAMES  # copy into profiles/ afterwards
