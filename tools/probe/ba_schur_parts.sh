#!/bin/bash
# Schur-block kernel: average duration per real trial for the in-tree build and the diagnostic
# builds without the diagonal blocks' pose sums (noPA) / b_schur (noBS) (timing only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in new tools/probe/lib_ba_noPA.so tools/probe/lib_ba_noBS.so; do
  if [ $v = new ]; then unset ORBSLAM2_AMD_LIB; n=new; else export ORBSLAM2_AMD_LIB=$PWD/$v; n=$(basename $v .so); fi
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bsp_$n -o run -- python3 tools/babench.py 10 > gpurun_out/bsp_$n.log 2>&1 || { tail -5 gpurun_out/bsp_$n.log; exit 1; }
  python3 - gpurun_out/bsp_$n $n <<'PY'
import csv, sys, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("orbamd::", "")
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if d > 6.5: acc[n].append(d)
print(sys.argv[2], {k: (len(v), round(sum(v) / len(v), 2)) for k, v in acc.items() if k.startswith("ba_")})
PY
done
