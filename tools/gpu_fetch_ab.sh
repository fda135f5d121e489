#!/bin/bash
# FETCH_SIZE of fast_cells for every tools/ab/lib_*.so, the in-tree library and ENVV variants (kbench pan, 1024 frames)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/fetch_ab
for lib in tools/ab/lib_*.so new $ENVV; do
  ev=""
  if [ "$lib" = new ]; then unset ORBSLAM2_AMD_LIB; v=new;
  elif [[ "$lib" == *=* ]]; then unset ORBSLAM2_AMD_LIB; v=env_${lib//=/_}; ev=$lib;
  else export ORBSLAM2_AMD_LIB=$PWD/$lib; v=$(basename $lib .so); fi
  env $ev timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d gpurun_out/fetch_ab/$v -o run -- \
      python3 tools/kbench.py --iters 2 --frames 1024 --pan > gpurun_out/fetch_ab/$v.log 2>&1 || { tail -5 gpurun_out/fetch_ab/$v.log; exit 1; }
  python3 - "$v" <<'PY'
import csv, sys, glob, collections
v = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/fetch_ab/{v}/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("orbamd::", "").replace("void ", "").split("<")[0]
        acc[n].append(float(r["Counter_Value"]))
print(v, {k: round(sum(x) / len(x) / 1e9, 3) for k, x in acc.items() if k in ("fast_cells_kernel", "describe_kernel")})
PY
done
