#!/bin/bash
# GPU tests (all) then the default bench line; each GPU step time-limited, chain stops on failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -ra > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 2; }
tail -2 gpurun_out/pytest_gpu.log
fi
timeout -k 10 600 python -u bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 4; }
grep '^{' gpurun_out/bench.log | python -c "
import json,sys
r=json.loads(sys.stdin.read())
def short(d, depth=0):
    out={}
    for k,v in d.items():
        if isinstance(v,dict) and depth<2: out[k]=short(v,depth+1)
        elif isinstance(v,float): out[k]=round(v,4)
        else: out[k]=v
    return out
print(json.dumps(short(r), indent=1))
"
