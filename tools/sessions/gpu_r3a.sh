#!/bin/bash
# Round-3 GPU check: new matcher rows' parity, then the exchange path at N = 1 and a short bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_init_gpu.py tests/test_projection_reloc_gpu.py tests/test_projection_motion_gpu.py tests/test_projection_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r3a_pytest.log 2>&1 || { tail -30 gpurun_out/r3a_pytest.log; exit 2; }
tail -2 gpurun_out/r3a_pytest.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --frames 1024 --no-legs --no-cpu-baseline --force-exchange > gpurun_out/r3a_bench_x.log 2>&1 || { tail -30 gpurun_out/r3a_bench_x.log; exit 3; }
grep '^{' gpurun_out/r3a_bench_x.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'], json.dumps(r.get('c5')))"
