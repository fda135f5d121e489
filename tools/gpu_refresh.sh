#!/bin/bash
# Round evidence in one GPU session: parity tests, smoke, PMC traffic passes, the bench line (reading
# the fresh traffic json) and the rocprofv3 kernel-trace stats of the C2 bench leg alone (its per-kernel
# averages must agree with the bench line's live HIP-event launch times), then of the secondary legs.
# Every GPU step has its own time limit; the chain stops at the first failure.  Outputs land in
# gpurun_out/profiles_<tag>/ and are copied into profiles/ on the CPU side after the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r02}
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -ra \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 2; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
fi
bash tools/gpu_traffic.sh $TAG || exit 4
mkdir -p gpurun_out/profiles_$TAG
cp gpurun_out/traffic_$TAG/${TAG}_traffic.json gpurun_out/profiles_$TAG/${TAG}_traffic.json
cp gpurun_out/traffic_$TAG/${TAG}_traffic.json profiles/${TAG}_traffic.json
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_$TAG.log 2>&1 || { tail -30 gpurun_out/bench_$TAG.log; exit 5; }
grep '^{' gpurun_out/bench_$TAG.log > gpurun_out/profiles_$TAG/${TAG}_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-legs --no-c5 \
    > gpurun_out/prof_${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_bench.log; exit 6; }
grep '^{' gpurun_out/prof_${TAG}_bench.log > gpurun_out/profiles_$TAG/${TAG}_bench_under_rocprof.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_legs -o run -- \
    python3 bench.py --steps 3 --warmup 1 --frames 1024 --no-cpu-baseline > gpurun_out/prof_${TAG}_legs.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_legs.log; exit 7; }
cp $(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1) gpurun_out/profiles_$TAG/${TAG}_kernel_stats.csv
cp $(find gpurun_out/prof_${TAG}_legs -name "*kernel_stats.csv" | head -1) gpurun_out/profiles_$TAG/${TAG}_kernel_stats_legs.csv
ls gpurun_out/profiles_$TAG
echo refresh done
