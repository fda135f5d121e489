set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/g1_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/g1_pytest.log; [ $rc -ne 0 ] && exit $rc
for F in 128 512 1024 2048; do timeout -k 10 120 python tools/kbench.py --frames $F --iters 20 --match --no-profile 2>&1 | grep fps || exit 7; done
