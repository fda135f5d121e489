cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py tests/test_cpp_dropin_gpu.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -x > gpurun_out/pytest_ba.log 2>&1 || { tail -30 gpurun_out/pytest_ba.log; exit 1; }
tail -2 gpurun_out/pytest_ba.log
bash tools/ba_tl.sh > gpurun_out/ba_tl_summary.txt || exit 2
tail -16 gpurun_out/ba_tl_summary.txt
timeout -k 10 120 python tools/diag/ba_stamps.py > gpurun_out/ba_stamps.log 2>&1 || { tail gpurun_out/ba_stamps.log; exit 3; }
grep -v amdgpu gpurun_out/ba_stamps.log
ORBBA_DEBUG_TIMING=1 timeout -k 10 60 python tools/babench.py 3 2>&1 | grep -v amdgpu | tail -24
timeout -k 10 60 python tools/babench.py 30 2>&1 | grep LocalBA
