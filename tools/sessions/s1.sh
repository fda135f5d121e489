cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
bash tools/ba_tl.sh || exit 2
timeout -k 10 120 python tools/diag/fast_stamps.py 128 textured > gpurun_out/fs_tex.log 2>&1 || { tail gpurun_out/fs_tex.log; exit 3; }
timeout -k 10 120 python tools/diag/fast_stamps.py 128 > gpurun_out/fs_g.log 2>&1 || exit 3
grep -v amdgpu gpurun_out/fs_tex.log; grep -v amdgpu gpurun_out/fs_g.log
