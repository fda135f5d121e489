set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_init_gpu.py tests/test_projection_reloc_gpu.py tests/test_projection_motion_gpu.py tests/test_projection_gpu.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/init.log 2>&1; rc=$?; tail -25 gpurun_out/init.log; exit $rc
