cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
# one LocalBA call's GPU timeline: kernels + memory copies (no counters)
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/ba_tl -o run -- python3 tools/babench.py 5 > gpurun_out/ba_tl.log 2>&1 || { tail -5 gpurun_out/ba_tl.log; exit 1; }
tail -3 gpurun_out/ba_tl.log
python3 tools/ba_timeline.py gpurun_out/ba_tl v > gpurun_out/ba_tl.txt
tail -14 gpurun_out/ba_tl.txt
