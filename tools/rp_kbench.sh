cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp_kb -o run -- python3 tools/kbench.py --iters 20 --match > gpurun_out/rp_kb.log 2>&1 || exit 1
grep wall gpurun_out/rp_kb.log
python3 - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/rp_kb/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'].split('(')[0][:40]:40s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:10.1f} us")
PY
