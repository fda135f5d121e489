set -o pipefail
mkdir -p gpurun_out
timeout -k 10 100 ./tools/probe/issue_probe3 > gpurun_out/issue_probe3.txt 2>&1
