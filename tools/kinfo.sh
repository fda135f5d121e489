#!/bin/bash
# Register / LDS metadata of the kernels of one source file (device asm, no GPU): tools/kinfo.sh orbx [pattern]
f=${1:-orbx}; pat=${2:-.}
cd "$(dirname "$0")/../orb_slam2_refactored_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../../include -I. -mllvm -amdgpu-mfma-vgpr-form \
  $EXTRA --cuda-device-only -S $f.hip -o /tmp/kinfo_$f.s 2>/dev/null
awk -v pat="$pat" '/\.name:/{n=$2} /\.sgpr_count:|\.vgpr_count:|spill_count:/{if (n ~ pat) printf "%s %s %s\n", n, $1, $2}' /tmp/kinfo_$f.s
