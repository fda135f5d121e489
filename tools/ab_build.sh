#!/bin/bash
# Builds an A/B variant of the library: tools/ab/lib_<name>.so = the in-tree objects with <src>.hip
# recompiled under extra flags.  Usage: tools/ab_build.sh <name> <src (e.g. orbba)> <flags...>
# With REV=<git revision>, <src>.hip is taken from that revision instead of the working tree.
# (runs on the CPU side; the .so travels to the GPU box with the tree).
set -e
cd "$(dirname "$0")/../orb_slam2_refactored_amd/csrc"
name=$1; src=$2; shift 2
make -s
mkdir -p _build/ab ../../tools/ab
extra=""
case $src in orbx|orbm) extra="-mllvm -amdgpu-mfma-vgpr-form";; esac
[ -n "$NO_VGPR_FORM" ] && extra=""   # MFMA results in AGPRs (the compiler's default form)
file=$src.hip
if [ -n "$REV" ]; then file=_build/ab/${src}_$name.hip; git show "$REV:orb_slam2_refactored_amd/csrc/$src.hip" > $file; fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result \
    -I../../include -I. $extra "$@" -c $file -o _build/ab/${src}_$name.o
objs=""
for o in _build/*.o; do
  b=$(basename $o .o)
  if [ "$b" = "$src" ]; then objs="$objs _build/ab/${src}_$name.o"; else objs="$objs $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/ab/lib_$name.so $objs
echo "tools/ab/lib_$name.so"
