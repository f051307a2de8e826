#!/bin/bash
# Build libyalm_hip.so from the sources of git revision $1 into yalm_amd/ab/libyalm_hip_$1.so
# (for A/B runs on one box: YALM_LIB=<that path> python tools/kernel_times.py ...).
set -e
rev=$1
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" yalm_amd/csrc include | tar -x -C "$tmp"
mkdir -p "$root/yalm_amd/ab"
for f in yalm_hip prefill; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -o "$tmp/$f.o" "$tmp/yalm_amd/csrc/$f.hip" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o "$root/yalm_amd/ab/libyalm_hip_$rev.so" \
  "$tmp/yalm_hip.o" "$tmp/prefill.o" -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$tmp"
echo "$root/yalm_amd/ab/libyalm_hip_$rev.so"
