#!/bin/bash
# Build libyalm_hip.so from the sources of git revision $1 ("wt": the working tree) into yalm_amd/ab/libyalm_hip_$1.so
# (for A/B runs on one box: YALM_LIB=<that path> python tools/kernel_times.py ...).
# $2 = "ab": compile with -DYALM_AB (the tuning / tracing environment knobs, decoder.h ab_env)
# into yalm_amd/ab/libyalm_hip_$1_ab.so.
set -e
rev=$1
def=""; suf=""
if [ "$2" = "ab" ]; then def="-DYALM_AB"; suf="_ab"; fi
[ -n "${AB_SUFFIX:-}" ] && suf="${suf}_${AB_SUFFIX}"
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
if [ "$rev" = wt ]; then  # the working tree
  mkdir -p "$tmp/yalm_amd" && cp -r "$root/yalm_amd/csrc" "$tmp/yalm_amd/" && cp -r "$root/include" "$tmp/"
else
  git -C "$root" archive "$rev" yalm_amd/csrc include | tar -x -C "$tmp"
fi
mkdir -p "$root/yalm_amd/ab"
for f in yalm_hip prefill; do  # EXTRA_DEFS: more -D flags for the A/B build
  extra=""; [ $f = prefill ] && extra="-mllvm -amdgpu-mfma-vgpr-form"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $def ${EXTRA_DEFS:-} $extra -c -o "$tmp/$f.o" "$tmp/yalm_amd/csrc/$f.hip" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o "$root/yalm_amd/ab/libyalm_hip_$rev$suf.so" \
  "$tmp/yalm_hip.o" "$tmp/prefill.o" -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$tmp"
echo "$root/yalm_amd/ab/libyalm_hip_$rev$suf.so"
