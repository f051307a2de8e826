#!/bin/bash
# round 4: key splits of the fused attention + Wo launch (A/B YALM_AWO_SPLITS; default = what fits, 25)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4s2
mkdir -p $o
NEW=yalm_amd/ab/libyalm_hip_wt_ab.so
for dt in fp16 fp8; do
  for sp in 25 20 16 12 25 20 16 12; do
    YALM_LIB=$NEW YALM_AWO_SPLITS=$sp timeout -k 10 200 python tools/kernel_times.py --dtype $dt --iters 128 \
      --ctxs 300,500,1000,2000,4000 --kernels 8 > $o/kt_${dt}_$sp.txt 2>&1 || { echo "kt failed"; tail -5 $o/kt_${dt}_$sp.txt; exit 1; }
    echo "$dt S $sp: $(grep ' 8 attn' $o/kt_${dt}_$sp.txt | awk '{printf "%s ", $4}')"
  done
done
echo done
