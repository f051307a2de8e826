#!/bin/bash
# round 4: head-mode threshold (A/B YALM_ATTN_HEADMAX chunks; default 4) on the final attention
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4hm
mkdir -p $o
NEW=yalm_amd/ab/libyalm_hip_wt_ab.so
for dt in fp16 fp8; do
  for hm in 2 4 6 8 2 4 6 8; do
    YALM_LIB=$NEW YALM_ATTN_HEADMAX=$hm timeout -k 10 200 python tools/kernel_times.py --dtype $dt --iters 128 \
      --ctxs 100,190,250,300,380,500 --kernels 8 > $o/kt_${dt}_$hm.txt 2>&1 || { echo "kt failed"; tail -5 $o/kt_${dt}_$hm.txt; exit 1; }
    echo "$dt headmax $hm: $(grep ' 8 attn' $o/kt_${dt}_$hm.txt | awk '{printf "%s ", $4}')"
  done
done
echo done
