#!/bin/bash
# round 4 (m): fused attention + Wo -- Wo slice delay sweep with timelines (do the head
# units' stores wait behind the co-resident Wo workgroup's slice loads?), then the prefill run (r4l)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4m
mkdir -p $o
NEW=yalm_amd/ab/libyalm_hip_wt_ab.so
for dt in fp8 fp16; do
  for dl in 0 50 150 250 350; do
    YALM_LIB=$NEW YALM_ATTN_WO_DELAY=$dl timeout -k 10 200 python tools/kernel_times.py --dtype $dt --iters 128 \
      --ctxs 16,100,250 --kernels 8 > $o/dl_${dt}_$dl.txt 2>&1 || { echo "dl failed"; tail -5 $o/dl_${dt}_$dl.txt; exit 1; }
    echo "$dt delay $dl: $(grep ' 8 attn' $o/dl_${dt}_$dl.txt | awk '{printf "%s ", $4}')"
  done
done
for dl in 50 250; do
  YALM_LIB=$NEW YALM_ATTN_WO_DELAY=$dl timeout -k 10 120 python tools/attn_wo_trace.py --dtype fp8 --ctx 16 > $o/trace_fp8_16_$dl.txt 2>&1 || { echo "trace failed"; tail -5 $o/trace_fp8_16_$dl.txt; exit 1; }
  echo "== trace fp8 ctx 16 delay $dl"; grep -E "span|loads landed|P.V in|P.V->|head signalled|Wo slice|Wo poll|Wo end" $o/trace_fp8_16_$dl.txt
done
bash tools/gpu_r4l.sh
