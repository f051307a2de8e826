#!/bin/bash
# round 6 (s): head-mode threshold (YALM_ATTN_HEADMAX, A/B build) on the default 256-step bench (kv 22..277),
# fp16 and fp8, interleaved; plus the fused launch time per kv (kernel id 8) at each threshold
o=gpurun_out/r6s; mkdir -p $o
export YALM_LIB=$PWD/yalm_amd/ab/libyalm_hip_wt_ab.so
for hm in 2 4 6; do
  YALM_ATTN_HEADMAX=$hm timeout -k 10 240 python tools/kernel_times.py --kernels 8 --iters 128 --ctxs 60,120,180,230,250,270 > $o/kt_fp16_hm$hm.txt 2>&1 || { echo "kt failed"; tail $o/kt_fp16_hm$hm.txt; exit 1; }
  echo "== head_max $hm"; cat $o/kt_fp16_hm$hm.txt
done
for rep in 1 2; do
  for dt in fp16 fp8; do
    for hm in 2 3 4 6; do
      v=$(YALM_ATTN_HEADMAX=$hm timeout -k 10 200 python bench.py --dtype $dt --no-cpu-baseline --no-envelope --no-prefill --no-fp8 --no-long 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'])") || { echo "bench failed"; exit 1; }
      echo "rep $rep $dt head_max $hm: $v tok/s (256 steps)" | tee -a $o/ab.txt
    done
  done
done
