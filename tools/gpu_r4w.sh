#!/bin/bash
# round 4 (w): Wo workgroups on the head units' CUs issue the second slice half late
# (YALM_AWO_SPLIT_DELAY ticks) -- kernel times, traces, bench A/B; plus the fp16 Wo delay 20 vs 50
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4w
mkdir -p $o
NEW=yalm_amd/ab/libyalm_hip_wt_ab.so
for dt in fp8 fp16; do
  for sd in 0 100 200 0 100 200; do
    YALM_LIB=$NEW YALM_AWO_SPLIT_DELAY=$sd timeout -k 10 200 python tools/kernel_times.py --dtype $dt --iters 128 \
      --ctxs 16,100,250,1000 --kernels 8 > $o/kt_${dt}_$sd.txt 2>&1 || { echo "kt failed"; tail -5 $o/kt_${dt}_$sd.txt; exit 1; }
    echo "$dt split_delay $sd: $(grep ' 8 attn' $o/kt_${dt}_$sd.txt | awk '{printf "%s ", $4}')"
  done
done
for dl in 20 50 20 50; do
  YALM_LIB=$NEW YALM_ATTN_WO_DELAY=$dl timeout -k 10 200 python tools/kernel_times.py --dtype fp16 --iters 128 \
    --ctxs 16,100,250,1000 --kernels 8 > $o/dl_$dl.txt 2>&1 || { echo "kt failed"; tail -5 $o/dl_$dl.txt; exit 1; }
  echo "fp16 delay $dl: $(grep ' 8 attn' $o/dl_$dl.txt | awk '{printf "%s ", $4}')"
done
for sd in 100 200; do
  YALM_LIB=$NEW YALM_AWO_SPLIT_DELAY=$sd timeout -k 10 120 python tools/attn_wo_trace.py --dtype fp8 --ctx 16 > $o/trace_fp8_16_$sd.txt 2>&1 || { echo "trace failed"; exit 1; }
  echo "== trace fp8 ctx 16 split_delay $sd"; grep -E "span|P.V->|head signalled|Wo slice|Wo poll|Wo end" $o/trace_fp8_16_$sd.txt
done
for dt in fp8 fp16; do
  for sd in 0 150 0 150; do
    r=$(YALM_LIB=$NEW YALM_AWO_SPLIT_DELAY=$sd timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-envelope --no-prefill --no-fp8 --no-long --dtype $dt | \
        python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'])")
    echo "$dt split_delay $sd bench(20): $r tok/s"
  done
done
echo done
