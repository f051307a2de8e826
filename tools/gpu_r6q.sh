#!/bin/bash
# round 6 (q): A/B of delaying the Wo workgroups that share a CU with the head units (fp8, short
# contexts; YALM_AWO_HEAD_DELAY=workgroups:ticks, A/B build), interleaved bench rounds; the placement trace
o=gpurun_out/r6q; mkdir -p $o
export YALM_LIB=$PWD/yalm_amd/ab/libyalm_hip_wt_ab.so
timeout -k 10 120 python -u tools/attn_wo_trace.py --dtype fp8 --ctx 16 > $o/trace_fp8_16.txt 2>&1 || { echo "trace failed"; tail -20 $o/trace_fp8_16.txt; exit 1; }
grep -E "placement|head writer|Wo poll passed|Wo end" $o/trace_fp8_16.txt
for rep in 1 2 3; do
  for s in "none" "32:150" "32:220" "32:300"; do
    if [ "$s" = none ]; then unset YALM_AWO_HEAD_DELAY; else export YALM_AWO_HEAD_DELAY=$s; fi
    v=$(timeout -k 10 120 python bench.py --dtype fp8 --steps 20 --warmup 5 --no-cpu-baseline --no-envelope --no-prefill --no-fp8 --no-long 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'])") || { echo "bench failed"; exit 1; }
    echo "rep $rep fp8 head-delay $s: $v tok/s" | tee -a $o/ab.txt
  done
done
unset YALM_AWO_HEAD_DELAY
