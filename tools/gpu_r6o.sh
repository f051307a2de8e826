#!/bin/bash
# round 6 (o): fused attention + Wo timelines at the driver's short contexts, fp8 and fp16
o=gpurun_out/r6o; mkdir -p $o
export YALM_LIB=$PWD/yalm_amd/ab/libyalm_hip_wt_ab.so
for dt in fp8 fp16; do
  for ctx in 16 63; do
    timeout -k 10 240 python -u tools/attn_wo_trace.py --dtype $dt --ctx $ctx --time 200 > $o/trace_${dt}_$ctx.txt 2>&1 || { echo "trace $dt $ctx failed"; tail -20 $o/trace_${dt}_$ctx.txt; exit 1; }
    cat $o/trace_${dt}_$ctx.txt
  done
done
