#!/bin/bash
# round 6 (p): where the fused launch's workgroups run (HW_ID / XCC_ID per workgroup) at kv 17, fp8 and fp16
o=gpurun_out/r6p; mkdir -p $o
export YALM_LIB=$PWD/yalm_amd/ab/libyalm_hip_wt_ab.so
for dt in fp8 fp16; do
  timeout -k 10 240 python -u tools/attn_wo_trace.py --dtype $dt --ctx 16 > $o/trace_${dt}_16.txt 2>&1 || { echo "trace $dt failed"; tail -20 $o/trace_${dt}_16.txt; exit 1; }
  cat $o/trace_${dt}_16.txt
done
