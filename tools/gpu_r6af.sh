#!/bin/bash
# round 6 (af): QKV GEMV device time outside vs inside the sink regime (kv_len 31 vs 4101):
# what the workgroup-0 sink-key rotation in PQKV::prologue costs per launch
o=gpurun_out/r6af; mkdir -p $o
timeout -k 10 200 python -u tools/kernel_times.py --ctxs 30,4100 --kernels 0,8 --iters 200 > $o/kt_fp16.log 2>&1 || { tail -20 $o/kt_fp16.log; exit 1; }
timeout -k 10 200 python -u tools/kernel_times.py --dtype fp8 --ctxs 30,4100 --kernels 0,8 --iters 200 > $o/kt_fp8.log 2>&1 || { tail -20 $o/kt_fp8.log; exit 1; }
cat $o/kt_fp16.log $o/kt_fp8.log
