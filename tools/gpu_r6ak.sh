#!/bin/bash
# round 6 (ak): the QKV epilogue pair stores combined (one 4-byte K / V store, one
# 8-byte q store per row pair); decode parity suites, then QKV device time A/B (HEAD vs tree)
o=gpurun_out/r6ak; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_tp.py tests/test_gpu_ref_glue.py tests/test_gpu_mistral_dims.py tests/test_gpu_attn_wo.py -m gpu -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $o/tests.log | head -20; exit 1; }
for rep in 1 2; do
  for dt in fp16 fp8; do
    for lib in yalm_amd/ab/libyalm_hip_HEAD.so yalm_amd/libyalm_hip.so; do
      YALM_LIB=$lib timeout -k 5 200 python tools/kernel_times.py --ctxs 30,4100 --kernels 0 --iters 400 --dtype $dt > $o/kt.txt 2>&1 || { cat $o/kt.txt; exit 1; }
      echo "rep $rep $dt $(basename $lib): $(awk '$1=="0"{printf "%s ", $3}' $o/kt.txt) us (kv_len 31, 4101)"
    done
  done
done
