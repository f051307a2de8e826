#!/bin/bash
# round 6 (ae): RoPE (cos, sin) once per step in the step kernel instead of at the QKV GEMV's tail:
# decode parity suites, then QKV kernel time and the bench, HEAD library vs the working tree, alternating
o=gpurun_out/r6ae; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_ref_glue.py tests/test_gpu_ref_infer.py \
  tests/test_gpu_mistral.py tests/test_gpu_mistral_dims.py tests/test_gpu_tp.py tests/test_gpu_attn_wo.py -q -x --timeout 600 --timeout-method thread > $o/tests.txt 2>&1 || { echo "tests failed"; grep -E "^FAILED|Error" $o/tests.txt | head; tail -5 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for rep in 1 2 3; do
  for lib in HEAD wt; do
    if [ $lib = HEAD ]; then export YALM_LIB=$PWD/yalm_amd/ab/libyalm_hip_HEAD.so; else unset YALM_LIB; fi
    for dt in fp16 fp8; do
      k=$(timeout -k 10 120 python tools/kernel_times.py --dtype $dt --kernels 0 --iters 256 --ctx 30 | grep -E " 0 QKV" | awk '{print $3}')
      v=$(timeout -k 10 200 python bench.py --dtype $dt --steps 20 --warmup 5 --no-cpu-baseline --no-envelope --no-prefill --no-fp8 --no-long 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'])")
      echo "rep $rep $lib $dt: QKV $k us, bench(20) $v tok/s" | tee -a $o/ab.txt
    done
  done
done
