#!/bin/bash
# round 6 (y): the QKV epilogue's transposed 8-byte stores: prefill tests, then prefill time A/B
# (HEAD library vs the working tree), alternating processes
o=gpurun_out/r6y; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_prefill.py tests/test_gpu_prefill_llama.py tests/test_host.py > $o/tests.txt 2>&1 || { echo "tests failed"; tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for rep in 1 2 3 4; do
  for lib in HEAD wt; do
    if [ $lib = HEAD ]; then export YALM_LIB=$PWD/yalm_amd/ab/libyalm_hip_HEAD.so; else unset YALM_LIB; fi
    v=$(timeout -k 10 200 python3 tools/ab_prefill_forms.py --rounds 3 x= 2>/dev/null | tail -1)
    echo "rep $rep $lib $v" | tee -a $o/ab.txt
  done
done
