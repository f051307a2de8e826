#!/bin/bash
# round 6 (ac): the suite's prefix up to the Mistral-dims file (the context of the one TP8 miss), 4 times
o=gpurun_out/r6ac; mkdir -p $o
for rep in 1 2 3 4; do
  timeout -k 10 600 python -u -m pytest tests/test_gpu_argmax.py tests/test_gpu_attn_wo.py tests/test_gpu_decode.py \
    tests/test_gpu_kernels.py tests/test_gpu_mistral.py tests/test_gpu_mistral_dims.py -q -s --timeout 500 --timeout-method thread > $o/prefix_$rep.log 2>&1
  echo "rep $rep rc=$?: $(tail -1 $o/prefix_$rep.log)"
  grep -E "^FAILED|AssertionError: \[" $o/prefix_$rep.log | head -4
done
