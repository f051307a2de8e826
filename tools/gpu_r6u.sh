#!/bin/bash
# round 6 (u): the TP IPC rehearsal at Mistral dims (2 / 4 / 8 CU-masked ranks on one GPU), three times
o=gpurun_out/r6u; mkdir -p $o
for rep in 1 2 3; do
  timeout -k 10 600 python -u -m pytest tests/test_gpu_mistral_dims.py -k "tensor_parallel" -q -s --timeout 500 --timeout-method thread > $o/tp_$rep.log 2>&1
  echo "rep $rep rc=$?: $(tail -1 $o/tp_$rep.log)"
  grep -E "AssertionError: \(" $o/tp_$rep.log | head -3
done
