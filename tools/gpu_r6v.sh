#!/bin/bash
# round 6 (v): how often does the TP8 rehearsal at Mistral dims miss the oracle? the TP8 case alone x10,
# then the whole Mistral-dims file x3 (the order the suite runs it in)
o=gpurun_out/r6v; mkdir -p $o
for rep in $(seq 1 10); do
  timeout -k 10 300 python -u -m pytest "tests/test_gpu_mistral_dims.py::test_tensor_parallel_ipc_mistral_dims_vs_oracle[8]" -q -s --timeout 200 --timeout-method thread > $o/tp8_$rep.log 2>&1
  echo "tp8 rep $rep rc=$?: $(tail -1 $o/tp8_$rep.log) $(grep -oE 'AssertionError: \([^)]*\)' $o/tp8_$rep.log | head -1)"
done
for rep in 1 2 3; do
  timeout -k 10 600 python -u -m pytest tests/test_gpu_mistral_dims.py -q -s --timeout 500 --timeout-method thread > $o/file_$rep.log 2>&1
  echo "file rep $rep rc=$?: $(tail -1 $o/file_$rep.log) $(grep -oE 'AssertionError: \([^)]*\)' $o/file_$rep.log | head -1)"
done
