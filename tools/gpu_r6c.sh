#!/bin/bash
# round 6: realistic model (residual-dominated), fp8 prefill KV check, range guard
o=gpurun_out/r6c; mkdir -p $o
T="python -u -m pytest -x -v --timeout 900 --timeout-method thread -s"
timeout -k 10 300 $T tests/test_gpu_prefill.py -k "fp8 or range_guard or split" > $o/prefill.log 2>&1 || { echo "prefill failed"; tail -30 $o/prefill.log; exit 1; }
timeout -k 10 300 $T tests/test_gpu_mistral_dims.py -k realistic > $o/mdims.log 2>&1 || { echo "mdims failed"; tail -30 $o/mdims.log; exit 1; }
timeout -k 10 600 $T tests/test_gpu_prefill_llama.py -k "realistic or peaked" > $o/pfl.log 2>&1 || { echo "pfl failed"; tail -30 $o/pfl.log; exit 1; }
timeout -k 10 900 $T tests/test_gpu_mistral.py -k realistic > $o/m2.log 2>&1 || { echo "m2 failed"; tail -30 $o/m2.log; exit 1; }
grep -hE "passed|failed|realistic|worst|per-layer|d log ppl|split .* fast" $o/*.log | tail -40
