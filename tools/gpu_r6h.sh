#!/bin/bash
o=gpurun_out/r6h; mkdir -p $o
T="python -u -m pytest -x -v --timeout 900 --timeout-method thread -s"
timeout -k 10 300 $T tests/test_host.py -k perplexity > $o/host.log 2>&1 || { echo "host failed"; tail -30 $o/host.log; exit 1; }
timeout -k 10 300 $T tests/test_gpu_mistral_dims.py -k "fp8-realistic" > $o/mdims.log 2>&1 || { echo "mdims failed"; tail -30 $o/mdims.log; exit 1; }
timeout -k 10 600 $T tests/test_gpu_prefill_llama.py -k full_depth > $o/pfl.log 2>&1 || { echo "pfl failed"; tail -30 $o/pfl.log; exit 1; }
grep -hoE "fp(16|8): \|d log ppl.*|worst max-rel.*|llama-3b dims, (14|28) layers.*" $o/*.log
grep -h "passed\|failed" $o/*.log
