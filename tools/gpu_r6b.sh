#!/bin/bash
# round 6: CU-masked TP rehearsal, realistic model, fp8 prefill, range guard
o=gpurun_out/r6b; mkdir -p $o
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread -s"
timeout -k 10 300 $T tests/test_gpu_tp.py > $o/tp.log 2>&1 || { echo "tp failed"; tail -30 $o/tp.log; exit 1; }
timeout -k 10 300 $T tests/test_gpu_prefill.py -k "fp8 or range_guard or split" > $o/prefill.log 2>&1 || { echo "prefill failed"; tail -30 $o/prefill.log; exit 1; }
timeout -k 10 300 $T tests/test_gpu_attn_wo.py > $o/awo.log 2>&1 || { echo "awo failed"; tail -30 $o/awo.log; exit 1; }
timeout -k 10 600 $T tests/test_gpu_mistral_dims.py > $o/mdims.log 2>&1 || { echo "mdims failed"; tail -30 $o/mdims.log; exit 1; }
timeout -k 10 600 $T tests/test_gpu_prefill_llama.py -k realistic > $o/pfl.log 2>&1 || { echo "pfl failed"; tail -30 $o/pfl.log; exit 1; }
timeout -k 10 900 $T tests/test_gpu_mistral.py -k realistic > $o/m2.log 2>&1 || { echo "m2 failed"; tail -30 $o/m2.log; exit 1; }
grep -E "PASS|FAIL|realistic|worst|per-layer|d log ppl" $o/*.log | tail -60
