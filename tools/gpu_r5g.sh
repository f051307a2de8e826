#!/bin/bash
# round 5 (g): peaked-logit parity (config-2 256 tokens, 28-layer prefill), the -T 16384 window
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r5g
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_gpu_mistral_dims.py -x -v -s --timeout 400 --timeout-method thread -k "16k" > $o/dims.log 2>&1 || { echo "dims failed"; grep -E "FAILED|Error|error|assert" $o/dims.log | head -30; tail -20 $o/dims.log; exit 1; }
grep -E "16384|PASSED|SKIPPED" $o/dims.log | head; tail -1 $o/dims.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_prefill_llama.py -x -v -s --timeout 600 --timeout-method thread -k "peaked" > $o/prefill.log 2>&1 || { echo "prefill failed"; grep -E "FAILED|Error|error|assert|llama-3b" $o/prefill.log | head -30; tail -20 $o/prefill.log; exit 1; }
grep -E "llama-3b" $o/prefill.log; tail -1 $o/prefill.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_mistral.py -x -v -s --timeout 600 --timeout-method thread -k "config2" > $o/config2.log 2>&1 || { echo "config2 failed"; grep -E "FAILED|Error|error|assert|peak" $o/config2.log | head -30; tail -20 $o/config2.log; exit 1; }
grep -E "peak" $o/config2.log; tail -1 $o/config2.log
