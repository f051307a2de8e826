#!/bin/bash
# round 5 (c): launch-lean tensor parallelism (IPC exchange folded into producers / consumers,
# fused attention + Wo on every rank): TP tests, then the TP8 Mistral-dims test and the rest
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r5c
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_tp.py -x -v --timeout 300 --timeout-method thread > $o/tp.log 2>&1 || { echo "tp tests failed"; grep -E "FAILED|Error|error|assert" $o/tp.log | head -30; tail -20 $o/tp.log; exit 1; }
tail -1 $o/tp.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_mistral_dims.py -x -v --timeout 400 --timeout-method thread -k "tensor_parallel" > $o/tp_mistral.log 2>&1 || { echo "tp mistral failed"; grep -E "FAILED|Error|error|assert" $o/tp_mistral.log | head -30; tail -20 $o/tp_mistral.log; exit 1; }
tail -1 $o/tp_mistral.log
