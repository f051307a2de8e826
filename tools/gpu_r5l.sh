#!/bin/bash
# round 5 (l): split units' third chunk through LDS-DMA (attention.h): parity, then an interleaved A/B
# of HEAD vs the working tree (long-context leg and the default decode line)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r5l
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_gpu_mistral_dims.py tests/test_gpu_attn_wo.py tests/test_gpu_decode.py tests/test_gpu_kernels.py -x -q --timeout 400 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error|assert" $o/tests.log | head -30; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for lib in HEAD wt HEAD wt; do
  YALM_LIB=$PWD/yalm_amd/ab/libyalm_hip_$lib.so timeout -k 10 300 python bench.py --long-only --long-steps 64 --kernel-iters 32 > $o/long_$lib.json 2> $o/long_$lib.err || { echo "long $lib failed"; tail -20 $o/long_$lib.err; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('$o/long_$lib.json') if l.startswith('{')][-1]; lc=d.get('long_context', d); print('$lib long', lc.get('value'), lc.get('kernels_at_kv_max'))"
done
for lib in HEAD wt HEAD wt; do
  YALM_LIB=$PWD/yalm_amd/ab/libyalm_hip_$lib.so timeout -k 10 300 python bench.py --steps 64 --warmup 5 --no-cpu-baseline --no-prefill --no-long > $o/ab_$lib.json 2> $o/ab_$lib.err || { echo "ab $lib failed"; tail -20 $o/ab_$lib.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/ab_$lib.json')); print('$lib fp16', d['value'], 'fp8', d['fp8']['value'])"
done
