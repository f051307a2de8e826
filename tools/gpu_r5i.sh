#!/bin/bash
# round 5 (i): fused W2 + next-layer QKV launch: decode parity, then the bench
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r5i
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_mistral_dims.py tests/test_gpu_tp.py -x -v --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error|assert" $o/tests.log | head -30; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-prefill --no-long > $o/bench.json 2> $o/bench.err || { echo "bench failed"; tail -20 $o/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$o/bench.json')); print('fp16', d['value'], d['step_roofline']['frac'], 'k/tok', d.get('kernels_per_token'), 'fp8', d['fp8']['value'], d['fp8']['step_roofline']['frac'], d['fp8'].get('kernels_per_token'))"
for v in 0 1 0 1; do
  YALM_LIB=$PWD/yalm_amd/ab/libyalm_hip_wt_ab.so YALM_W2QKV=$v timeout -k 10 300 python bench.py --steps 64 --warmup 5 --no-cpu-baseline --no-prefill --no-long > $o/ab_$v.json 2> $o/ab_$v.err || { echo "ab $v failed"; tail -20 $o/ab_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/ab_$v.json')); print('W2QKV=$v fp16', d['value'], 'k/tok', d.get('kernels_per_token'), 'fp8', d['fp8']['value'])"
done
