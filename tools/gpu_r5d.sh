#!/bin/bash
# round 5 (d): whole GPU suite after the TP rework, the driver's bench, TP1 through both
# transports (kernels per token, the folded exchange's cost on one GPU)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r5d
mkdir -p $o
timeout -k 10 1000 python -u -m pytest ${R5D_TESTS:-tests} -m gpu -x -v -s --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $o/tests.log | head -20; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $o/bench20.json 2> $o/bench20.err || { echo "bench failed"; tail -20 $o/bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('$o/bench20.json')); print('fp16', d['value'], d['step_roofline']['frac'], 'k/tok', d.get('kernels_per_token'), 'fp8', d['fp8']['value'], d['fp8']['step_roofline']['frac'], 'long', d['long_context']['value'], d['long_context']['step_roofline']['frac'], 'prefill', d['prefill']['value'])"
for tr in ipc rccl; do
  timeout -k 10 300 python bench.py --steps 64 --warmup 5 --tp --tp-transport $tr --no-cpu-baseline --no-prefill --no-fp8 --no-long > $o/bench_tp1_$tr.json 2> $o/bench_tp1_$tr.err || { echo "tp1 $tr failed"; tail -20 $o/bench_tp1_$tr.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/bench_tp1_$tr.json')); print('tp1 $tr', d['value'], 'k/tok', d.get('kernels_per_token'), d['config']['parallelism'])"
done
timeout -k 10 300 python bench.py --steps 64 --warmup 5 --no-cpu-baseline --no-prefill --no-fp8 --no-long > $o/bench_single64.json 2> $o/bench_single64.err && python3 -c "import json; d=json.load(open('$o/bench_single64.json')); print('single', d['value'], 'k/tok', d.get('kernels_per_token'))"
