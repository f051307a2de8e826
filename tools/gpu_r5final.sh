#!/bin/bash
# round 5 final: the committed tree's in-tree library -- whole GPU suite, smoke, the driver's command
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r5final
mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $o/tests.log | head -20; tail -30 $o/tests.log; exit 1; }
tail -n 1 $o/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $o/smoke.log; exit 1; }
tail -n 1 $o/smoke.log
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $o/bench_20.json 2> $o/bench_20.err || { echo "bench 20 failed"; tail -20 $o/bench_20.err; exit 1; }
python3 -c "import json; d=json.load(open('$o/bench_20.json')); print('driver cmd', 'fp16', d['value'], d['step_roofline']['frac'], 'fp8', d['fp8']['value'], d['fp8']['step_roofline']['frac'], 'long', d['long_context']['value'], 'prefill', d['prefill']['value'])"
echo done
