#!/bin/bash
# round 5 (q): final-tree check after the TP fast-fail and bench gloo-timeout commits -- whole GPU suite,
# smoke, the default bench line and the driver's 20-step line
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r5q
mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $o/tests.log | head -20; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 500 python bench.py > $o/bench_default.json 2> $o/bench_default.err || { echo "bench failed"; tail -20 $o/bench_default.err; exit 1; }
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $o/bench_20.json 2> $o/bench_20.err || { echo "bench 20 failed"; tail -20 $o/bench_20.err; exit 1; }
for f in bench_default bench_20; do
python3 -c "import json; d=json.load(open('$o/$f.json')); print('$f', 'fp16', d['value'], d['step_roofline']['frac'], 'fp8', d['fp8']['value'], 'long', d['long_context']['value'], 'prefill', d['prefill']['value'])"
done
echo done
