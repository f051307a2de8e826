#!/bin/bash
# round 5 (k): final tree -- whole GPU suite, smoke, default bench line, rocprofv3 kernel stats + FETCH_SIZE
# (decode fp16 / fp8, and the long-context leg at kv 4086-4096)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r5k
mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $o/tests.log | head -20; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 500 python bench.py > $o/bench_default.json 2> $o/bench_default.err || { echo "bench failed"; tail -20 $o/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$o/bench_default.json')); print('fp16', d['value'], d['step_roofline']['frac'], 'fp8', d['fp8']['value'], 'long', d['long_context']['value'], 'prefill', d['prefill']['value'])"
timeout -k 10 600 bash tools/profile_round.sh fp16 fp8 || { echo "profile failed"; exit 1; }
YALM_EAGER=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $o/long_trace -o long -- \
  python3 bench.py --long-only --long-steps 32 --kernel-iters 16 > $o/long_trace.log 2>&1 || { echo "long trace failed"; tail -5 $o/long_trace.log; exit 1; }
YALM_EAGER=1 timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/long_pmc -o pmc -- \
  python3 bench.py --long-only --long-steps 8 --kernel-iters 4 > $o/long_pmc.log 2>&1 || { echo "long pmc failed"; tail -5 $o/long_pmc.log; exit 1; }
echo done
