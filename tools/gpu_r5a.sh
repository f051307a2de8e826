#!/bin/bash
# round 5 (a): soffset probe, whole GPU suite (per-chunk K/V descriptors, explicit prefill
# forms), the driver's bench command, FETCH_SIZE of the fused launch at short and long context
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r5a
mkdir -p $o
timeout -k 10 60 tools/soffset_probe > $o/soffset_probe.txt 2>&1 || { echo "probe failed"; cat $o/soffset_probe.txt; exit 1; }
cat $o/soffset_probe.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $o/tests.log | head -20; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $o/bench20.json 2> $o/bench20.err || { echo "bench failed"; tail -20 $o/bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('$o/bench20.json')); print('fp16', d['value'], d['step_roofline']['frac'], 'fp8', d['fp8']['value'], d['fp8']['step_roofline']['frac'], 'long', d['long_context']['value'], d['long_context']['step_roofline']['frac'], 'prefill', d['prefill']['value'])"
YALM_EAGER=1 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/pmc -o pmc -- \
  python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-gpu-state --no-prefill --no-fp8 --no-long --no-envelope --kernel-iters 8 > $o/pmc_bench.log 2>&1 || { echo "pmc failed"; tail -5 $o/pmc_bench.log; exit 1; }
YALM_EAGER=1 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/pmc_long -o pmc -- \
  python3 bench.py --long-only --long-steps 8 --kernel-iters 4 > $o/pmc_long.log 2>&1 || { echo "pmc long failed"; tail -5 $o/pmc_long.log; exit 1; }
echo done
