#!/bin/bash
# round 6 (n): the prefill suites on the wave-per-row norm tree, then the bench (driver's 20 steps)
o=gpurun_out/r6n; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_prefill.py tests/test_gpu_prefill_llama.py tests/test_host.py > $o/tests.txt 2>&1 || { echo "tests failed"; tail -30 $o/tests.txt; exit 1; }
tail -2 $o/tests.txt
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > $o/bench_20.json.txt 2> $o/bench_20.err || { echo "bench failed"; tail -20 $o/bench_20.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$o/bench_20.json.txt').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['fp8']['value'], d['long_context']['value'], d['prefill']['value'], d['prefill'].get('split_form',{}).get('value'))"
