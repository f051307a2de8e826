#!/bin/bash
# round 5 (ac): fp8 attention + Wo at kv_len <= 64 in the eager greedy loop launched with S = 1
# (new default) vs the 25-split grid (A/B build, YALM_AWO_SHORT_S1=0), interleaved, at the driver's
# 20 steps and the default 256; then the whole GPU suite, smoke and the driver's command
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r5ac
mkdir -p $o
AB=$PWD/yalm_amd/ab/libyalm_hip_wt_ab.so
for r in 1 2 3; do
  for m in s1 s25; do
    for st in 20; do
      if [ $m = s25 ]; then export YALM_AWO_SHORT_S1=0; else unset YALM_AWO_SHORT_S1; fi
      YALM_LIB=$AB timeout -k 10 200 python bench.py --dtype fp8 --steps $st --warmup 5 --no-prefill --no-long --no-cpu-baseline --no-envelope --no-gpu-state > $o/$m.$st.$r.json 2> $o/$m.$st.$r.err || { echo "$m failed"; tail -5 $o/$m.$st.$r.err; exit 1; }
      python3 -c "import json; d=json.load(open('$o/$m.$st.$r.json')); print('round $r $m steps $st', 'fp8', d['value'])"
    done
  done
done
unset YALM_AWO_SHORT_S1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $o/tests.log | head -20; tail -30 $o/tests.log; exit 1; }
tail -n 1 $o/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $o/smoke.log; exit 1; }
tail -n 1 $o/smoke.log
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $o/bench_20.json 2> $o/bench_20.err || { echo "bench 20 failed"; tail -20 $o/bench_20.err; exit 1; }
python3 -c "import json; d=json.load(open('$o/bench_20.json')); print('driver cmd', 'fp16', d['value'], d['step_roofline']['frac'], 'fp8', d['fp8']['value'], d['fp8']['step_roofline']['frac'], 'long', d['long_context']['value'], 'prefill', d['prefill']['value'])"
echo done
