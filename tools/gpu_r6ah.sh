#!/bin/bash
# round 6 (ah): final tree (after the RoPE table and the spread sink rotation) -- the GPU suite + smoke, rocprofv3 kernel stats + FETCH_SIZE (fp16, fp8),
# the default bench line (256 steps) and the driver's 20 steps
o=gpurun_out/r6ah; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 600 --timeout-method thread > $o/tests.log 2>&1
rc=$?
tail -3 $o/tests.log
[ $rc -eq 0 ] || { echo "suite failed rc=$rc"; grep -E "FAILED|Error" $o/tests.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 700 ./tools/profile_round.sh fp16 fp8 > $o/prof.log 2>&1 || { echo "profile failed"; tail -20 $o/prof.log; exit 1; }
tail -2 $o/prof.log
timeout -k 10 400 python bench.py > $o/bench_default.json 2> $o/bench_default.err || { echo "bench default failed"; tail -20 $o/bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $o/bench_20.json 2> $o/bench_20.err || { echo "bench 20 failed"; tail -20 $o/bench_20.err; exit 1; }
cut -c1-300 $o/bench_default.json; cut -c1-300 $o/bench_20.json
