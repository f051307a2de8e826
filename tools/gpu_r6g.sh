#!/bin/bash
# round 6: rocprofv3 kernel stats + FETCH_SIZE (fp16, fp8), the default bench line (256 steps) and the driver's 20
o=gpurun_out/r6g; mkdir -p $o
timeout -k 10 700 ./tools/profile_round.sh fp16 fp8 > $o/prof.log 2>&1 || { echo "profile failed"; tail -20 $o/prof.log; exit 1; }
cat $o/prof.log
timeout -k 10 400 python bench.py > $o/bench_default.json 2> $o/bench_default.err || { echo "bench default failed"; tail -20 $o/bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $o/bench_20.json 2> $o/bench_20.err || { echo "bench 20 failed"; tail -20 $o/bench_20.err; exit 1; }
cut -c1-600 $o/bench_default.json; cut -c1-300 $o/bench_20.json
