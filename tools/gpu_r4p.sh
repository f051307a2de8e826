#!/bin/bash
# round 4 (p): the default bench line (fp16 + fp8 + prefill + long context + CPU baselines),
# the driver's 20-step line, rocprofv3 kernel stats + FETCH_SIZE per dtype
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4p
mkdir -p $o
timeout -k 10 500 python bench.py > $o/bench_default.json 2> $o/bench_default.err || { echo "bench failed"; tail -20 $o/bench_default.err; exit 1; }
cat $o/bench_default.json
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $o/bench_20.json 2> $o/bench_20.err || { echo "bench20 failed"; tail -20 $o/bench_20.err; exit 1; }
cat $o/bench_20.json
timeout -k 10 600 bash tools/profile_round.sh fp16 fp8 || { echo "profile failed"; exit 1; }
echo done
