#!/bin/bash
# rocprofv3 evidence for the decode bench, in separate runs (counters never
# combined with trace domains): per dtype (fp16, fp8) (1) kernel trace + stats
# of the bench's kernels (--eager: the same kernels launched eagerly --
# rocprofv3's kernel trace of hipGraph replays crashes in the profiler), (2) the
# FETCH_SIZE counter. Output under gpurun_out/prof/; copy summaries to profiles/.
# usage: tools/profile_round.sh [fp16|fp8 ...]   (default: fp16 fp8)
set -e
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/prof
mkdir -p $out
dtypes="${@:-fp16 fp8}"
for dt in $dtypes; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_$dt -o bench -- \
    python3 bench.py --steps 64 --warmup 4 --no-cpu-baseline --no-gpu-state --no-prefill --no-fp8 --no-long --eager --dtype $dt > $out/trace_bench_$dt.log 2>&1
  echo "trace $dt ok"
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_$dt -o pmc -- \
    python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-gpu-state --no-prefill --no-fp8 --no-long --no-envelope --kernel-iters 8 --eager --dtype $dt \
    > $out/pmc_bench_$dt.log 2>&1
  echo "pmc $dt ok"
done
echo done
