#!/bin/bash
# round 4 (r): the config-2 workload (256 tokens, 32 layers) against the oracle; then one
# attempt at a rocprofv3 kernel trace of the GRAPH replays (round 1 saw the profiler crash)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4r
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread \
  tests/test_gpu_mistral.py > $o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $o/tests.log | head -20; tail -30 $o/tests.log; exit 1; }
grep -E "256 tokens|passed|failed" $o/tests.log
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/graph -o graph -- \
  python3 bench.py --steps 64 --warmup 4 --no-cpu-baseline --no-gpu-state --no-prefill --no-fp8 --no-long --no-envelope > $o/graph_bench.log 2>&1
echo "graph trace rc $?"
tail -3 $o/graph_bench.log
ls $o/graph 2>/dev/null | head
echo done
