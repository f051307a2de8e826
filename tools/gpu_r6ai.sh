#!/bin/bash
# round 6 (ai): rocprofv3 kernel stats + FETCH_SIZE of the long-context leg (kv 4086-4096, sink regime) on
# the final tree (eager launches: the profiler's kernel trace of graph replays is unreliable)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r6ai; mkdir -p $o
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $o/long_trace -o long -- \
  python3 bench.py --long-only --long-steps 32 --kernel-iters 16 --eager > $o/long_trace.log 2>&1 || { echo "long trace failed"; tail -5 $o/long_trace.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/long_pmc -o pmc -- \
  python3 bench.py --long-only --long-steps 8 --kernel-iters 4 --eager > $o/long_pmc.log 2>&1 || { echo "long pmc failed"; tail -5 $o/long_pmc.log; exit 1; }
timeout -k 10 300 python3 bench.py --long-only > $o/long_graph.json 2>$o/long_graph.err || { echo "long graph failed"; tail -5 $o/long_graph.err; exit 1; }
cut -c1-400 $o/long_graph.json
echo done
