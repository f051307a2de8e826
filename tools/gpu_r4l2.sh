#!/bin/bash
# round 4: rocprofv3 evidence for decode at kv 4086-4096 (bench.py --long-only, eager launches):
# kernel stats, then FETCH_SIZE in its own pass
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4l2
mkdir -p $o
YALM_EAGER=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o long -- \
  python3 bench.py --long-only --long-steps 32 --kernel-iters 16 > $o/trace.log 2>&1 || { echo "trace failed"; tail -5 $o/trace.log; exit 1; }
grep '"metric"' $o/trace.log | head -1 | cut -c1-400
YALM_EAGER=1 timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/pmc -o pmc -- \
  python3 bench.py --long-only --long-steps 8 --kernel-iters 4 > $o/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $o/pmc.log; exit 1; }
echo done
