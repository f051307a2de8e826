#!/bin/bash
# round 4 (u): small-T prefill kernel profile (Mistral, T = 13)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4u
mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/sp -o sp -- python tools/bench_small_prefill.py --ts 13 --reps 3 > $o/sp.log 2>&1 || { echo "prof failed"; tail -5 $o/sp.log; exit 1; }
grep "T " $o/sp.log
echo done
