#!/bin/bash
# round 5 (e): per-kernel cost of the folded IPC exchange at TP1 (rocprofv3, eager launches)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r5e
mkdir -p $o
for m in single ipc; do
  extra=""; [ $m = ipc ] && extra="--tp --tp-transport ipc"
  YALM_EAGER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace_$m -o k -- \
    python3 bench.py --steps 32 --warmup 4 --no-cpu-baseline --no-gpu-state --no-prefill --no-fp8 --no-long --no-envelope $extra > $o/bench_$m.log 2>&1 || { echo "trace $m failed"; tail -5 $o/bench_$m.log; exit 1; }
  f=$(ls $o/trace_$m/*kernel_stats.csv | head -1)
  python3 tools/prof_summary.py $f > $o/stats_$m.txt
  head -12 $o/stats_$m.txt
done
