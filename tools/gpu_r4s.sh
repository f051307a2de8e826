#!/bin/bash
# round 4 (s): vendor GEMM ceiling on the prefill shapes (torch -> hipBLASLt), and the
# prefill's own per-kernel profile (one-launch QKV)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4s
mkdir -p $o
true

cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/pf -o pf -- python3 tools/bench_prefill.py --iters 3 --check 1 > $o/pf.log 2>&1 || { echo "pf prof failed"; tail -5 $o/pf.log; exit 1; }
python tools/prof_summary.py $o/pf/pf_kernel_stats.csv | head -16
echo done
