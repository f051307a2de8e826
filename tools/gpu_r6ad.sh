#!/bin/bash
# round 6 (ad): prefill (config 4, Llama-3.2-3B T 4096) on the final tree: rocprofv3 kernel stats, then
# an MFMA counter pass (busy cycles, clock) -- the final tree (wave-per-row norms)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r6ad
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats -o pf -- \
  python3 tools/bench_prefill.py --iters 2 --check 4 > $o/stats_log.txt 2>&1 || { echo "stats failed"; tail -5 $o/stats_log.txt; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $o/pmc -o pf -- \
  python3 tools/bench_prefill.py --iters 1 --check 4 > $o/pmc_log.txt 2>&1 || { echo "pmc failed"; tail -5 $o/pmc_log.txt; exit 1; }
find $o -name "*counter_collection.csv" | head -1 | xargs -I{} python3 tools/mfma_util.py {} > $o/mfma.txt
cat $o/mfma.txt
echo done
