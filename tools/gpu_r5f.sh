#!/bin/bash
# round 5 (f): granule IPC exchange (no counters): TP tests, the TP1 per-kernel cost against one
# GPU (rocprofv3, eager launches), then the Mistral-dims TP2/4/8 parity
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r5f
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_tp.py -x -v --timeout 300 --timeout-method thread > $o/tp.log 2>&1 || { echo "tp tests failed"; grep -E "FAILED|Error|error|assert" $o/tp.log | head -30; tail -20 $o/tp.log; exit 1; }
tail -1 $o/tp.log
for m in single ipc; do
  extra=""; [ $m = ipc ] && extra="--tp --tp-transport ipc"
  YALM_EAGER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace_$m -o k -- \
    python3 bench.py --steps 32 --warmup 4 --no-cpu-baseline --no-gpu-state --no-prefill --no-fp8 --no-long --no-envelope $extra > $o/bench_$m.log 2>&1 || { echo "trace $m failed"; tail -5 $o/bench_$m.log; exit 1; }
  f=$(ls $o/trace_$m/*kernel_stats.csv | head -1)
  python3 tools/prof_summary.py $f > $o/stats_$m.txt
  head -12 $o/stats_$m.txt
done
timeout -k 10 300 python bench.py --steps 64 --warmup 5 --tp --tp-transport ipc --no-cpu-baseline --no-prefill --no-fp8 --no-long > $o/bench_tp1_ipc.json 2> $o/bench_tp1_ipc.err || { echo "tp1 ipc failed"; tail -20 $o/bench_tp1_ipc.err; exit 1; }
python3 -c "import json; d=json.load(open('$o/bench_tp1_ipc.json')); print('tp1 ipc', d['value'], 'k/tok', d.get('kernels_per_token'), d['config']['parallelism'])"
timeout -k 10 900 python -u -m pytest tests/test_gpu_mistral_dims.py -x -v --timeout 400 --timeout-method thread -k "tensor_parallel" > $o/tp_mistral.log 2>&1 || { echo "tp mistral failed"; grep -E "FAILED|Error|error|assert" $o/tp_mistral.log | head -30; tail -20 $o/tp_mistral.log; exit 1; }
tail -1 $o/tp_mistral.log
