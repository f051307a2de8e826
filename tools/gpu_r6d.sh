#!/bin/bash
# round 6: peaked-scale split prefill; config-5 rehearsal lines (N ranks on one GPU, CU-masked); N=1 bench
o=gpurun_out/r6d; mkdir -p $o
T="python -u -m pytest -x -v --timeout 900 --timeout-method thread -s"
timeout -k 10 600 $T tests/test_gpu_prefill_llama.py -k peaked > $o/pfl_peaked.log 2>&1 || { echo "pfl failed"; tail -30 $o/pfl_peaked.log; exit 1; }
grep -o "llama-3b dims, peaked.*" $o/pfl_peaked.log
for n in 2 4 8; do
  timeout -k 10 400 python bench.py --gpus $n --rehearse --steps 64 --warmup 5 --no-envelope > $o/bench_tp${n}_rehearsal.json 2> $o/bench_tp${n}.err || { echo "tp$n failed"; tail -20 $o/bench_tp${n}.err; exit 1; }
  cat $o/bench_tp${n}_rehearsal.json
done
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $o/bench_20.json 2> $o/bench_20.err || { echo "bench failed"; tail -20 $o/bench_20.err; exit 1; }
cat $o/bench_20.json
