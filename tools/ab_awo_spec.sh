#!/bin/bash
# A/B of the speculative granule gather in the fused attention + Wo launch
# (YALM_AWO_SPEC): per-launch time (kernel id 8) at two contexts and the decode
# bench, interleaved on one box
for rep in 1 2 3; do
  for sp in 0 1; do
    k1=$(YALM_AWO_SPEC=$sp timeout -k 5 60 python tools/kernel_times.py --iters 256 --ctx 16 | grep "attn+Wo gran" | awk '{print $4}')
    k2=$(YALM_AWO_SPEC=$sp timeout -k 5 60 python tools/kernel_times.py --iters 256 --ctx 150 | grep "attn+Wo gran" | awk '{print $4}')
    v=$(YALM_AWO_SPEC=$sp timeout -k 5 120 python bench.py --steps 64 --no-cpu-baseline | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'])")
    echo "rep $rep spec $sp : attn+Wo kv17 $k1 us, kv151 $k2 us, bench $v tok/s"
  done
done
