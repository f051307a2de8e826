#!/bin/bash
# A/B of the fused attention + Wo hand-off's combined first attempt (YALM_AWO_SPEC,
# attn_wo.h awo_gather_gran): per-launch time (kernel id 8, fresh epoch per launch)
# at two contexts next to the plain Wo GEMV (id 2), and the decode bench at the
# driver's 20 steps, interleaved on one box. usage: tools/ab_awo_spec.sh [fp16|fp8]
dt=${1:-fp16}
for rep in 1 2; do
  for sp in 0 1; do
    k1=$(YALM_AWO_SPEC=$sp timeout -k 5 60 python tools/kernel_times.py --iters 256 --ctx 16 --dtype $dt | awk '/attn\+Wo gran/{a=$4} / Wo /{w=$3} END{print a" (Wo "w")"}')
    k2=$(YALM_AWO_SPEC=$sp timeout -k 5 60 python tools/kernel_times.py --iters 256 --ctx 150 --dtype $dt | awk '/attn\+Wo gran/{a=$4} / Wo /{w=$3} END{print a" (Wo "w")"}')
    v=$(YALM_AWO_SPEC=$sp timeout -k 5 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-envelope --dtype $dt | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'])")
    echo "$dt rep $rep spec $sp : attn+Wo kv17 $k1 us, kv151 $k2 us, bench(20) $v tok/s"
  done
done
