#!/bin/bash
# Interleaved A/B of environment settings on one box: per-launch fused attention +
# Wo time (kernel id 8, fresh epoch per launch) next to the plain Wo GEMV (id 2) at
# kv_len 17 and 151, and the decode bench at the driver's 20 steps.
# usage: tools/ab_env.sh fp16|fp8 "A=1 B=2" "A=3" ...   (each arg: one setting)
dt=$1; shift
for rep in 1 2; do
  for setting in "$@"; do
    k1=$(env $setting timeout -k 5 60 python tools/kernel_times.py --iters 256 --ctx 16 --dtype $dt | awk '/attn\+Wo gran/{a=$4} / Wo /{w=$3} END{print a" (Wo "w")"}')
    k2=$(env $setting timeout -k 5 60 python tools/kernel_times.py --iters 256 --ctx 150 --dtype $dt | awk '/attn\+Wo gran/{a=$4} / Wo /{w=$3} END{print a" (Wo "w")"}')
    v=$(env $setting timeout -k 5 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-envelope --no-prefill --no-fp8 --dtype $dt | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'])")
    echo "$dt rep $rep [$setting]: attn+Wo kv17 $k1 us, kv151 $k2 us, bench(20) $v tok/s"
  done
done
