#!/bin/bash
# Interleaved A/B (separate processes, one box) of environment settings for the decode
# GEMVs: per-kernel times (tools/kernel_times.py) and the bench at the driver's 20 steps.
# usage: tools/ab_gemv_env.sh fp16|fp8 "YALM_GEMV_XREG=0" "YALM_GEMV_XREG=1" ...
dt=$1; shift
for rep in 1 2; do
  for setting in "$@"; do
    k=$(env $setting timeout -k 5 60 python tools/kernel_times.py --iters 256 --ctx 16 --dtype $dt | awk '/ QKV /{q=$3} /W1\|W3/{g=$3} / W2 /{w=$3} END{print "QKV "q" GLU "g" W2 "w}')
    v=$(env $setting timeout -k 5 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-envelope --no-prefill --no-fp8 --dtype $dt | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'])")
    echo "$dt rep $rep [$setting]: $k us, bench(20) $v tok/s"
  done
done
