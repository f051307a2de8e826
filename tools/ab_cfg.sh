#!/bin/bash
# Interleaved A/B (separate processes, one box) of decode GEMV geometries
# (YALM_GEMV_CFG="kind:threads:unroll:wg_per_cu", kinds 0 QKV 1 Wo 2 W1|W3 3 W2 4 logits):
# per-kernel times (tools/kernel_times.py) and the bench at the driver's 20 steps.
# usage: tools/ab_cfg.sh fp16|fp8 "" "3:512:4:1" ...   ("" = defaults)
dt=$1; shift
for rep in 1 2; do
  for cfg in "$@"; do
    k=$(YALM_GEMV_CFG="$cfg" timeout -k 5 60 python tools/kernel_times.py --iters 256 --ctx 16 --dtype $dt | awk '/ QKV /{q=$3} /W1\|W3/{g=$3} / W2 /{w=$3} END{print "QKV "q" GLU "g" W2 "w}')
    v=$(YALM_GEMV_CFG="$cfg" timeout -k 5 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-envelope --no-prefill --no-fp8 --dtype $dt | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'])")
    echo "$dt rep $rep [cfg '$cfg']: $k us, bench(20) $v tok/s"
  done
done
