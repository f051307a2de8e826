#!/bin/bash
# Interleaved A/B (separate processes, same box) of the decode GEMV's whole-row mode
# (gemv.h ROWS; YALM_GEMV_ROWS=0 = chunk order): per-kernel times (tools/kernel_times.py)
# and the decode bench at the driver's 20 steps.   usage: tools/ab_rows.sh [fp16|fp8 ...]
for rep in 1 2 3; do
  for dt in ${@:-fp16 fp8}; do
    for setting in "YALM_GEMV_ROWS=1" "YALM_GEMV_ROWS=0"; do
      k=$(env $setting timeout -k 5 60 python tools/kernel_times.py --iters 256 --ctx 16 --dtype $dt | awk '/ QKV /{q=$3} /W1\|W3/{g=$3} / W2 /{w=$3} END{print "QKV "q" GLU "g" W2 "w}')
      v=$(env $setting timeout -k 5 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-envelope --dtype $dt | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'])")
      echo "$dt rep $rep [$setting]: $k us, bench(20) $v tok/s"
    done
  done
done
