#!/bin/bash
# A/B of the W1|W3 GEMV W3 row rotation (YALM_GLU_W3_ROT): per-launch GLU time
# (kernel_times, layers rotated) and the decode bench, interleaved on one box
for rep in 1 2 3; do
  for rot in 0 1; do
    k=$(YALM_GLU_W3_ROT=$rot timeout -k 5 60 python tools/kernel_times.py --iters 256 | grep "W1|W3")
    v=$(YALM_GLU_W3_ROT=$rot timeout -k 5 120 python bench.py --steps 64 --no-cpu-baseline | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'], d['roofline']['avg_launch_us'])")
    echo "rep $rep rot $rot : bench $v | $k"
  done
done
