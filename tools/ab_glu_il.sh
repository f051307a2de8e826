#!/bin/bash
# A/B of the interleaved W1|W3 copy (YALM_GLU_INTERLEAVE=1) vs the two separate
# matrices: per-launch GLU time (kernel_times, layers rotated) and the decode
# bench, interleaved on one box
for rep in 1 2 3; do
  for il in 0 1; do
    k=$(YALM_GLU_INTERLEAVE=$il timeout -k 5 60 python tools/kernel_times.py --iters 256 | grep "W1|W3")
    v=$(YALM_GLU_INTERLEAVE=$il timeout -k 5 120 python bench.py --steps 64 --no-cpu-baseline | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'], d['roofline']['avg_launch_us'])")
    echo "rep $rep interleave $il : bench $v | $k"
  done
done
