#!/bin/bash
# interleaved A/B of GEMV geometries on one box (bench.py --steps 64)
for rep in 1 2 3; do
  for cfg in "" "2:512:2:2" "2:512:2:2,0:512:4:2" "0:512:4:2"; do
    v=$(YALM_GEMV_CFG="$cfg" timeout -k 5 120 python bench.py --steps 64 --no-cpu-baseline | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'], d['roofline']['avg_launch_us'])")
    echo "rep $rep cfg [$cfg] : $v"
  done
done
