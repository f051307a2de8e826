#!/bin/bash
# Timing ablation: bench with parts of the layer skipped (YALM_ABLATE bitmask).
for m in 0 1 2 4 8 16 30 31; do
  v=$(YALM_ABLATE=$m python bench.py --steps 128 --warmup 4 --no-cpu-baseline | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")
  echo "ablate=$m ms_per_step=$v"
done
