#!/bin/bash
# Interleaved A/B of two library builds on one box: standalone attention (kernel 1),
# plain Wo GEMV (2) and fused attention + Wo (8) at several contexts, then the decode
# bench at the driver's 20 steps.  usage: tools/ab_lib.sh A.so B.so "fp16 fp8" "16 150 1000"
a=$1; b=$2; dts=${3:-"fp16 fp8"}; ctxs=${4:-"16 150 1000"}
for rep in 1 2; do
  for dt in $dts; do
    for ctx in $ctxs; do
      for lib in $a $b; do
        r=$(YALM_LIB=$lib timeout -k 5 120 python tools/kernel_times.py --iters 256 --ctx $ctx --dtype $dt | \
            awk '$1=="1"{at=$3} $1=="2"{wo=$3} $1=="8"{f=$4} END{print "attn "at"  Wo "wo"  attn+Wo "f}')
        echo "rep $rep $dt kv $((ctx + 1)) $(basename $lib): $r us"
      done
    done
    for lib in $a $b; do
      v=$(YALM_LIB=$lib timeout -k 5 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-envelope --no-prefill --no-fp8 --dtype $dt | \
          python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'])")
      echo "rep $rep $dt bench(20) $(basename $lib): $v tok/s"
    done
  done
done
