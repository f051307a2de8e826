#!/bin/bash
# round 4 (n): fused attention + Wo with the first Wo workgroups launched before the mergers
# (the mergers share the head units' CUs) -- parity, A/B YALM_AWO_EARLY, traces, bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4n
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_attn_wo.py tests/test_gpu_decode.py > $o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $o/tests.log | head -20; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
NEW=yalm_amd/ab/libyalm_hip_wt_ab.so
for dt in fp8 fp16; do
  for e in 0 1; do
    for dl in 20 50; do
      YALM_LIB=$NEW YALM_AWO_EARLY=$e YALM_ATTN_WO_DELAY=$dl timeout -k 10 200 python tools/kernel_times.py --dtype $dt --iters 128 \
        --ctxs 16,100,250,500,1000,4000 --kernels 8 > $o/kt_${dt}_e${e}_d$dl.txt 2>&1 || { echo "kt failed"; tail -5 $o/kt_${dt}_e${e}_d$dl.txt; exit 1; }
      echo "$dt early $e delay $dl: $(grep ' 8 attn' $o/kt_${dt}_e${e}_d$dl.txt | awk '{printf "%s ", $4}')"
    done
  done
done
for dt in fp8 fp16; do
  for ctx in 16 150; do
    YALM_LIB=$NEW timeout -k 10 120 python tools/attn_wo_trace.py --dtype $dt --ctx $ctx > $o/trace_${dt}_$ctx.txt 2>&1 || { echo "trace failed"; tail -5 $o/trace_${dt}_$ctx.txt; exit 1; }
    echo "== trace $dt ctx $ctx"; grep -E "span|loads landed|P.V in|P.V->|head signalled|Wo slice|Wo poll|Wo end|poll->end" $o/trace_${dt}_$ctx.txt
  done
done
for dt in fp8 fp16; do
  for e in 0 1 0 1; do
    r=$(YALM_LIB=$NEW YALM_AWO_EARLY=$e timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-envelope --no-prefill --no-fp8 --no-long --dtype $dt | \
        python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'])")
    echo "$dt early $e bench(20): $r tok/s"
  done
done
echo done
