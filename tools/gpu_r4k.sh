#!/bin/bash
# round 4 (k): decode -- parity, then A/B (dc1e452 / working tree / working tree with the
# sentinel poll first): kernel times, fused-launch traces, 20-step bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4k
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_attn_wo.py tests/test_gpu_decode.py tests/test_gpu_ref_infer.py > $o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $o/tests.log | head -20; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
OLD=yalm_amd/ab/libyalm_hip_dc1e452_ab.so
NEW=yalm_amd/ab/libyalm_hip_wt_ab.so
for dt in fp8 fp16; do
  for v in old new new-g0; do
    lib=$NEW; g=1; [ $v = old ] && lib=$OLD; [ $v = new-g0 ] && g=0
    YALM_LIB=$lib YALM_AWO_GFIRST=$g timeout -k 10 200 python tools/kernel_times.py --dtype $dt --iters 128 \
      --ctxs 16,100,250,500,1000,4000 --kernels 1,2,4,8 > $o/kt_${dt}_$v.txt 2>&1 || { echo "kt failed"; tail -5 $o/kt_${dt}_$v.txt; exit 1; }
    echo "== $dt $v"
    awk '/kv_len/{kv=$5} / 1 attention/{a=$3} / 2 Wo/{w=$3} / 4 W2/{w2=$3} / 8 attn/{print "kv " kv ": attn " a "  Wo " w "  W2 " w2 "  attn+Wo " $4}' $o/kt_${dt}_$v.txt
  done
done
for dt in fp8 fp16; do
  for ctx in 16 150 1000; do
    YALM_LIB=$NEW timeout -k 10 120 python tools/attn_wo_trace.py --dtype $dt --ctx $ctx > $o/trace_${dt}_$ctx.txt 2>&1 || { echo "trace failed"; tail -5 $o/trace_${dt}_$ctx.txt; exit 1; }
    echo "== trace $dt ctx $ctx"; grep -E "span|loads landed|head signalled|merger|Wo slice|Wo poll|Wo end|poll->end" $o/trace_${dt}_$ctx.txt
  done
done
for dt in fp8 fp16; do
  for v in old new new-g0 old new new-g0; do
    lib=$NEW; g=1; [ $v = old ] && lib=$OLD; [ $v = new-g0 ] && g=0
    r=$(YALM_LIB=$lib YALM_AWO_GFIRST=$g timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-envelope --no-prefill --no-fp8 --no-long --dtype $dt | \
        python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'])")
    echo "$dt $v bench(20): $r tok/s"
  done
done
echo done
