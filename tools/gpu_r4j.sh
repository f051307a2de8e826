#!/bin/bash
# round 4 (i, j): attention head units + split units (no speculation miss), residual rows
# prefetched in the Wo / W2 epilogues, pipelined skinny prefill -- parity, A/B kernel
# times, delay sweep, traces, bench A/B, small-T prefill
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4j
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_attn_wo.py tests/test_gpu_decode.py tests/test_gpu_ref_infer.py tests/test_gpu_prefill.py tests/test_gpu_prefill_llama.py > $o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $o/tests.log | head -20; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
OLD=yalm_amd/ab/libyalm_hip_dc1e452_ab.so
NEW=yalm_amd/ab/libyalm_hip_wt_ab.so
for dt in fp8 fp16; do
  for lib in $OLD $NEW; do
    n=$(basename $lib .so)
    YALM_LIB=$lib timeout -k 10 200 python tools/kernel_times.py --dtype $dt --iters 128 \
      --ctxs 16,100,150,250,500,1000,4000 --kernels 1,2,4,8 > $o/kt_${dt}_$n.txt 2>&1 || { echo "kt failed"; tail -5 $o/kt_${dt}_$n.txt; exit 1; }
    echo "== $dt $n"
    awk '/kv_len/{kv=$5} / 1 attention/{a=$3} / 2 Wo/{w=$3} / 4 W2/{w2=$3} / 8 attn/{print "kv " kv ": attn " a "  Wo " w "  W2 " w2 "  attn+Wo " $4}' $o/kt_${dt}_$n.txt
  done
done
for dt in fp8 fp16; do
  for dl in 0 50 100 150; do
    YALM_LIB=$NEW YALM_ATTN_WO_DELAY=$dl timeout -k 10 200 python tools/kernel_times.py --dtype $dt --iters 128 \
      --ctxs 16,150,1000 --kernels 8 > $o/dl_${dt}_$dl.txt 2>&1 || { echo "dl failed"; tail -5 $o/dl_${dt}_$dl.txt; exit 1; }
    echo "$dt delay $dl: $(grep ' 8 attn' $o/dl_${dt}_$dl.txt | awk '{printf "%s ", $4}')"
  done
done
for dt in fp8 fp16; do
  for ctx in 16 150; do
    YALM_LIB=$NEW timeout -k 10 120 python tools/attn_wo_trace.py --dtype $dt --ctx $ctx > $o/trace_${dt}_$ctx.txt 2>&1 || { echo "trace failed"; tail -5 $o/trace_${dt}_$ctx.txt; exit 1; }
    echo "== trace $dt ctx $ctx"; grep -E "span|loads landed|head signalled|Wo slice|Wo poll|Wo end|poll->end" $o/trace_${dt}_$ctx.txt
  done
done
for dt in fp8 fp16; do
  for lib in $OLD $NEW $OLD $NEW; do
    v=$(YALM_LIB=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-envelope --no-prefill --no-fp8 --no-long --dtype $dt | \
        python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'])")
    echo "$dt $(basename $lib) bench(20): $v tok/s"
  done
done
for v in 1 0 1 0; do
  echo "prefill QKV1=$v: $(YALM_PF_QKV1=$v timeout -k 10 300 python tools/bench_prefill.py --iters 3 --check 8 | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'], 'ms', d['roofline']['achieved'], 'TF/s')")"
done
for m in mistral-7b llama-3.2-3b; do
  timeout -k 10 300 python tools/bench_small_prefill.py --model $m --ts 1,2,5,13,32,64 > $o/small_$m.txt 2>&1 || { echo "small failed"; tail -5 $o/small_$m.txt; exit 1; }
  cat $o/small_$m.txt
done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/sp -o sp -- python tools/bench_small_prefill.py --ts 1 --reps 3 > $o/sp.log 2>&1 || { echo "prof failed"; tail -5 $o/sp.log; exit 1; }
python tools/prof_summary.py $o/sp/sp_kernel_stats.csv > $o/sp_stats.txt; head -24 $o/sp_stats.txt
echo done
