#!/bin/bash
# round 4 (h): dual speculative first-chunk loads (attention key mode) -- parity, A/B kernel
# times against the previous build, fused-launch timelines, small-T prefill kernel profile
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4h
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_attn_wo.py tests/test_gpu_decode.py > $o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $o/tests.log | head -20; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for dt in fp8 fp16; do
  for lib in yalm_amd/ab/libyalm_hip_dc1e452_ab.so yalm_amd/ab/libyalm_hip_wt_ab.so; do
    n=$(basename $lib .so)
    YALM_LIB=$lib timeout -k 10 200 python tools/kernel_times.py --dtype $dt --iters 128 \
      --ctxs 16,100,150,250,500,1000,4000 --kernels 1,2,8 > $o/kt_${dt}_$n.txt 2>&1 || { echo "kt failed"; tail -5 $o/kt_${dt}_$n.txt; exit 1; }
    echo "== $dt $n"
    awk '/kv_len/{kv=$5} / 1 attention/{a=$3} / 2 Wo/{w=$3} / 8 attn/{print "kv " kv ": attn " a "  Wo " w "  attn+Wo " $4}' $o/kt_${dt}_$n.txt
  done
done
for dt in fp8 fp16; do
  for ctx in 16 150; do
    echo "== trace $dt ctx $ctx"
    YALM_LIB=yalm_amd/ab/libyalm_hip_wt_ab.so timeout -k 10 120 python tools/attn_wo_trace.py --dtype $dt --ctx $ctx > $o/trace_${dt}_$ctx.txt 2>&1 || { echo "trace failed"; tail -5 $o/trace_${dt}_$ctx.txt; exit 1; }
    cat $o/trace_${dt}_$ctx.txt
  done
done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/sp -o sp -- python tools/bench_small_prefill.py --ts 1 --reps 3 > $o/sp.log 2>&1 || { echo "prof failed"; tail -5 $o/sp.log; exit 1; }
cat $o/sp.log | grep -E "T "
python tools/prof_summary.py $o/sp/sp_kernel_stats.csv > $o/sp_stats.txt; head -40 $o/sp_stats.txt
echo done
