#!/bin/bash
# round 4 (f): decode attention head mode -- parity, then head_max sweep (A/B build) and prefill A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4f
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_ref_infer.py tests/test_gpu_kernels.py tests/test_gpu_attn_wo.py tests/test_gpu_mistral_dims.py \
  tests/test_gpu_decode.py > $o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $o/tests.log | head -20; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
AB=$(ls yalm_amd/ab/libyalm_hip_*_ab.so | head -1)
for dt in fp16 fp8; do
  for hm in 0 1 2 4 8; do
    echo "== $dt head_max $hm"
    YALM_LIB=$AB YALM_ATTN_HEADMAX=$hm timeout -k 10 200 python tools/kernel_times.py --dtype $dt --iters 128 \
      --ctxs 16,100,150,250,500 --kernels 1,8 > $o/kt_${dt}_$hm.txt 2>&1 || { echo "kt failed"; tail -5 $o/kt_${dt}_$hm.txt; exit 1; }
    grep -E "kv_len| 1 | 8 " $o/kt_${dt}_$hm.txt | awk '/kv_len/{kv=$5} / 1 attention/{a=$3} / 8 attn/{print "kv " kv ": attn " a "  attn+Wo " $4}'
  done
done
for dt in fp16 fp8; do
  for hm in 0 4 0 4; do
    v=$(YALM_LIB=$AB YALM_ATTN_HEADMAX=$hm timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-envelope --no-prefill --no-fp8 --no-long --dtype $dt | \
        python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'])")
    echo "$dt head_max $hm bench(20): $v tok/s"
  done
done
for lib in yalm_amd/ab/libyalm_hip_6ee20fc.so yalm_amd/libyalm_hip.so yalm_amd/ab/libyalm_hip_6ee20fc.so yalm_amd/libyalm_hip.so; do
  echo "$(basename $lib): $(YALM_LIB=$lib timeout -k 10 300 python tools/bench_prefill.py --iters 3 --check 8 | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'], 'ms', d['roofline']['achieved'], 'TF/s')")"
done
echo done
