#!/bin/bash
# round 4 (q): split units without the speculative first-chunk load (YALM_ATTN_SPEC_SPLIT=0):
# parity, kernel times over contexts, FETCH_SIZE of the fused launch, bench A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4q
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_attn_wo.py tests/test_gpu_kernels.py -k "attn or mha" > $o/tests.log 2>&1 || { echo "tests failed"; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
NEW=yalm_amd/ab/libyalm_hip_wt_ab.so
for dt in fp8 fp16; do
  for sp in 1 0 1 0; do
    YALM_LIB=$NEW YALM_ATTN_SPEC_SPLIT=$sp timeout -k 10 200 python tools/kernel_times.py --dtype $dt --iters 128 \
      --ctxs 16,100,250,500,1000,4000 --kernels 1,8 > $o/kt_${dt}_$sp.txt 2>&1 || { echo "kt failed"; tail -5 $o/kt_${dt}_$sp.txt; exit 1; }
    echo "$dt spec $sp attn: $(grep ' 1 attention' $o/kt_${dt}_$sp.txt | awk '{printf "%s ", $4}')  attn+Wo: $(grep ' 8 attn' $o/kt_${dt}_$sp.txt | awk '{printf "%s ", $4}')"
  done
done
for dt in fp8 fp16; do
  for sp in 1 0 1 0; do
    r=$(YALM_LIB=$NEW YALM_ATTN_SPEC_SPLIT=$sp timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-envelope --no-prefill --no-fp8 --dtype $dt | \
        python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'], d['long_context']['value'])")
    echo "$dt spec $sp bench(20) / long: $r tok/s"
  done
done
echo done
