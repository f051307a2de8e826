#!/bin/bash
# round 4 (t): skinny prefill with LDS-DMA weight stages + batched A staging -- parity, small-T A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4t
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_prefill.py -k "short_prompt or forms_match or matches_decode" > $o/tests.log 2>&1 || { echo "tests failed"; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for v in 1 0; do
  for m in mistral-7b llama-3.2-3b; do
    YALM_PF_SKL=$v timeout -k 10 300 python tools/bench_small_prefill.py --model $m --ts 1,2,5,13,32,64 > $o/small_${m}_$v.txt 2>&1 || { echo "small failed"; tail -5 $o/small_${m}_$v.txt; exit 1; }
    echo "SKL=$v"; cat $o/small_${m}_$v.txt
  done
done
echo done
