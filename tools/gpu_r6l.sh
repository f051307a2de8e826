#!/bin/bash
# round 6 (l): causal attention key split (prefill.h KSPLIT): parity tests, then A/B of the
# whole Llama-3B 4096 prefill (fast and split forms) against the plain grid
o=gpurun_out/r6l; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_prefill.py tests/test_gpu_prefill_llama.py > $o/tests.txt 2>&1 || { echo "tests failed"; tail -30 $o/tests.txt; exit 1; }
tail -3 $o/tests.txt
timeout -k 10 300 python3 -u tools/ab_prefill_forms.py --rounds 7 base=ksplit:0,wnorm:0 ks=wnorm:0 wn=ksplit:0 both= ks8=ksplit:8 > $o/ab_fast.txt 2>&1 || { echo "ab failed"; tail -20 $o/ab_fast.txt; exit 1; }
cat $o/ab_fast.txt
timeout -k 10 300 python3 -u tools/ab_prefill_forms.py --split --rounds 5 base=ksplit:0,wnorm:0 both= > $o/ab_split.txt 2>&1 || { echo "ab split failed"; tail -20 $o/ab_split.txt; exit 1; }
cat $o/ab_split.txt
