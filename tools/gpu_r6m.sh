#!/bin/bash
# round 6 (m): the key split with a fence-free hand-off (sc1 stores / loads, relaxed add), attention
# parity tests, A/B of the Llama-3B 4096 prefill; the QKV epilogue variants (LDS RoPE table)
o=gpurun_out/r6m; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_prefill.py -k "attn_prefill or ksplit" > $o/tests.txt 2>&1 || { echo "tests failed"; tail -30 $o/tests.txt; exit 1; }
tail -2 $o/tests.txt
timeout -k 10 300 python3 -u tools/ab_prefill_forms.py --rounds 5 base=ksplit:0,wnorm:0 wn=ksplit:0 both= ks32=ksplit:32 > $o/ab_fast.txt 2>&1 || { echo "ab failed"; tail -20 $o/ab_fast.txt; exit 1; }
cat $o/ab_fast.txt
timeout -k 10 180 ./tools/qkv_epi_bench > $o/qkv_epi.txt 2>&1 || { echo "epi bench failed"; tail -20 $o/qkv_epi.txt; exit 1; }
cat $o/qkv_epi.txt
