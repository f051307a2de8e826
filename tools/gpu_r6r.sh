#!/bin/bash
# round 6 (r): prefill causal attention, K / V staged through registers (RSTG) vs LDS-DMA
o=gpurun_out/r6r; mkdir -p $o
timeout -k 10 120 ./tools/attn_pf_bench 4096 7 10 > $o/attn_pf.txt 2>&1 || { echo "bench failed"; tail -20 $o/attn_pf.txt; exit 1; }
cat $o/attn_pf.txt
timeout -k 10 120 ./tools/attn_pf_bench 1024 7 20 >> $o/attn_pf.txt 2>&1 || { echo "bench 1024 failed"; exit 1; }
tail -4 $o/attn_pf.txt
