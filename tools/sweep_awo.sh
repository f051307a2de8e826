#!/bin/bash
# sweep the fused attention + Wo launch knobs: per-launch time (kernel id 8)
for ctx in 16 150; do
for dl in 0 20 40 60; do
for win in 0 16 24; do
  r=$(YALM_ATTN_WO_DELAY=$dl YALM_ATTN_WO_WIN=$win timeout -k 5 60 python tools/kernel_times.py --ctx $ctx --iters 256 2>&1 | grep "attn+Wo gran")
  echo "ctx $ctx delay $dl win $win : $r"
done; done; done
