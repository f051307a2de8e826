#!/bin/bash
# Timelines of the fused attention + Wo launch (tools/attn_wo_trace.py) for fp16 / fp8 at
# several contexts, and with the Wo weight stream removed (YALM_ABLATE=32, timing only).
set -e
for dt in fp16; do for c in 16 150; do
echo "== $dt ctx $c"; timeout -k 10 90 python tools/attn_wo_trace.py --dtype $dt --ctx $c
done; done
for c in 16; do
echo "== fp16 ctx $c, no Wo weight loads"; YALM_ABLATE=32 timeout -k 10 90 python tools/attn_wo_trace.py --dtype fp16 --ctx $c
done

echo "== fp16 ctx 16, Wo slice loads delayed 1 us"; YALM_ATTN_WO_DELAY=100 timeout -k 10 90 python tools/attn_wo_trace.py --dtype fp16 --ctx 16
