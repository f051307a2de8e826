#!/bin/bash
# round 6: prefill attention A/B (setprio), split-form attention cost; prefill leg (both forms)
o=gpurun_out/r6e; mkdir -p $o
timeout -k 10 120 ./tools/attn_pf_bench 4096 7 10 > $o/attn_pf.txt 2>&1 || { echo "attn bench failed"; cat $o/attn_pf.txt; exit 1; }
cat $o/attn_pf.txt
timeout -k 10 300 python -c "
import json, bench
from yalm_amd import runtime as R, models as M
print(json.dumps(bench.prefill_leg(R, M, iters=3)))
" > $o/prefill_leg.json 2> $o/prefill_leg.err || { echo "prefill leg failed"; tail $o/prefill_leg.err; exit 1; }
cat $o/prefill_leg.json
