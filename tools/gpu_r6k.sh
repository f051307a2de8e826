#!/bin/bash
# round 6 (k): the GPU suite on the rebuilt tree, then the fused attention + Wo timeline with the
# key-mode phases stamped (merger spin / fold, partial issue) at kv 151 and 4096 (fp16) and 4096 (fp8
# hydrated one forward at a time is too slow: fp16 only at long context)
o=gpurun_out/r6k; mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -s --timeout 900 --timeout-method thread > $o/tests.log 2>&1
rc=$?
tail -5 $o/tests.log
[ $rc -eq 0 ] || { echo "suite failed rc=$rc"; grep -E "FAILED|Error" $o/tests.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $o/smoke.log; exit 1; }
tail -3 $o/smoke.log
export YALM_LIB=$PWD/yalm_amd/ab/libyalm_hip_wt_ab.so
for ctx in 150 4095; do
  timeout -k 10 240 python -u tools/attn_wo_trace.py --ctx $ctx --time 200 > $o/trace_fp16_$ctx.txt 2>&1 || { echo "trace $ctx failed"; tail -20 $o/trace_fp16_$ctx.txt; exit 1; }
  cat $o/trace_fp16_$ctx.txt
done
timeout -k 10 180 ./tools/qkv_epi_bench > $o/qkv_epi.txt 2>&1 || { echo "epi bench failed"; tail -20 $o/qkv_epi.txt; exit 1; }
cat $o/qkv_epi.txt
