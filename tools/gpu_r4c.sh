#!/bin/bash
# round 4 (b): long-kv attention rework -- GPU parity of everything attention touches, then an
# interleaved A/B against the previous library (tools/ab_lib.sh) and the long-context leg.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4c
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_ref_infer.py tests/test_gpu_kernels.py tests/test_gpu_attn_wo.py tests/test_gpu_mistral_dims.py \
  tests/test_gpu_decode.py > $o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $o/tests.log | head -20; tail -30 $o/tests.log; exit 1; }
tail -3 $o/tests.log
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread \
  "tests/test_gpu_prefill_llama.py::test_prefill_llama3b_full_depth_vs_oracle" > $o/prefill_depth.log 2>&1
rc=$?; [ $rc -gt 1 ] && { echo "prefill depth test crashed rc=$rc"; tail -20 $o/prefill_depth.log; exit 1; }
grep -E "llama-3b dims|passed|failed" $o/prefill_depth.log
OLD=yalm_amd/ab/libyalm_hip_6ee20fc.so
NEW=yalm_amd/libyalm_hip.so
for lib in $OLD $NEW; do
  YALM_LIB=$lib timeout -k 10 300 python bench.py --long-only --long-steps 64 > $o/long_$(basename $lib).json 2>$o/long_$(basename $lib).err || { echo "long failed $lib"; tail -5 $o/long_$(basename $lib).err; exit 1; }
  echo "$(basename $lib): $(cat $o/long_$(basename $lib).json)"
done
timeout -k 10 600 bash tools/ab_lib.sh $OLD $NEW "fp16 fp8" "16 150 1000 4095" > $o/ab.txt 2>&1 || { echo "ab failed"; tail -20 $o/ab.txt; exit 1; }
cat $o/ab.txt
echo done
