#!/bin/bash
# round 4 (e): prefill with the split-f16 K / V operand -- parity, precision at depth, time
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4e
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_prefill.py tests/test_host.py > $o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $o/tests.log | head -20; tail -30 $o/tests.log; exit 1; }
tail -3 $o/tests.log
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread \
  tests/test_gpu_prefill_llama.py -k "not full_4096" > $o/prefill_depth.log 2>&1
rc=$?; [ $rc -gt 1 ] && { echo "prefill depth test crashed rc=$rc"; tail -20 $o/prefill_depth.log; exit 1; }
grep -E "llama-3b dims|passed|failed" $o/prefill_depth.log
for lib in yalm_amd/ab/libyalm_hip_6ee20fc.so yalm_amd/libyalm_hip.so yalm_amd/ab/libyalm_hip_6ee20fc.so yalm_amd/libyalm_hip.so; do
  echo "$(basename $lib): $(YALM_LIB=$lib timeout -k 10 300 python tools/bench_prefill.py --iters 3 --check 8)"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/pfprof -o pf -- \
    python3 tools/bench_prefill.py --iters 2 --check 4 > $o/pfprof.log 2>&1 || { echo "prof failed"; tail -5 $o/pfprof.log; exit 1; }
python tools/kstats.py $o/pfprof 14
echo done
