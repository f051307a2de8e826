#!/bin/bash
# round 4 (l): prefill -- parity, one-launch QKV A/B (YALM_PF_QKV1), small-T tables, small-T kernel profile
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4l
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_prefill.py tests/test_gpu_prefill_llama.py > $o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $o/tests.log | head -20; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
grep -E "layers,|positions:" $o/tests.log | head -5
for v in 1 0 1 0; do
  echo "prefill QKV1=$v: $(YALM_PF_QKV1=$v timeout -k 10 300 python tools/bench_prefill.py --iters 3 --check 8 | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'], 'ms', d['roofline']['achieved'], 'TF/s')")"
done
for m in mistral-7b llama-3.2-3b; do
  timeout -k 10 300 python tools/bench_small_prefill.py --model $m --ts 1,2,5,13,32,64 > $o/small_$m.txt 2>&1 || { echo "small failed"; tail -5 $o/small_$m.txt; exit 1; }
  cat $o/small_$m.txt
done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/sp -o sp -- python tools/bench_small_prefill.py --ts 1 --reps 3 > $o/sp.log 2>&1 || { echo "prof failed"; tail -5 $o/sp.log; exit 1; }
python tools/prof_summary.py $o/sp/sp_kernel_stats.csv > $o/sp_stats.txt; head -24 $o/sp_stats.txt
echo done
