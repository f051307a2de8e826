#!/bin/bash
# round 4 (x): prefill causal attention with 32-key tiles (3 workgroups per CU) -- parity, A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4x
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_prefill.py -k "attn_prefill or forms_match" > $o/tests.log 2>&1 || { echo "tests failed"; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for v in 64 32 33 64 32 33; do
  echo "AKT=$v: $(YALM_PF_AKT=$v timeout -k 10 300 python tools/bench_prefill.py --iters 3 --check 8 | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'], 'ms', d['roofline']['achieved'], 'TF/s', d['spot_check']['max_abs_dlogp_vs_decode'])")"
done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
YALM_PF_AKT=33 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/pf -o pf -- python3 tools/bench_prefill.py --iters 3 --check 1 > $o/pf.log 2>&1 || { echo "pf prof failed"; exit 1; }
python tools/prof_summary.py $o/pf/pf_kernel_stats.csv | head -8
echo done
