#!/bin/bash
# round 6: epilogue A/B (round-5 vs templated) + prefill tests + prefill kernel stats
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r6j; mkdir -p $o
timeout -k 10 120 ./tools/gemm_epi_bench > $o/epi_ab.txt 2>&1 || { echo "epi bench failed"; tail -20 $o/epi_ab.txt; exit 1; }
cat $o/epi_ab.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_prefill.py tests/test_gpu_prefill_llama.py > $o/tests.txt 2>&1 || { echo "tests failed"; tail -30 $o/tests.txt; exit 1; }
tail -3 $o/tests.txt
for form in fast split; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace_$form -o pf -- \
    python3 tools/prefill_once.py $form > $o/pf_$form.log 2>&1 || { echo "$form failed"; tail -20 $o/pf_$form.log; exit 1; }
  echo "$form ok"; tail -2 $o/pf_$form.log
done
