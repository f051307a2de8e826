#!/bin/bash
# round 6: rocprofv3 kernel stats of the Llama-3.2-3B 4096-position prefill, fast and split forms
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r6i; mkdir -p $o
for form in fast split; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace_$form -o pf -- \
    python3 tools/prefill_once.py $form > $o/pf_$form.log 2>&1 || { echo "$form failed"; tail -20 $o/pf_$form.log; exit 1; }
  echo "$form ok"; tail -2 $o/pf_$form.log
done
