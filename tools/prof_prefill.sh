#!/bin/bash
# rocprofv3 kernel stats of the batched prefill (tools/bench_prefill.py), one run per
# setting given as "name|ENV=VAL ..." arguments; output under gpurun_out/pfprof_<name>/
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for spec in "$@"; do
  name="${spec%%|*}"; envs="${spec#*|}"
  out=gpurun_out/pfprof_$name
  mkdir -p $out
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o pf -- \
    python3 tools/bench_prefill.py --iters 2 --check 4 > $out/log.txt 2>&1 || exit $?
done
