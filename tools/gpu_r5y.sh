#!/bin/bash
# round 5 (y): graph replays vs eager launches for the timed greedy decode, interleaved (fp16 and fp8)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r5y
mkdir -p $o
for r in 1 2 3; do
  for m in graph eager; do
    e=0; [ $m = eager ] && e=1
    YALM_EAGER=$e timeout -k 10 200 python bench.py --steps 64 --warmup 5 --no-prefill --no-long --no-cpu-baseline --no-envelope --no-gpu-state > $o/$m.$r.json 2> $o/$m.$r.err || { echo "$m failed"; tail -5 $o/$m.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$o/$m.$r.json')); print('round $r $m', 'fp16', d['value'], 'fp8', d['fp8'].get('value'))"
  done
done
