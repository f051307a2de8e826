#!/bin/bash
# round 5 (s): A/B of the fused attention + Wo sentinel poll: one sample at a time (AWO_POLL_PAIR=0)
# against two staggered samples in flight (8 / 16 sleep units apart); A/B builds of the working tree
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r5s
mkdir -p $o
for v in "" _p8 _p16; do
  YALM_LIB=$PWD/yalm_amd/ab/libyalm_hip_wt_ab$v.so timeout -k 10 200 python -u tools/awo_delay_sweep.py --ctx 16,150,1023,4095 --delays 20 > $o/awo$v.txt 2>&1 || { echo "sweep $v failed"; tail -5 $o/awo$v.txt; exit 1; }
  YALM_LIB=$PWD/yalm_amd/ab/libyalm_hip_wt_ab$v.so timeout -k 10 200 python -u tools/awo_delay_sweep.py --dtype fp8 --ctx 16,150,1023 --delays 50 > $o/awo8$v.txt 2>&1 || { echo "sweep8 $v failed"; tail -5 $o/awo8$v.txt; exit 1; }
  echo "lib$v"; tail -n 1 $o/awo$v.txt; tail -n 1 $o/awo8$v.txt
done
for r in 1 2; do
  for v in "" _p8 _p16; do
    YALM_LIB=$PWD/yalm_amd/ab/libyalm_hip_wt_ab$v.so timeout -k 10 300 python bench.py --steps 64 --warmup 5 --no-prefill --no-cpu-baseline --no-long --no-envelope --no-gpu-state > $o/b$v.$r.json 2> $o/b$v.$r.err || { echo "bench $v failed"; tail -5 $o/b$v.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$o/b$v.$r.json')); print('round $r lib$v', 'fp16', d['value'], 'fp8', d['fp8'].get('value'))"
  done
done
echo done
