#!/bin/bash
# round 5 (j): fused W2 + QKV, one-wave sentinel poll: A/B (interleaved) and per-kernel profile
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r5j
mkdir -p $o
export YALM_LIB=$PWD/yalm_amd/ab/libyalm_hip_wt_ab.so
for v in 0 1 0 1; do
  YALM_W2QKV=$v timeout -k 10 300 python bench.py --steps 64 --warmup 5 --no-cpu-baseline --no-prefill --no-long > $o/ab_$v.json 2> $o/ab_$v.err || { echo "ab $v failed"; tail -20 $o/ab_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/ab_$v.json')); print('W2QKV=$v fp16', d['value'], 'k/tok', d.get('kernels_per_token'), 'fp8', d['fp8']['value'])"
done
for v in 0 1; do
  YALM_W2QKV=$v YALM_EAGER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace_$v -o k -- \
    python3 bench.py --steps 32 --warmup 4 --dtype fp8 --no-cpu-baseline --no-gpu-state --no-prefill --no-fp8 --no-long --no-envelope > $o/prof_$v.log 2>&1 || { echo "trace $v failed"; tail -5 $o/prof_$v.log; exit 1; }
  f=$(ls $o/trace_$v/*kernel_stats.csv | head -1)
  python3 tools/prof_summary.py $f > $o/stats_$v.txt
  head -8 $o/stats_$v.txt
done
