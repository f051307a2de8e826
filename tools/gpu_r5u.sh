#!/bin/bash
# round 5 (u): bench.py's transport fallback chain (tp-rccl -> tp-ipc -> replicas, every rank agreeing,
# decode failures included) on ONE GPU: two ranks sharing it (YALM_BENCH_NDEV=1), where RCCL cannot
# come up, so the line must come from the IPC transport; then the one-GPU driver command
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r5u
mkdir -p $o
YALM_BENCH_NDEV=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 \
  bench.py --gpus 2 --steps 20 --warmup 5 > $o/bench_tp2_default.json 2> $o/bench_tp2_default.err || { echo "tp2 default failed"; tail -20 $o/bench_tp2_default.err; exit 1; }
python3 -c "import json; d=json.loads(open('$o/bench_tp2_default.json').read().strip().splitlines()[-1]); print('tp2 default', d['value'], d['config']['parallelism'], d.get('fallback'), d.get('tp'))"
YALM_BENCH_NDEV=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29614 \
  bench.py --gpus 2 --steps 20 --warmup 5 --replicas > $o/bench_rep2.json 2> $o/bench_rep2.err || { echo "replicas failed"; tail -20 $o/bench_rep2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$o/bench_rep2.json').read().strip().splitlines()[-1]); print('replicas', d['value'], d['config']['parallelism'], d.get('fallback'))"
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $o/bench_20.json 2> $o/bench_20.err || { echo "bench 20 failed"; tail -20 $o/bench_20.err; exit 1; }
python3 -c "import json; d=json.load(open('$o/bench_20.json')); print('one GPU', 'fp16', d['value'], d['step_roofline']['frac'], 'fp8', d['fp8']['value'], 'long', d['long_context']['value'], 'prefill', d['prefill']['value'], d.get('fallback'))"
echo done
