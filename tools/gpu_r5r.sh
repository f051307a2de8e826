#!/bin/bash
# round 5 (r): the multi-rank bench flow on ONE GPU (two ranks sharing it, YALM_BENCH_NDEV=1):
# RCCL cannot put two ranks on one device, so the default line falls back to replicas; the IPC
# transport runs as the main line
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r5r
mkdir -p $o
export YALM_BENCH_NDEV=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus 2 --steps 20 --warmup 5 > $o/bench_tp2_default.json 2> $o/bench_tp2_default.err || { echo "default failed"; tail -20 $o/bench_tp2_default.err; exit 1; }
cat $o/bench_tp2_default.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('default', d['value'], d['config'], d.get('fallback'), d.get('tp_ipc'))"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 \
  bench.py --gpus 2 --steps 20 --warmup 5 --tp-transport ipc > $o/bench_tp2_ipc.json 2> $o/bench_tp2_ipc.err || { echo "ipc failed"; tail -20 $o/bench_tp2_ipc.err; exit 1; }
cat $o/bench_tp2_ipc.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('ipc', d['value'], d['config'], d.get('fallback'), d.get('tp'))"
echo done
