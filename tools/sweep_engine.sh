#!/bin/bash
# Engine loader sweep (GPU): one engine_trace.py run per (YALM_ENGINE_DBG,
# YALM_ENGINE_DEPTH, YALM_ENGINE_LOADERS, YALM_ENGINE_SLEEP, YALM_ENGINE_PF);
# prints the kernel span line of each.
# dbg=4: the consumers skip the ring, so the span is the loaders' pure stream time.
# usage: bash tools/sweep_engine.sh ["dbg depth loaders [sleep [pf_kb]]" ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cfgs=("$@")
[ ${#cfgs[@]} -eq 0 ] && cfgs=("0 1 4" "0 2 4" "0 1 3 1 128" "0 2 3 1 128" "0 2 3 1 256" "0 2 3 1 512")
for cfg in "${cfgs[@]}"; do
  set -- $cfg
  echo "=== dbg=$1 depth=$2 loaders=$3 sleep=${4:-1} pf=${5:-0}"
  YALM_ENGINE_DBG=$1 YALM_ENGINE_DEPTH=$2 YALM_ENGINE_LOADERS=$3 YALM_ENGINE_SLEEP=${4:-1} YALM_ENGINE_PF=${5:-0} \
    timeout -k 10 120 python -u tools/engine_trace.py > gpurun_out/sweep_engine.log 2>&1 || exit 1
  sed -n 1p gpurun_out/sweep_engine.log | sed 's/.*kernel span/span/'
done
