#!/bin/bash
# Engine loader sweep (GPU): one engine_trace.py run per (YALM_ENGINE_DBG,
# YALM_ENGINE_DEPTH, YALM_ENGINE_LOADERS); prints the kernel span line of each.
# dbg=4: the consumers skip the ring, so the span is the loaders' pure stream time.
# usage: bash tools/sweep_engine.sh ["dbg depth loaders" ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cfgs=("$@")
[ ${#cfgs[@]} -eq 0 ] && cfgs=("4 1 4" "4 2 4" "4 1 2" "4 2 2" "4 3 2" "4 2 1" "4 4 1" "0 1 4" "0 2 2" "0 3 2"
                               "0 1 2" "0 3 1" "0 4 1" "0 6 1" "0 2 3" "0 1 3")
for cfg in "${cfgs[@]}"; do
  set -- $cfg
  echo "=== dbg=$1 depth=$2 loaders=$3"
  YALM_ENGINE_DBG=$1 YALM_ENGINE_DEPTH=$2 YALM_ENGINE_LOADERS=$3 timeout -k 10 120 \
    python -u tools/engine_trace.py > gpurun_out/sweep_engine.log 2>&1 || exit 1
  sed -n 1p gpurun_out/sweep_engine.log | cut -c1-120
done
