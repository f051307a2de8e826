#!/bin/bash
# prefill A/B: persistent 8-phase GEMM (one workgroup per CU walking the tiles) vs one workgroup per tile
python tools/ab_prefill.py --rounds "${ROUNDS:-5}" "$@" "persist=YALM_PF_PERSIST=1" "per_tile=YALM_PF_PERSIST=0"
