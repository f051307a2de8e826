#!/bin/bash
# prefill A/B: QKV as one 2-phase 320-wide launch vs q (8-phase 192) + k | v (8-phase 128) launches
python tools/ab_prefill.py --rounds "${ROUNDS:-5}" "$@" \
  "one=YALM_PF_QKV_SPLIT=0" "split=YALM_PF_QKV_SPLIT=1" "split_kv2ph=YALM_PF_QKV_SPLIT=1;YALM_PF_8P=1"
