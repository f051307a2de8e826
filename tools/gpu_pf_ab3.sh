#!/bin/bash
# prefill A/B: auto (8-phase 192 for Wo / W2) vs Wo / W2 at 8-phase 256 vs all 2-phase
python tools/ab_prefill.py --rounds "${ROUNDS:-5}" "$@" \
  "auto=" "wow2_256=YALM_PF_G16=wo:256,w2:256" "2ph=YALM_PF_8P=0"
