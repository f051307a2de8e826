#!/bin/bash
# prefill tile-width A/B with the 8-phase 256 x 256 kernel (tools/ab_prefill.py, one process)
python tools/ab_prefill.py --rounds "${ROUNDS:-5}" "$@" \
  "auto=" "2ph=YALM_PF_8P=0" "wow2_256=YALM_PF_G16=wo:256,w2:256" "all256=YALM_PF_G16=qkv:256,wo:256,w2:256" \
  "qkv256=YALM_PF_G16=qkv:256"
