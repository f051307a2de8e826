#!/bin/bash
# prefill GEMM A/B: auto tile widths with the 2-phase vs 8-phase 256 x 256 kernel, and
# every GEMM forced to 256 x 256 in both schedules (tools/ab_prefill.py, one process)
ALL='YALM_PF_G16=qkv:256,wo:256,w2:256,glu:256,cls:256'
python tools/ab_prefill.py --rounds "${ROUNDS:-4}" "$@" \
  "2ph=YALM_PF_8P=0" "8ph=YALM_PF_8P=1" "all256_2ph=$ALL;YALM_PF_8P=0" "all256_8ph=$ALL;YALM_PF_8P=1"
