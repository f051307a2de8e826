set -o pipefail
timeout -k 10 120 tools/pattern_bench > gpurun_out/pattern.log 2>&1
bash tools/ab_env.sh fp16 "YALM_AWO_SPEC=0" "YALM_AWO_SPEC=1" "YALM_ATTN_WO_DELAY=0" "YALM_ATTN_WO_DELAY=50" > gpurun_out/ab_env_fp16.log 2>&1
bash tools/ab_env.sh fp8 "YALM_AWO_SPEC=0" "YALM_AWO_SPEC=1" "YALM_ATTN_WO_DELAY=0" "YALM_ATTN_WO_DELAY=50" > gpurun_out/ab_env_fp8.log 2>&1
