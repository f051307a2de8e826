set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_attn_wo.py tests/test_gpu_decode.py > gpurun_out/t_attn.log 2>&1 || { tail -30 gpurun_out/t_attn.log; exit 1; }
tail -3 gpurun_out/t_attn.log
bash tools/trace_awo_all.sh > gpurun_out/trace_awo.log 2>&1
bash tools/ab_lib.sh yalm_amd/ab/libyalm_hip_3d5d87f.so yalm_amd/libyalm_hip.so > gpurun_out/ab_lib.log 2>&1
