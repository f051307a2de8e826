#!/bin/bash
# prefill kernel profile (rocprofv3 kernel stats of tools/bench_prefill.py) + top kernels
tools/prof_prefill.sh "def|YALM_PF_8P=1" && python3 tools/kstats.py gpurun_out/pfprof_def 12
