set -o pipefail
timeout -k 10 120 tools/pattern_bench > gpurun_out/pattern.log 2>&1
timeout -k 10 120 python tools/kernel_times.py --iters 256 >> gpurun_out/pattern.log 2>&1
timeout -k 10 120 python -c "
import sys; sys.path.insert(0,'.')
from yalm_amd import runtime
runtime.check(runtime.lib.yalm_set_device(0))
print('envelope 235 MB back-to-back:', runtime.stream_envelope(234971136, 50))
" >> gpurun_out/pattern.log 2>&1
