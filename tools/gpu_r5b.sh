#!/bin/bash
# round 5 (b): the glue pinned on the reference's own functions (tests/test_gpu_ref_glue.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r5b
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_ref_glue.py -x -v -s --timeout 120 --timeout-method thread > $o/glue.log 2>&1 || { echo "glue tests failed"; grep -E "FAILED|Error|max " $o/glue.log | head -40; exit 1; }
grep -E "max .* f16 ulp" $o/glue.log
tail -1 $o/glue.log
