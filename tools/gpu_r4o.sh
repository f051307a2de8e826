#!/bin/bash
# round 4 (o): the whole GPU test suite
cd "${GRAFT_REPO_ROOT:-/root/repo}"
o=gpurun_out/r4o
mkdir -p $o
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $o/tests.log | head -20; tail -30 $o/tests.log; exit 1; }
tail -3 $o/tests.log
grep -E "layers,|positions:" $o/tests.log | head -5
