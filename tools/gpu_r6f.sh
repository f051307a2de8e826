#!/bin/bash
# round 6: the whole GPU suite + smoke on the round-6 tree
o=gpurun_out/r6f; mkdir -p $o
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -q -s --timeout 900 --timeout-method thread > $o/tests.log 2>&1
rc=$?
tail -5 $o/tests.log
[ $rc -eq 0 ] || { echo "suite failed rc=$rc"; grep -E "FAILED|Error" $o/tests.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $o/smoke.log; exit 1; }
tail -3 $o/smoke.log
