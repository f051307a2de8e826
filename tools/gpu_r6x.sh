#!/bin/bash
# round 6 (x): the whole GPU suite twice more (the TP8 rehearsal's intermittent miss: does it recur, and which shard)
o=gpurun_out/r6x; mkdir -p $o
for rep in 1 2; do
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 600 --timeout-method thread > $o/tests_$rep.log 2>&1
  echo "rep $rep rc=$?: $(tail -1 $o/tests_$rep.log)"
  grep -E "^FAILED|AssertionError: \[" $o/tests_$rep.log | head -5
done
