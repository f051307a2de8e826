#!/bin/bash
# round 4 (a): reference-kernel parity on the GPU + long-context decode measurement and profile
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r4a
o=gpurun_out/r4a
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ref_infer.py > $o/tests.log 2>&1 || { echo "tests failed"; tail -30 $o/tests.log; exit 1; }
tail -3 $o/tests.log
timeout -k 10 300 python bench.py --long-only --long-steps 64 > $o/long.json 2> $o/long.err || { echo "long failed"; tail -20 $o/long.err; exit 1; }
cat $o/long.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
YALM_EAGER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o long -- \
  python3 bench.py --long-only --long-steps 32 --kernel-iters 16 > $o/trace.log 2>&1 || { echo "trace failed"; tail -20 $o/trace.log; exit 1; }
python tools/kstats.py $o/trace 20
YALM_EAGER=1 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/pmc -o pmc -- \
  python3 bench.py --long-only --long-steps 8 --kernel-iters 4 > $o/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $o/pmc.log; exit 1; }
echo done
