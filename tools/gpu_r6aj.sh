#!/bin/bash
# round 6 (aj): the driver's bench command on the committed tree -- roofline.traffic must come from the
# newest FETCH_SIZE csv (profiles/r6ah_*), which now travels with the snapshot
o=gpurun_out/r6aj; mkdir -p $o
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $o/bench_20.json 2> $o/bench_20.err || { echo "bench failed"; tail -20 $o/bench_20.err; exit 1; }
python3 -c "import json; d=json.loads(open('$o/bench_20.json').readline()); r=d['roofline']; print(d['value'], d['step_roofline']['frac'], r['frac'], r['traffic'], r.get('traffic_source'), d['long_context']['value'], d['fp8']['value'], d['prefill']['value'])"
