#!/bin/bash
# Offline: does the SUT warmup (dummy 4096 x 500-frame batches before the first query) change the
# steady-state step?  Same box, alternating, current tree, plus round 3's tree as the control.
set -e
OUT=${OUT:-gpurun_out/r04offreg3}
mkdir -p $OUT
summ='import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d["roofline"]; print(sys.argv[2], d["value"], d["ms_per_step"], r.get("encode_ms_per_query"), r.get("greedy_ms_per_query"))'
for r in 1 2 3; do
  (cd build_dev/r03tree && timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline) > $OUT/r03_$r.json 2> $OUT/r03_$r.err
  python3 -c "$summ" $OUT/r03_$r.json r03
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --sut-warmup 0 > $OUT/w0_$r.json 2> $OUT/w0_$r.err
  python3 -c "$summ" $OUT/w0_$r.json sut_warmup0
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --sut-warmup 1 > $OUT/w1_$r.json 2> $OUT/w1_$r.err
  python3 -c "$summ" $OUT/w1_$r.json sut_warmup1
done
