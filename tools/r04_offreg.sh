#!/bin/bash
# Offline regression check (same box, alternating): round 3's tree (bench.py + Python + library,
# build_dev/r03tree) vs the current tree, the default bench line without the CPU baseline.
set -e
OUT=${OUT:-gpurun_out/r04offreg}
mkdir -p $OUT
summ='import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d["roofline"]; print(sys.argv[2], d["value"], d["ms_per_step"], r.get("encode_ms_per_query"), r.get("greedy_ms_per_query"), r["frac"])'
for r in 1 2 3; do
  (cd build_dev/r03tree && timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline) > $OUT/r03_$r.json 2> $OUT/r03_$r.err
  python3 -c "$summ" $OUT/r03_$r.json r03
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/cur_$r.json 2> $OUT/cur_$r.err
  python3 -c "$summ" $OUT/cur_$r.json cur
done
