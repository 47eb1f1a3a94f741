#!/bin/bash
# Offline: SUT warmup variants vs none (same box, alternating): dummy samples of 500 / 64 frames.
set -e
OUT=${OUT:-gpurun_out/r04offreg4}
mkdir -p $OUT
summ='import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d["roofline"]; print(sys.argv[2], d["value"], d["ms_per_step"], r.get("encode_ms_per_query"), r.get("greedy_ms_per_query"))'
for r in 1 2 3; do
  for v in 0:500 1:500 1:64; do
    w=${v%%:*}; f=${v#*:}
    timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --sut-warmup $w --sut-warmup-frames $f > $OUT/w${w}_f${f}_$r.json 2> $OUT/w${w}_f${f}_$r.err
    python3 -c "$summ" $OUT/w${w}_f${f}_$r.json w${w}_f${f}
  done
done
