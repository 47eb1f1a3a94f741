#!/bin/bash
# Server capacity A/B (tools/server_bench.py --burst): fcfs refill vs tile refill with the tick
# kernel's tile mask vs tile refill with prefix skipping, alternating, same box.
set -e
OUT=${OUT:-gpurun_out/r04srvcap}
mkdir -p $OUT
for r in 1 2; do
  for v in fcfs:0 tile:0 tile:1; do
    pol=${v%%:*}; pre=${v#*:}
    RNNT_STREAM_PREFIX=$pre timeout -k 10 300 python3 -u tools/server_bench.py --burst ${N:-60000} --refill $pol \
      > $OUT/cap_${pol}_${pre}_$r.json 2> $OUT/cap_${pol}_${pre}_$r.err
    tail -1 $OUT/cap_${pol}_${pre}_$r.json
  done
done
