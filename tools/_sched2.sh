#!/bin/bash
# Offline batch-size / in-flight sweep (development): CFGS="batch_inflight ..."
set -e
OUT=${OUT:-gpurun_out/sched2}
mkdir -p $OUT
for cfg in ${CFGS:-8192_3 12288_2 6144_4}; do
  b=${cfg%_*}; k=${cfg#*_}
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --batch $b --inflight $k > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b.json')); r=d['roofline']; print('$cfg', d['value'], d['ms_per_step'], r['frac'], r['encode_ms_per_query'], r['tick_launches_per_query'], r['greedy_ms_per_query'], r['isolated']['encode_ms_per_query'])"
done
