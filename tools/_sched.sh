#!/bin/bash
# Offline schedule sweep (development): bench lines for batch-size schedules, in-order encodes.
set -e
OUT=${OUT:-gpurun_out/sched}
mkdir -p $OUT
i=0
for bs in ${SCHEDS:-8192 8192,8192,6144,2048}; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --batch-sizes $bs > $OUT/b$i.json 2> $OUT/b$i.err || { tail -20 $OUT/b$i.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b$i.json')); r=d['roofline']; print('$bs', d['value'], d['ms_per_step'], r['frac'], r['encode_ms_per_query'], r['greedy_ms_per_query'], r['isolated']['encode_ms_per_query'])"
done
