#!/bin/bash
# Offline schedule sweep with held decodes (development): ARGS lines in $CFGFILE.
set -e
OUT=${OUT:-gpurun_out/sched3}
mkdir -p $OUT
while read -r cfg; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline $cfg > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b.json')); r=d['roofline']; print('[$cfg]', d['value'], d['ms_per_step'], r['frac'], r['encode_ms_per_query'], r['greedy_ms_per_query'])"
done < ${CFGFILE:-tools/_sched3_cfgs.txt}
