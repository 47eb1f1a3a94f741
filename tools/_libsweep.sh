#!/bin/bash
# bench lines per library variant (development), alternating, two rounds.
set -e
OUT=${OUT:-gpurun_out/libsweep}
mkdir -p $OUT
for r in 1 2; do
  for v in ${VARIANTS:-default}; do
    if [ $v = default ]; then L=""; else L=build_dev/lib_$v.so; fi
    RNNT_MI355X_LIB=$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/b.json')); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], r['frac'], r['encode_ms_per_query'], r['greedy_ms_per_query'], r['isolated']['greedy_ms_per_query'])"
  done
done
