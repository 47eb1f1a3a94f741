#!/bin/bash
# Same-box A/B of the end-to-end bench line over library variants (RNNT_MI355X_LIB), alternating:
#   VARIANTS="main base" ROUNDS=2 bash tools/ab_bench.sh gpurun_out/ab
set -e
OUT=${1:-gpurun_out/ab}
mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-main base}; do
    RNNT_MI355X_LIB=build_dev/lib_$v.so timeout -k 10 300 python3 -u bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline \
      > $OUT/bench_${v}_$r.json 2> $OUT/bench_${v}_$r.err
    python3 -c "import json; d=json.load(open('$OUT/bench_${v}_$r.json')); r=d['roofline']; print('$v', d['value'], r['encode_ms_per_query'], r['greedy_ms_per_query'], r['isolated']['greedy_ms_per_query'])"
  done
done
