#!/bin/bash
# A/B of decode variants (development): full GPU parity of the in-tree build, then the isolated
# greedy decode per library variant (tools/bench_decode.py), then the bench line.
set -e
OUT=${OUT:-gpurun_out/abdec}
mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
  tail -2 $OUT/parity.log
fi
for v in ${VARIANTS:-old default pref}; do
  if [ $v = default ]; then L=""; else L=build_dev/lib_$v.so; fi
  RNNT_MI355X_LIB=$L timeout -k 10 200 python tools/bench_decode.py > $OUT/d_$v.json 2> $OUT/d_$v.err || { tail -5 $OUT/d_$v.err; exit 1; }
  echo "$v $(cat $OUT/d_$v.json)"
done
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 600 python bench.py --steps ${STEPS:-3} --warmup 1 ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['encode_ms_per_query'], r['greedy_ms_per_query'], r['decode'], r['isolated'], d['parity_spot_check'])"
fi
