#!/bin/bash
# A/B of encoder builds (development): tile parity of the in-tree build, then per-library K-width
# layer-step timings (N=8192, the 256x256 tile) and, optionally, the bench line.
set -e
OUT=${OUT:-gpurun_out/abenc}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
for rep in 1 2; do
for v in ${VARIANTS:-old default}; do
  if [ $v = default ]; then L=""; else L=build_dev/lib_$v.so; fi
  RNNT_MI355X_LIB=$L RNNT_ENC_TILE=${TILE:-big} timeout -k 10 200 python tools/bench_kernels.py --n ${KN:-8192} --T 8 --layers 1,2,0 --skip-decode --reps 5 > $OUT/k_$v.json 2> $OUT/k_$v.err || { tail -5 $OUT/k_$v.err; exit 1; }
  echo "$v $(cat $OUT/k_$v.json)"
done
done
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 600 python bench.py --steps ${STEPS:-3} --warmup 1 ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['encode_ms_per_query'], r['isolated'])"
fi
