#!/bin/bash
# A/B of encoder kernel variants (development): parity of the default build, then per-variant
# layer-step timings and the stamps timeline.
set -e
OUT=${OUT:-gpurun_out/ab}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
for v in ${VARIANTS:-base split asm both}; do
  RNNT_MI355X_LIB=build_dev/lib_$v.so timeout -k 10 200 python tools/bench_kernels.py --n 8192 --T 8 --layers 1,2,0 --skip-decode --reps 5 > $OUT/k_$v.json 2> $OUT/k_$v.err || { tail -5 $OUT/k_$v.err; exit 1; }
  echo "$v $(cat $OUT/k_$v.json)"
done
if [ -n "$STAMPS" ]; then
  RNNT_MI355X_LIB=build_dev/lib_stamps.so timeout -k 10 200 python tools/enc_stamps.py --n 8192 --first 1 --T 4 > $OUT/stamps.json 2>&1 || { tail -5 $OUT/stamps.json; exit 1; }
  cat $OUT/stamps.json
fi
