#!/bin/bash
# A/B of library variants on BASELINE configs 2/3 (development), after the tile parity tests.
set -e
OUT=${OUT:-gpurun_out/abcfg}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
for v in ${VARIANTS:-old default old default}; do
  if [ $v = default ]; then L=""; else L=build_dev/lib_$v.so; fi
  RNNT_MI355X_LIB=$L timeout -k 10 300 python tools/bench_configs.py --concurrent ${CONC:-0} > $OUT/c.json 2> $OUT/c.err || { tail -5 $OUT/c.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/c.json').read().strip().splitlines()[-1]); c=d['config3_int8_full_n128']; print('$v', c['utt_per_s'], c['encode_ms'], c['greedy_ms'], c['encoder_int8_frac'], d.get('config3_int8_full_n128_concurrent', {}).get('utt_per_s'))"
done
