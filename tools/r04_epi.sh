#!/bin/bash
# Encoder epilogue schedule A/B (development variants, tools/build_variants.sh base nv:-DRNNT_EPI_NV
# ph:-DRNNT_EPI_PHASED): the K2048 layer-step at N = 8192 on the 256^2 tile, alternating on one
# box, then the encoder parity tests on each variant.
OUT=${OUT:-gpurun_out/r04epi}
mkdir -p $OUT
CMD="python3 tools/bench_kernels.py --n 8192 --layers 1 --T 8 --reps 3 --skip-decode"
for i in 1 2; do
  for v in base nv ph; do
    RNNT_MI355X_LIB=build_dev/lib_$v.so timeout -k 10 300 $CMD > $OUT/time_${v}_$i.json 2> $OUT/time_${v}_$i.err \
      || { echo "$v $i rc=$?"; tail -20 $OUT/time_${v}_$i.err; exit 1; }
    echo "$v $i $(tail -c 400 $OUT/time_${v}_$i.json)"
  done
done
for v in ph nv; do
  RNNT_MI355X_LIB=build_dev/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 \
    --timeout-method thread > $OUT/parity_$v.log 2>&1 || { echo "parity $v rc=$?"; tail -30 $OUT/parity_$v.log; exit 1; }
  echo "parity $v: $(tail -1 $OUT/parity_$v.log)"
done
