#!/bin/bash
# Decoder built without packed FP32 (-fno-slp-vectorize on decoder.hip / decoder_ops.hip) as a
# precaution: Offline bench alternating with the shipped build on one box, then the
# decode parity tests on the variant.
OUT=${OUT:-gpurun_out/r04ds}
mkdir -p $OUT
for i in 1 2; do
  for v in cur decnslp; do
    RNNT_MI355X_LIB=build_dev/lib_$v.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline \
      > $OUT/b_${v}_$i.json 2> $OUT/b_${v}_$i.err || { echo "$v rc=$?"; tail -20 $OUT/b_${v}_$i.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], r['isolated']['greedy_ms_per_query'], r['decode']['frac'])" $OUT/b_${v}_$i.json $v
  done
done
RNNT_MI355X_LIB=build_dev/lib_decnslp.so timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_f32_decode_gpu.py tests/test_torch_ops_gpu.py -x -q \
  --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
