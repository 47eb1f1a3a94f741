#!/bin/bash
# Offline regression attribution (same box, alternating): round 3's tree and the current tree,
# each with its own library and with the other's (native vs Python side of the difference).
set -e
OUT=${OUT:-gpurun_out/r04offreg2}
mkdir -p $OUT
R=$GRAFT_REPO_ROOT
CUR=$R/rnnt-inference_amd/rnnt_amd/librnnt_mi355x.so
OLD=$R/build_dev/r03tree/rnnt-inference_amd/rnnt_amd/librnnt_mi355x.so
summ='import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d["roofline"]; print(sys.argv[2], d["value"], d["ms_per_step"], r.get("encode_ms_per_query"), r.get("greedy_ms_per_query"), r["isolated"]["greedy_ms_per_query"])'
for r in 1 2; do
  (cd build_dev/r03tree && RNNT_MI355X_LIB=$OLD timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline) > $OUT/r03py_r03lib_$r.json 2> $OUT/r03py_r03lib_$r.err
  python3 -c "$summ" $OUT/r03py_r03lib_$r.json r03py_r03lib
  (cd build_dev/r03tree && RNNT_MI355X_LIB=$CUR timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline) > $OUT/r03py_curlib_$r.json 2> $OUT/r03py_curlib_$r.err
  python3 -c "$summ" $OUT/r03py_curlib_$r.json r03py_curlib
  RNNT_MI355X_LIB=$OLD timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/curpy_r03lib_$r.json 2> $OUT/curpy_r03lib_$r.err
  python3 -c "$summ" $OUT/curpy_r03lib_$r.json curpy_r03lib
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/curpy_curlib_$r.json 2> $OUT/curpy_curlib_$r.err
  python3 -c "$summ" $OUT/curpy_curlib_$r.json curpy_curlib
done
