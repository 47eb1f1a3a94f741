#!/bin/bash
# decode microbench for the in-tree library and build_dev variants (args)
set -e
mkdir -p gpurun_out/dec
timeout -k 10 200 python tools/bench_decode.py > gpurun_out/dec/intree.json 2> gpurun_out/dec/intree.err || { tail -5 gpurun_out/dec/intree.err; exit 1; }
cat gpurun_out/dec/intree.json
for v in "$@"; do
  RNNT_MI355X_LIB=build_dev/lib_$v.so timeout -k 10 200 python tools/bench_decode.py > gpurun_out/dec/$v.json 2> gpurun_out/dec/$v.err || { tail -5 gpurun_out/dec/$v.err; exit 1; }
  cat gpurun_out/dec/$v.json
done
