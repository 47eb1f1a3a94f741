#!/bin/bash
# encoder step microbench for the in-tree library and build_dev variants (args)
set -e
mkdir -p gpurun_out/kern
timeout -k 10 200 python tools/bench_kernels.py --n 8192 --T 8 --layers 0,1,2 --skip-decode > gpurun_out/kern/intree.json 2> gpurun_out/kern/intree.err || { tail -5 gpurun_out/kern/intree.err; exit 1; }
echo "intree $(cat gpurun_out/kern/intree.json)"
for v in "$@"; do
  RNNT_MI355X_LIB=build_dev/lib_$v.so timeout -k 10 200 python tools/bench_kernels.py --n 8192 --T 8 --layers 0,1,2 --skip-decode > gpurun_out/kern/$v.json 2> gpurun_out/kern/$v.err || { tail -5 gpurun_out/kern/$v.err; exit 1; }
  echo "$v $(cat gpurun_out/kern/$v.json)"
done
