#!/bin/bash
# One GPU iteration: parity tests, kernel microbenchmarks, the bench line.  Each step has its
# own time limit and the chain stops at the first failure.
set -e
OUT=${OUT:-gpurun_out/check}
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python tools/bench_kernels.py --n ${KN:-2560} --T 16 --layers 0,1,2 > $OUT/kernels.json 2> $OUT/kernels.err
cat $OUT/kernels.json
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 600 python bench.py --steps 3 --warmup 1 ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err
  cat $OUT/bench.json
fi
