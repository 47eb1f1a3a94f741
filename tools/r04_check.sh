#!/bin/bash
# Round-4 GPU pass: smoke (one decode through the step kernels) first, then the GPU suite, then
# the bench line.  Each step has its own time limit; the chain stops at the first failure.
OUT=${OUT:-gpurun_out/r04}
mkdir -p $OUT
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 600 python -u bench.py --steps ${STEPS:-5} --warmup 2 ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -30 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
