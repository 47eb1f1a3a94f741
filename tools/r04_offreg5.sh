#!/bin/bash
# Offline: the SUT warmup with gather-form dummy samples (no dense batch) vs none, same box,
# alternating; the Offline GPU tests (which run the warmup) first.
set -e
OUT=${OUT:-gpurun_out/r04offreg5}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_offline_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
summ='import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d["roofline"]; print(sys.argv[2], d["value"], d["ms_per_step"], r.get("encode_ms_per_query"), r.get("greedy_ms_per_query"))'
for r in 1 2 3; do
  for w in 0 1; do
    timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --sut-warmup $w > $OUT/w${w}_$r.json 2> $OUT/w${w}_$r.err
    python3 -c "$summ" $OUT/w${w}_$r.json sut_warmup$w
  done
done
