#!/bin/bash
# Server tile refill: GPU parity of the stream path with batch-tile masks (incl. holes), then a
# same-box A/B at saturating targets: fcfs refill, tile refill with the tick kernel skipping any
# done tile (mask), tile refill with only trailing done tiles skipped (RNNT_STREAM_PREFIX=1).
set -e
OUT=${OUT:-gpurun_out/r04srv}
mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_server_gpu.py tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
for q in ${QPS:-80000 95000}; do
  for r in 1 2; do
    for v in fcfs:0 tile:0 tile:1; do
      pol=${v%%:*}; pre=${v#*:}
      RNNT_STREAM_PREFIX=$pre timeout -k 10 300 python3 -u tools/server_bench.py --qps $q --duration ${DUR:-8} --refill $pol \
        > $OUT/srv_${q}_${pol}_${pre}_$r.json 2> $OUT/srv_${q}_${pol}_${pre}_$r.err
      python3 -c "
import json; d=json.loads(open('$OUT/srv_${q}_${pol}_${pre}_$r.json').read().strip().splitlines()[-1]); p=d['points'][-1]
print('$q $pol prefix=$pre', {k: p.get(k) for k in ('achieved_qps', 'p50_ms', 'p99_ms', 'valid', 'rounds')})"
    done
  done
done
