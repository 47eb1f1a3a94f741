#!/bin/bash
# Server regression check (same box): round 3's tree (library + Python) vs the current tree, fcfs
# refill, at one target QPS, alternating.
set -e
OUT=${OUT:-gpurun_out/r04srvreg}
mkdir -p $OUT
Q=${QPS:-70000}
for r in 1 2; do
  timeout -k 10 300 python3 -u build_dev/r03tree/tools/server_bench.py --qps $Q --duration 8 > $OUT/r03_$r.json 2> $OUT/r03_$r.err
  python3 -c "import json; p=json.loads(open('$OUT/r03_$r.json').read().strip().splitlines()[-1])['points'][-1]; print('r03', {k: p.get(k) for k in ('achieved_qps','p50_ms','p99_ms','rounds')})"
  timeout -k 10 300 python3 -u tools/server_bench.py --qps $Q --duration 8 > $OUT/cur_$r.json 2> $OUT/cur_$r.err
  python3 -c "import json; p=json.loads(open('$OUT/cur_$r.json').read().strip().splitlines()[-1])['points'][-1]; print('cur', {k: p.get(k) for k in ('achieved_qps','p50_ms','p99_ms','rounds')})"
  RNNT_MI355X_LIB=build_dev/lib_r03.so timeout -k 10 300 python3 -u tools/server_bench.py --qps $Q --duration 8 > $OUT/curpy_r03lib_$r.json 2> $OUT/curpy_r03lib_$r.err
  python3 -c "import json; p=json.loads(open('$OUT/curpy_r03lib_$r.json').read().strip().splitlines()[-1])['points'][-1]; print('curpy+r03lib', {k: p.get(k) for k in ('achieved_qps','p50_ms','p99_ms','rounds')})"
done
