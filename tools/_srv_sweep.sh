#!/bin/bash
# Server configuration sweep at fixed target QPS (development): one config per line in $CFGFILE.
set -e
OUT=${OUT:-gpurun_out/srvs}
mkdir -p $OUT
i=0
while read -r cfg; do
  i=$((i+1))
  for q in ${QPS:-70000 80000}; do
    timeout -k 10 200 python tools/server_bench.py --qps $q --duration 8 $cfg > $OUT/p$i.json 2> $OUT/p$i.err || { tail -5 $OUT/p$i.err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/p$i.json').read().strip().splitlines()[-1]); p=d['points'][0]; print('[$cfg]', $q, p['achieved_qps'], p['p50_ms'], p['p99_ms'], p['valid'])"
  done
done < ${CFGFILE:-tools/_srv_cfgs.txt}
