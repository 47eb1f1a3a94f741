#!/bin/bash
# Small-batch greedy decode (tools/bench_decode.py on BATCH-row batches of the bench query): per-step
# time of the four-launch loop vs the persistent tail decode.
#   bash tools/dec_small.sh ROWS ...     (ROWS = RNNT_DEC_PERSIST_ROWS; 0 = the four-launch loop)
# The environment knob is read by development builds only: tools/build_variants.sh dev first.
set -o pipefail
OUT=${OUT:-gpurun_out/dec_small}; BATCH=${BATCH:-64}
mkdir -p $OUT
for v in "$@"; do
  tag=b${BATCH}_p$v
  RNNT_MI355X_LIB=${RNNT_MI355X_LIB:-build_dev/lib_dev.so} RNNT_BENCH_BATCH=$BATCH RNNT_DEC_PERSIST_ROWS=$v timeout -k 10 300 python3 -u tools/bench_decode.py \
    > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag rc=$?"; tail -20 $OUT/$tag.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/$tag.json'))
b=[v for k,v in d.items() if k.startswith('batch')]
ms=sum(x['decode_ms'] for x in b); st=sum(x['steps'] for x in b)
print('$tag', 'ms', round(ms,2), 'steps', st, 'us/step', round(1e3*ms/st,2))"
done
