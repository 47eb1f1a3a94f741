#!/bin/bash
# Decode tail host loop A/B (isolated decode of the bench query, tools/bench_decode.py, same box,
# alternating): tail chunk size (RNNT_DEC_TAIL_CHUNK) and spin polling (RNNT_DEC_SPIN), plus one
# kernel trace of the default for the per-step gaps (tools/dec_gaps.py).
set -e
OUT=${OUT:-gpurun_out/r04dectail}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export RNNT_MI355X_LIB=build_dev/lib_main.so
for r in 1 2; do
  for v in 8:0 8:1 4:0 4:1 16:0 32:1; do
    c=${v%%:*}; s=${v#*:}
    RNNT_DEC_TAIL_CHUNK=$c RNNT_DEC_SPIN=$s timeout -k 10 240 python3 -u tools/bench_decode.py > $OUT/dec_${c}_${s}_$r.json 2> $OUT/dec_${c}_${s}_$r.err
    python3 -c "import json; d=json.load(open('$OUT/dec_${c}_${s}_$r.json')); print('tail_chunk $c spin $s', round(sum(v['decode_ms'] for k, v in d.items() if k.startswith('batch')), 2))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace -o tr -- python3 tools/bench_decode.py > $OUT/trace.log 2>&1
python3 tools/dec_gaps.py $OUT/trace > $OUT/gaps.json
cat $OUT/gaps.json | head -60
find $OUT/trace -name "*.csv" -delete
