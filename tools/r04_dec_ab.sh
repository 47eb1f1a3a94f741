#!/bin/bash
# Decode step-structure A/B (isolated decode of the bench query, tools/bench_decode.py): the
# four-launch reference build (lib_4l) against the main library at several switch points to
# three-launch steps (RNNT_DEC_TAIL3_ROWS), alternating, plus one kernel trace of each extreme
# for per-step times (tools/dec_steps_csv.py).
set -e
OUT=${OUT:-gpurun_out/r04dec}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for v in 4l:0 main:0 main:32 main:128 main:512 main:100000; do
    lib=${v%%:*}; t=${v#*:}
    RNNT_DEC_TAIL3_ROWS=$t RNNT_MI355X_LIB=build_dev/lib_$lib.so timeout -k 10 240 python3 -u tools/bench_decode.py > $OUT/dec_${lib}_${t}_$r.json 2> $OUT/dec_${lib}_${t}_$r.err
    python3 -c "import json; d=json.load(open('$OUT/dec_${lib}_${t}_$r.json')); print('$lib $t', round(sum(v['decode_ms'] for k, v in d.items() if k.startswith('batch')), 2))"
  done
done
for t in 0 100000; do
  RNNT_DEC_TAIL3_ROWS=$t RNNT_MI355X_LIB=build_dev/lib_main.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$t -o tr -- python3 tools/bench_decode.py > $OUT/trace_$t.log 2>&1
  python3 tools/dec_steps_csv.py $(find $OUT/trace_$t -name "*kernel_trace.csv") > $OUT/steps_$t.json
  find $OUT/trace_$t -name "*kernel_trace.csv" -delete
done
