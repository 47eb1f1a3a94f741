#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/trd
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/t -o t -- python3 tools/bench_decode.py > $OUT/log 2>&1
python3 tools/trace_steps.py $OUT/t > $OUT/steps.txt
find $OUT -name "*.csv" -delete
cat $OUT/steps.txt
