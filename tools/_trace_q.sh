#!/bin/bash
# per-batch timeline of one bench query (kernel trace)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/tq
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/t -o t -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline "$@" > $OUT/log 2>&1
python3 tools/trace_query.py $OUT/t > $OUT/timeline.txt
find $OUT -name "*.csv" -delete
cat $OUT/timeline.txt
