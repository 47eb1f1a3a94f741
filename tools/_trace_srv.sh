#!/bin/bash
# per-round timeline of a short Server run (kernel trace)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/tsrv
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/t -o t -- python3 tools/server_bench.py --qps ${QPS:-80000} --duration ${DUR:-2} > $OUT/log 2>&1
python3 tools/trace_query.py $OUT/t > $OUT/timeline.txt
find $OUT -name "*.csv" -delete
tail -40 $OUT/timeline.txt
