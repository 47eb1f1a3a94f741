#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/tr
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/ov -o t -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/ov.log 2>&1
python3 tools/trace_decode.py $OUT/ov overlapped > $OUT/ov.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/one -o t -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --inflight 1 > $OUT/one.log 2>&1
python3 tools/trace_decode.py $OUT/one inflight1 > $OUT/one.json
find $OUT -name "*.csv" -delete
cat $OUT/ov.json $OUT/one.json
