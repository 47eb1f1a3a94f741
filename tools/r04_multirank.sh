#!/bin/bash
# Multi-rank rehearsal of bench.py's data path on a 1-GPU box (the 8-GPU run is the driver's):
# ranks launched by bench.py itself (torch.distributed.run child, before anything touches HIP),
# every rank on cuda:0 with real engines, gloo control plane (--share-device), dynamic batch
# claims and the tagged response stream; then the same total query on one rank, and the gathered
# responses compared row by row.  Each step has its own time limit; the chain stops at the first
# failure.
OUT=${OUT:-gpurun_out/r04mr}
mkdir -p $OUT
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 420 python -u bench.py "$@" --dump-responses $OUT/$name.npz > $OUT/$name.json 2> $OUT/$name.err \
    || { echo "$name rc=$?"; tail -30 $OUT/$name.err; exit 1; }
  cat $OUT/$name.json
}
run dyn2 --gpus 2 --share-device --steps 2 --warmup 1 --query 6144
run static3 --gpus 3 --share-device --deal static --steps 2 --warmup 1 --query 4096
run one --gpus 1 --steps 2 --warmup 1 --query 12288 --no-cpu-baseline
python tools/compare_responses.py $OUT/dyn2.npz $OUT/one.npz > $OUT/compare_dyn2.json; cat $OUT/compare_dyn2.json
python tools/compare_responses.py $OUT/static3.npz $OUT/one.npz > $OUT/compare_static3.json; cat $OUT/compare_static3.json
