#!/bin/bash
# Encoder staging: how much of the K2048 layer-step (256^2 tile, N = 8192) is MALL latency?
# Ablations make an operand L2-resident (wrong values, timing only): every gate tile reads tile 0's
# weights (w1), every batch tile reads tile 0's activations (x1), both (wx1).  Alternating runs,
# PMC pass for the EA (L2-miss) bytes.  Build first:
#   tools/build_variants.sh base w1:-DRNNT_ABL_W1 x1:-DRNNT_ABL_X1 wx1:"-DRNNT_ABL_W1 -DRNNT_ABL_X1"
set -e
OUT=${1:-gpurun_out/l2abl}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CMD="python3 tools/bench_kernels.py --n 8192 --layers 1 --T 8 --reps 3 --skip-decode"
for r in 1 2; do
  for v in base w1 x1 wx1; do
    RNNT_MI355X_LIB=build_dev/lib_$v.so timeout -k 10 300 $CMD > $OUT/time_${v}_$r.json 2> $OUT/time_${v}_$r.err
    echo "$v run $r: $(tail -c 400 $OUT/time_${v}_$r.json)"
  done
done
for v in base wx1; do
  RNNT_MI355X_LIB=build_dev/lib_$v.so timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum \
    --kernel-trace --output-format csv -d $OUT/pmc_$v -o pmc -- $CMD > $OUT/pmc_$v.log 2>&1
done
