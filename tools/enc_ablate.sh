#!/bin/bash
# Encoder epilogue LDS attribution: the K2048 layer-step on the 256^2 tile,
# baseline vs ablations (σ-table reads replaced by VALU, LDS image stores removed), each with the
# LDS PMC pass and the timing pass.  Build the variants on the CPU first:
#   tools/build_variants.sh base notab:-DRNNT_ABL_NOTAB noimg:-DRNNT_ABL_NOIMG both:"-DRNNT_ABL_NOTAB -DRNNT_ABL_NOIMG" \
#     noc:-DRNNT_ABL_NOC   (cell state not read / written: what on-chip state could save at most)
set -e
OUT=${1:-gpurun_out/ablate}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CMD="python3 tools/bench_kernels.py --n 8192 --layers 1 --T 8 --reps 3 --skip-decode"
for v in base notab noimg both noc; do
  export RNNT_MI355X_LIB=build_dev/lib_$v.so
  timeout -k 10 300 $CMD > $OUT/time_$v.json 2> $OUT/time_$v.err
  timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES \
    --kernel-trace --output-format csv -d $OUT/pmc_$v -o pmc -- $CMD > $OUT/pmc_$v.log 2>&1
done
python3 tools/summarize_ablate.py $OUT > $OUT/summary.json
cat $OUT/summary.json
