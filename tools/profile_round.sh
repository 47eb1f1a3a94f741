#!/bin/bash
# Round profile: kernel-trace stats of the default bench workload + separate PMC passes
# (kernel-trace only; FETCH_SIZE and WRITE_SIZE in their own passes, MI355X_MICROARCH.md HBM
# section).  Outputs under $OUT (gpurun_out/...); tools/summarize_profile.py condenses them.
set -e
OUT=${1:-gpurun_out/prof_round}
STEPS=${STEPS:-1}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
BENCH="python3 bench.py --steps $STEPS --warmup 1 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- $BENCH > $OUT/trace.log 2>&1
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/pmc$i -o pmc -- $BENCH > $OUT/pmc$i.log 2>&1
done
# condense on the box (the raw per-dispatch CSVs are far larger than what gpurun copies back)
PREFIX=${PREFIX:-$OUT/summary/r}
python3 tools/summarize_profile.py $OUT $PREFIX
find $OUT -name "*_kernel_trace.csv" -delete
find $OUT -name "*_counter_collection.csv" -size +8M -delete
