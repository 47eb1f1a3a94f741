#!/bin/bash
# One parameterised runner for GPU-box passes (gpurun -- 'bash tools/gpu.sh <task> ...').  Every GPU
# step has its own time limit, the chain stops at the first failure, outputs go under $OUT.
#
#   check                  smoke, then the -m gpu suite, then one bench line      (NO_TESTS / NO_BENCH skip)
#   ab  V1 V2 ...          end-to-end bench lines over variants, alternating ROUNDS times
#   decab V1 V2 ...        isolated decode of the bench query (tools/bench_decode.py) over variants
#   kernels                encoder layer-step microbenchmarks (tools/bench_kernels.py)
#   profile                kernel-trace stats of the bench + separate PMC passes (summaries in $OUT/summary)
#   multirank              2 / 3 ranks on one GPU (gloo, --share-device) vs one rank, responses compared
#   timeline               kernel trace of warmup + one timed query: per-batch encode / decode spans (trace_query.py)
#
# A variant is NAME[:VAR=VAL[,VAR=VAL...]]: NAME "main" is the shipped library, any other NAME loads
# build_dev/lib_NAME.so (RNNT_MI355X_LIB); the VAR=VAL pairs are set in that run's environment.
# Knobs: OUT (gpurun_out/<task>), STEPS (5), ROUNDS (2), BENCH_ARGS, PYTEST_ARGS, PREFIX (profile).
set -o pipefail
TASK=${1:?task}; shift
OUT=${OUT:-gpurun_out/$TASK}
STEPS=${STEPS:-5}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1

die() { echo "$1"; [ -n "$2" ] && tail -40 "$2"; exit 1; }

# run_variant NAME[:ENV...] cmd...  (in a subshell, so the variant's environment stays local)
run_variant() {
  local v=$1; shift
  local name=${v%%:*} envs=""
  [ "$v" != "$name" ] && envs=${v#*:}
  (
    [ "$name" != main ] && export RNNT_MI355X_LIB=build_dev/lib_$name.so
    IFS=, read -ra kv <<< "$envs"
    for p in "${kv[@]}"; do [ -n "$p" ] && export "$p"; done
    "$@"
  )
}

case $TASK in
check)
  timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || die "smoke rc=$?" $OUT/smoke.log
  tail -1 $OUT/smoke.log
  if [ -z "$NO_TESTS" ]; then
    timeout -k 10 1100 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread ${PYTEST_ARGS} \
      > $OUT/pytest_gpu.log 2>&1 || die "pytest rc=$?" $OUT/pytest_gpu.log
    tail -3 $OUT/pytest_gpu.log
  fi
  if [ -z "$NO_BENCH" ]; then
    timeout -k 10 600 python -u bench.py --steps $STEPS --warmup 2 ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err \
      || die "bench rc=$?" $OUT/bench.err
    cat $OUT/bench.json
  fi
  ;;
ab)
  for r in $(seq 1 ${ROUNDS:-2}); do
    for v in "$@"; do
      tag=$(echo "$v" | tr ':,=/' '____')
      run_variant "$v" timeout -k 10 300 python3 -u bench.py --steps $STEPS --warmup 2 --no-cpu-baseline ${BENCH_ARGS} \
        > $OUT/bench_${tag}_$r.json 2> $OUT/bench_${tag}_$r.err || die "$v rc=$?" $OUT/bench_${tag}_$r.err
      python3 -c "import json; d=json.load(open('$OUT/bench_${tag}_$r.json')); r=d['roofline']; print('$v', d['value'], r['encode_ms_per_query'], r['greedy_ms_per_query'], r['isolated']['encode_ms_per_query'], r['isolated']['greedy_ms_per_query'])"
    done
  done
  ;;
decab)
  for r in $(seq 1 ${ROUNDS:-2}); do
    for v in "$@"; do
      tag=$(echo "$v" | tr ':,=/' '____')
      run_variant "$v" timeout -k 10 240 python3 -u tools/bench_decode.py ${DEC_ARGS} > $OUT/dec_${tag}_$r.json 2> $OUT/dec_${tag}_$r.err \
        || die "$v rc=$?" $OUT/dec_${tag}_$r.err
      python3 -c "import json; d=json.load(open('$OUT/dec_${tag}_$r.json')); print('$v', round(sum(v['decode_ms'] for k, v in d.items() if k.startswith('batch')), 2))"
    done
  done
  ;;
kernels)
  timeout -k 10 300 python3 -u tools/bench_kernels.py ${KERNEL_ARGS:---n 8192 --T 16 --layers 0,1,2} > $OUT/kernels.json 2> $OUT/kernels.err \
    || die "kernels rc=$?" $OUT/kernels.err
  cat $OUT/kernels.json
  ;;
profile)
  # kernel-trace stats of the default bench workload + separate PMC passes (kernel-trace only;
  # FETCH_SIZE and WRITE_SIZE in their own passes, MI355X_MICROARCH.md HBM section)
  BENCH="python3 bench.py --steps ${PSTEPS:-1} --warmup 1 --no-cpu-baseline ${BENCH_ARGS}"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- $BENCH > $OUT/trace.log 2>&1 \
    || die "trace rc=$?" $OUT/trace.log
  i=0
  for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -k 10 600 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/pmc$i -o pmc -- $BENCH > $OUT/pmc$i.log 2>&1 \
      || die "pmc pass $i rc=$?" $OUT/pmc$i.log
  done
  # condense on the box (the raw per-dispatch CSVs are far larger than what gpurun copies back)
  python3 tools/summarize_profile.py $OUT ${PREFIX:-$OUT/summary/r}
  find $OUT -name "*_kernel_trace.csv" -delete
  find $OUT -name "*_counter_collection.csv" -size +8M -delete
  ;;
timeline)
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o tl -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $OUT/trace.log 2>&1 || die "trace rc=$?" $OUT/trace.log
  python3 tools/trace_query.py $OUT/trace > $OUT/timeline.txt && cat $OUT/timeline.txt
  python3 tools/dec_overlap.py $OUT/trace > $OUT/dec_overlap.json && cat $OUT/dec_overlap.json
  [ -n "$KEEP_TRACE" ] || find $OUT/trace -name "*_kernel_trace.csv" -delete
  ;;
multirank)
  # bench.py's multi-rank data path on a 1-GPU box (the 8-GPU run is the driver's): ranks launched by
  # bench.py itself, every rank on cuda:0 with real engines, gloo control plane, dynamic claims and the
  # tagged response stream; then the same total query on one rank, compared row by row
  mr() {
    local name=$1; shift
    timeout -k 10 420 python -u bench.py "$@" --dump-responses $OUT/$name.npz > $OUT/$name.json 2> $OUT/$name.err \
      || die "$name rc=$?" $OUT/$name.err
    cat $OUT/$name.json
  }
  mr dyn2 --gpus 2 --share-device --steps 2 --warmup 1 --query 6144
  mr static3 --gpus 3 --share-device --deal static --steps 2 --warmup 1 --query 4096
  mr one --gpus 1 --steps 2 --warmup 1 --query 12288 --no-cpu-baseline
  for k in dyn2 static3; do
    python tools/compare_responses.py $OUT/$k.npz $OUT/one.npz > $OUT/compare_$k.json || die "compare $k" $OUT/compare_$k.json
    cat $OUT/compare_$k.json
  done
  ;;
*)
  echo "unknown task $TASK (check | ab | decab | kernels | profile | multirank | timeline)"; exit 2 ;;
esac
