#!/bin/bash
# Round-4 measurement pass (after tools/r04_check.sh is green): decode A/B of the early
# weight-slice issue (base vs earlyw, alternating), the encoder epilogue LDS ablations, then the
# round profile (kernel-trace stats + separate PMC passes) of the default bench.  Each step has
# its own time limit; the chain stops at the first failure.  Build first on the CPU:
#   make -C rnnt-inference_amd/csrc && cp rnnt-inference_amd/rnnt_amd/librnnt_mi355x.so build_dev/lib_base.so
#   tools/build_variants.sh earlyw:-DRNNT_DEC_EARLY_W=1 notab:-DRNNT_ABL_NOTAB noimg:-DRNNT_ABL_NOIMG \
#     both:"-DRNNT_ABL_NOTAB -DRNNT_ABL_NOIMG"
set -e
OUT=${OUT:-gpurun_out/r04perf}
mkdir -p $OUT
if [ -z "$NO_AB" ]; then
  for r in 1 2; do
    for v in 4l base earlyw; do
      RNNT_MI355X_LIB=build_dev/lib_$v.so timeout -k 10 240 python3 -u tools/bench_decode.py > $OUT/dec_${v}_$r.json 2> $OUT/dec_${v}_$r.err
      tail -c 400 $OUT/dec_${v}_$r.json; echo
    done
  done
fi
if [ -z "$NO_ABL" ]; then
  timeout -k 10 900 bash tools/enc_ablate.sh $OUT/ablate > $OUT/ablate.log 2>&1
  tail -c 1500 $OUT/ablate/summary.json; echo
fi
if [ -z "$NO_PROF" ]; then
  PREFIX=$OUT/summary/r04 timeout -k 10 1500 bash tools/profile_round.sh $OUT/prof > $OUT/prof.log 2>&1
  tail -20 $OUT/prof.log
fi
