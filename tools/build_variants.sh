#!/bin/bash
# Development: build variants of the engine library with extra compile flags into build_dev/
# (git-ignored; selected at run time with RNNT_MI355X_LIB=build_dev/lib_<name>.so).  Variants read the
# development environment knobs (RNNT_ENC_TILE, RNNT_DEC_PERSIST_ROWS, RNNT_DEC_RG, ...: -DRNNT_DEV_KNOBS);
# the product library does not.
#   tools/build_variants.sh base "asm0:-DRNNT_FRAG_ASM=0" "stamps:-DRNNT_DEV_STAMPS"
set -e
cd "$(dirname "$0")/../rnnt-inference_amd/csrc"
OUTD=../../build_dev
mkdir -p $OUTD
HIPCC="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -w -DRNNT_DEV_KNOBS -fno-slp-vectorize -Xclang -target-feature -Xclang -packed-fp32-ops"
build() {
  local name=$1; shift
  local objs=""
  for src in engine encoder encoder_f32 decoder decoder_f32 decoder_ops featurizer processor_ops; do
    local extra=""
    [ $src = encoder -o $src = featurizer ] && extra="-fno-slp-vectorize"
    $HIPCC $extra "$@" -c $src.hip -o $OUTD/${src}_$name.o &
    objs="$objs $OUTD/${src}_$name.o"
  done
  g++ -std=c++17 -O2 -fPIC -c crash_report.cpp -o $OUTD/crash_report_$name.o &
  objs="$objs $OUTD/crash_report_$name.o"
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o $OUTD/lib_$name.so
  echo "built $OUTD/lib_$name.so"
}
for v in "$@"; do
  name=${v%%:*}
  flags=""
  [[ $v == *:* ]] && flags=${v#*:}
  build $name $flags
done
