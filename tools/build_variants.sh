#!/bin/bash
# Development: build ablation variants of the engine library into build_dev/ (git-ignored;
# selected at run time with RNNT_MI355X_LIB=build_dev/lib_<name>.so).
set -e
cd "$(dirname "$0")/../rnnt-inference_amd/csrc"
OUTD=../../build_dev
mkdir -p $OUTD
build() { /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -w "${@:2}" engine.hip encoder.hip decoder.hip -o $OUTD/lib_$1.so; }
for v in "$@"; do
  case $v in
    base) build base ;;
    noepi) build noepi -DRNNT_DEV_NO_EPI ;;
    nomfma) build nomfma -DRNNT_DEV_NO_MFMA ;;
    nomfma_noepi) build nomfma_noepi -DRNNT_DEV_NO_MFMA -DRNNT_DEV_NO_EPI ;;
    *) echo "unknown variant $v"; exit 1 ;;
  esac
done
