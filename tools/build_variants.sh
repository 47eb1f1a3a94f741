#!/bin/bash
# Development: build ablation variants of the engine library into build_dev/ (git-ignored;
# selected at run time with RNNT_MI355X_LIB=build_dev/lib_<name>.so).
set -e
cd "$(dirname "$0")/../rnnt-inference_amd/csrc"
OUTD=../../build_dev
mkdir -p $OUTD
build() {
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -w "${@:2}" -c encoder.hip -o $OUTD/enc_$1.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -w "${@:2}" -c engine.hip -o $OUTD/eng_$1.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -w "${@:2}" -c decoder.hip -o $OUTD/dec_$1.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -w "${@:2}" -c encoder_f32.hip -o $OUTD/f32_$1.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OUTD/eng_$1.o $OUTD/dec_$1.o $OUTD/enc_$1.o $OUTD/f32_$1.o -o $OUTD/lib_$1.so
}
for v in "$@"; do
  case $v in
    base) build base ;;
    noepi) build noepi -DRNNT_DEV_NO_EPI ;;
    nomfma) build nomfma -DRNNT_DEV_NO_MFMA ;;
    nomfma_noepi) build nomfma_noepi -DRNNT_DEV_NO_MFMA -DRNNT_DEV_NO_EPI ;;
    same_nomfma_noepi) build same_nomfma_noepi -DRNNT_DEV_SAME_TILE -DRNNT_DEV_NO_MFMA -DRNNT_DEV_NO_EPI ;;
    noload_noepi) build noload_noepi -DRNNT_DEV_NO_LOAD -DRNNT_DEV_NO_EPI ;;
    noload) build noload -DRNNT_DEV_NO_LOAD ;;
    ji1) build ji1 -DRNNT_JOINT_ITERS=1 ;;
    ji2) build ji2 -DRNNT_JOINT_ITERS=2 ;;
    ji4) build ji4 -DRNNT_JOINT_ITERS=4 ;;
    ji8) build ji8 -DRNNT_JOINT_ITERS=8 ;;
    pred_nomfma) build pred_nomfma -DRNNT_DEV_PRED_NOMFMA ;;
    pred_nostage) build pred_nostage -DRNNT_DEV_PRED_NOSTAGE ;;
    pred_nowload) build pred_nowload -DRNNT_DEV_PRED_NOWLOAD ;;
    ns3) build ns3 -DRNNT_NSTAGE=3 ;;
    ns5) build ns5 -DRNNT_NSTAGE=5 ;;
    ns3_noepi) build ns3_noepi -DRNNT_NSTAGE=3 -DRNNT_DEV_NO_EPI ;;
    ns5_noepi) build ns5_noepi -DRNNT_NSTAGE=5 -DRNNT_DEV_NO_EPI ;;
    same_noepi) build same_noepi -DRNNT_DEV_SAME_TILE -DRNNT_DEV_NO_EPI ;;
    *) echo "unknown variant $v"; exit 1 ;;
  esac
done
