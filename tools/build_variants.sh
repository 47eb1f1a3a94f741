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
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -w "${@:2}" -c decoder_ops.hip -o $OUTD/dops_$1.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -w "${@:2}" -c featurizer.hip -o $OUTD/fz_$1.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OUTD/eng_$1.o $OUTD/dec_$1.o $OUTD/enc_$1.o $OUTD/f32_$1.o $OUTD/dops_$1.o $OUTD/fz_$1.o -o $OUTD/lib_$1.so
}
for v in "$@"; do
  case $v in
    base) build base ;;
    nostagger) build nostagger -DRNNT_STAGGER=0 ;;
    stagger1) build stagger1 -DRNNT_STAGGER=1 -DRNNT_STAGGER_AT=1 ;;
    stagger_p1) build stagger_p1 -DRNNT_STAGGER=1 -DRNNT_PRIO_MODE=1 ;;
    stagger_p2) build stagger_p2 -DRNNT_STAGGER=1 -DRNNT_PRIO_MODE=2 ;;
    stagger3) build stagger3 -DRNNT_STAGGER=1 -DRNNT_STAGGER_AT=3 ;;
    persist) build persist -DRNNT_PERSIST=1 ;;
    persist2) build persist2 -DRNNT_PERSIST=2 ;;
    stamps_p2) build stamps_p2 -DRNNT_DEV_STAMPS -DRNNT_PERSIST=2 ;;
    persist2_f1) build persist2_f1 -DRNNT_PERSIST=2 -DRNNT_PERSIST_FREE=1 ;;
    persist2_f2) build persist2_f2 -DRNNT_PERSIST=2 -DRNNT_PERSIST_FREE=2 ;;
    epi_nobq) build epi_nobq -DRNNT_DEV_EPI_NOBQ ;;
    epi_nostore) build epi_nostore -DRNNT_DEV_EPI_NOSTORE ;;
    epi_nostore_notab) build epi_nostore_notab -DRNNT_DEV_EPI_NOSTORE -DRNNT_DEV_NO_TAB ;;
    fz_noload) build fz_noload -DRNNT_DEV_FZ_NO_LOAD ;;
    fz_nofft) build fz_nofft -DRNNT_DEV_FZ_NO_FFT ;;
    fz_nomel) build fz_nomel -DRNNT_DEV_FZ_NO_MEL ;;
    fz_nofft_nomel) build fz_nofft_nomel -DRNNT_DEV_FZ_NO_FFT -DRNNT_DEV_FZ_NO_MEL ;;
    fz_none) build fz_none -DRNNT_DEV_FZ_NO_LOAD -DRNNT_DEV_FZ_NO_FFT -DRNNT_DEV_FZ_NO_MEL ;;
    noepi) build noepi -DRNNT_DEV_NO_EPI ;;
    nomfma) build nomfma -DRNNT_DEV_NO_MFMA ;;
    nomfma_noepi) build nomfma_noepi -DRNNT_DEV_NO_MFMA -DRNNT_DEV_NO_EPI ;;
    same_nomfma_noepi) build same_nomfma_noepi -DRNNT_DEV_SAME_TILE -DRNNT_DEV_NO_MFMA -DRNNT_DEV_NO_EPI ;;
    noload_noepi) build noload_noepi -DRNNT_DEV_NO_LOAD -DRNNT_DEV_NO_EPI ;;
    noload) build noload -DRNNT_DEV_NO_LOAD ;;
    ji1) build ji1 -DRNNT_JOINT_ITERS=1 ;;
    stamps) build stamps -DRNNT_DEV_STAMPS ;;
    bk64) build bk64 -DRNNT_BK128=0 ;;
    pr96) build pr96 -DRNNT_PRED_RG=96 ;;
    pw1024) build pw1024 -DRNNT_PRED_WIDE_MIN=1024 ;;
    pw2048) build pw2048 -DRNNT_PRED_WIDE_MIN=2048 ;;
    pw4096) build pw4096 -DRNNT_PRED_WIDE_MIN=4096 ;;
    pr32) build pr32 -DRNNT_PRED_RG=32 ;;
    jg1024) build jg1024 -DRNNT_JOINT_G=1024 ;;
    gr192) build gr192 -DRNNT_G_RG=192 ;;
    xg8) build xg8 -DRNNT_XCD_G=8 ;;
    is3) build is3 -DRNNT_BK128_ISSUE=3 ;;
    is4) build is4 -DRNNT_BK128_ISSUE=4 ;;
    is5) build is5 -DRNNT_BK128_ISSUE=5 ;;
    jt_old) build jt_old -DRNNT_JT_GEMM=0 ;;
    bk128_i1) build bk128_i1 -DRNNT_BK128_ISSUE=1 ;;
    stamps_bk64) build stamps_bk64 -DRNNT_DEV_STAMPS -DRNNT_BK128=0 ;;
    bk128_i0) build bk128_i0 -DRNNT_BK128_ISSUE=0 ;;
    bk64_noepi) build bk64_noepi -DRNNT_BK128=0 -DRNNT_DEV_NO_EPI ;;
    tab16) build tab16 -DRNNT_TAB_COPIES=16 ;;
    rt64) build rt64 -DRNNT_DEC_RT=64 ;;
    ji3) build ji3 -DRNNT_JOINT_ITERS=3 ;;
    ji6) build ji6 -DRNNT_JOINT_ITERS=6 ;;
    jg128) build jg128 -DRNNT_JOINT_G=128 ;;
    jg256) build jg256 -DRNNT_JOINT_G=256 ;;
    ji2) build ji2 -DRNNT_JOINT_ITERS=2 ;;
    ji4) build ji4 -DRNNT_JOINT_ITERS=4 ;;
    ji8) build ji8 -DRNNT_JOINT_ITERS=8 ;;
    pred_nomfma) build pred_nomfma -DRNNT_DEV_PRED_NOMFMA ;;
    pred_nostage) build pred_nostage -DRNNT_DEV_PRED_NOSTAGE ;;
    pred_nowload) build pred_nowload -DRNNT_DEV_PRED_NOWLOAD ;;
    dg_a) build dg_a -DRNNT_PRED_RG=25 -DRNNT_G_RG=96 -DRNNT_JOINT_G=512 ;;
    dg_b) build dg_b -DRNNT_PRED_RG=8 -DRNNT_G_RG=24 -DRNNT_JOINT_G=128 ;;
    dg_c) build dg_c -DRNNT_PRED_RG=12 -DRNNT_G_RG=40 -DRNNT_JOINT_G=256 ;;
    dg_d) build dg_d -DRNNT_PRED_RG=5 -DRNNT_G_RG=16 -DRNNT_JOINT_G=64 ;;
    wn1) build wn1 -DENC_WN=1 ;;
    wn1_ns4) build wn1_ns4 -DENC_WN=1 -DRNNT_NSTAGE=4 ;;
    wn1_noepi) build wn1_noepi -DENC_WN=1 -DRNNT_DEV_NO_EPI ;;
    noread_noload_noepi) build noread_noload_noepi -DRNNT_DEV_NO_READ -DRNNT_DEV_NO_LOAD -DRNNT_DEV_NO_EPI ;;
    noread_noepi) build noread_noepi -DRNNT_DEV_NO_READ -DRNNT_DEV_NO_EPI ;;
    il) build il -DRNNT_INTERLEAVE=1 ;;
    il_noepi) build il_noepi -DRNNT_INTERLEAVE=1 -DRNNT_DEV_NO_EPI ;;
    notab) build notab -DRNNT_DEV_NO_TAB ;;
    ns3) build ns3 -DRNNT_NSTAGE=3 ;;
    ns5) build ns5 -DRNNT_NSTAGE=5 ;;
    ns3_noepi) build ns3_noepi -DRNNT_NSTAGE=3 -DRNNT_DEV_NO_EPI ;;
    ns5_noepi) build ns5_noepi -DRNNT_NSTAGE=5 -DRNNT_DEV_NO_EPI ;;
    same_noepi) build same_noepi -DRNNT_DEV_SAME_TILE -DRNNT_DEV_NO_EPI ;;
    *) echo "unknown variant $v"; exit 1 ;;
  esac
done
