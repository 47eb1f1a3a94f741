set -e
OUT=gpurun_out/c9 BENCH_ARGS=--no-cpu-baseline tools/gpu_check.sh
echo -n "noepi " ; RNNT_MI355X_LIB=build_dev/lib_noepi.so timeout -k 10 200 python tools/bench_kernels.py --n 2560 --T 16 --layers 1 --skip-decode
