set -e
mkdir -p gpurun_out/c5
for v in base noepi nomfma_noepi noload_noepi noload; do
  for n in 2560 5120; do
    echo -n "$v $n " >> gpurun_out/c5/abl.txt
    RNNT_MI355X_LIB=build_dev/lib_$v.so timeout -k 10 200 python tools/bench_kernels.py --n $n --T 16 --layers 1 --skip-decode >> gpurun_out/c5/abl.txt 2>gpurun_out/c5/$v.err || echo "FAIL $v" >> gpurun_out/c5/abl.txt
  done
done
cat gpurun_out/c5/abl.txt
