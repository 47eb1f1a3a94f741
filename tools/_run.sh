set -e
mkdir -p gpurun_out/c11
for v in base p0 p0prio base p0 p0prio; do
  echo -n "$v " >> gpurun_out/c11/abl.txt
  RNNT_MI355X_LIB=build_dev/lib_$v.so timeout -k 10 300 python tools/bench_kernels.py --n 8192 --T 16 --layers 1,2,0 >> gpurun_out/c11/abl.txt 2>gpurun_out/c11/$v.err || echo FAIL >> gpurun_out/c11/abl.txt
done
python3 - <<'P'
import json
for line in open('gpurun_out/c11/abl.txt'):
    v, js = line.split(' ', 1)
    d = json.loads(js)
    print(v, d['step_K1280']['us_per_launch'], d['step_K2048']['us_per_launch'], d['step_K3072']['us_per_launch'], d['infer_batch']['encode_ms'])
P
