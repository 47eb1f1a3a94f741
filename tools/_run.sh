set -e
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { tail -20 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/t7
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/t7/tr -o kb -- python3 tools/bench_kernels.py --n 8192 --layers "" > gpurun_out/t7/kb.log 2>&1
python3 - <<'P'
import csv, glob, sys, numpy as np
f = glob.glob('gpurun_out/t7/tr/**/kb_kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
dec = [(r['Kernel_Name'].split('(')[0].replace('rnnt::', ''), int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in rows if 'dec_' in r['Kernel_Name']]
dec = dec[len(dec)//2:]
out = []
for name in ('dec_pred_kernel', 'dec_g_kernel', 'dec_joint_kernel'):
    d = np.array([(e - s) / 1e3 for n, s, e in dec if n == name])
    out.append(f"{name}: n={len(d)} med={np.median(d):.2f} tail={np.median(d[-len(d)//3:]):.2f} max={d.max():.1f} sum={d.sum()/1e3:.1f}ms")
print(" | ".join(out))
P
find gpurun_out/t7 -name "*.csv" -delete
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_c16.json 2> gpurun_out/bench_c16.err
python3 -c "
import json; d=json.load(open('gpurun_out/bench_c16.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['encode_ms_per_query'], r['greedy_ms_per_query'], r['isolated'])"
