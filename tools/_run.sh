set -e
mkdir -p gpurun_out/s3
for cfg in "--inflight 3 --batch 8192" "--inflight 3 --batch 6144" "--inflight 4 --batch 6144" "--inflight 4 --batch 4096" "--inflight 6 --batch 4096" "--inflight 3 --batch 4096"; do
  echo "$cfg" >> gpurun_out/s3/res.txt
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline $cfg >> gpurun_out/s3/res.txt 2>gpurun_out/s3/err.txt
done
cat gpurun_out/s3/res.txt | python3 -c "
import sys,json
for line in sys.stdin:
    line=line.strip()
    if line.startswith('{'):
        d=json.loads(line); r=d['roofline']; print(d['value'], d['ms_per_step'], r['encode_ms_per_query'], r['greedy_ms_per_query'], r['joint_trans_ms_per_query'])
    else: print(line)
"
