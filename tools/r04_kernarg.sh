#!/bin/bash
# A/B of where the HIP runtime puts kernel arguments (HIP_FORCE_DEV_KERNARG: 1 = device memory,
# 0 = host memory the command processor fetches over PCIe) for the Offline bench; the decode
# issues four dependent launches per step, so its isolated time is the sensitive figure.
OUT=${OUT:-gpurun_out/r04ka}
mkdir -p $OUT
for i in 1 2; do
  for k in def 1 0; do
    if [ $k = def ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$k; fi
    timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline \
      > $OUT/ka${k}_$i.json 2> $OUT/ka${k}_$i.err || { echo "ka$k run $i rc=$?"; tail -20 $OUT/ka${k}_$i.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['frac'], r['isolated']['encode_ms_per_query'], r['isolated']['greedy_ms_per_query'], r['decode']['isolated_frac'])" $OUT/ka${k}_$i.json ka$k
  done
done
