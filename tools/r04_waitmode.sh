#!/bin/bash
# A/B of how the host waits for the GPU (HSA_ENABLE_INTERRUPT=0: the runtime polls completion
# signals instead of sleeping on an interrupt) for the Offline bench: an encode's gate is released
# only when its host thread has seen the encode finish, and the decode loop polls one chunk behind.
OUT=${OUT:-gpurun_out/r04wm}
mkdir -p $OUT
for i in 1 2; do
  for m in def 0; do
    if [ $m = def ]; then unset HSA_ENABLE_INTERRUPT; else export HSA_ENABLE_INTERRUPT=$m; fi
    timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline \
      > $OUT/int${m}_$i.json 2> $OUT/int${m}_$i.err || { echo "int$m run $i rc=$?"; tail -20 $OUT/int${m}_$i.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['frac'], r['isolated']['encode_ms_per_query'], r['isolated']['greedy_ms_per_query'])" $OUT/int${m}_$i.json int$m
  done
done
