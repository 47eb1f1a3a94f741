#!/bin/bash
# A/B of the HIP hardware-queue count (GPU_MAX_HW_QUEUES, 4 by default on the box) for the Offline
# bench: streams beyond the queue count share an in-order hardware queue, so an encode and a
# decode that land on one queue cannot overlap.  Same box, alternating; each run has its own limit.
OUT=${OUT:-gpurun_out/r04hwq}
mkdir -p $OUT
for i in 1 2; do
  for q in 4 8 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline \
      > $OUT/q${q}_$i.json 2> $OUT/q${q}_$i.err || { echo "q$q run $i rc=$?"; tail -20 $OUT/q${q}_$i.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['decode']['frac'])" $OUT/q${q}_$i.json q$q
  done
done
