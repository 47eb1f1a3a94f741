#!/bin/bash
# Featurizer throughput per variant library (alternating, one box): shipped (3 chunks per
# workgroup, CU-owning LDS, packed FP32) vs the round-2 shape without the reservation and without
# packed FP32 (-fno-slp-vectorize: the corruption's trigger).
OUT=${OUT:-gpurun_out/r04fzp}
mkdir -p $OUT
for i in 1 2; do
  for v in ${VARIANTS:-fzbase fz1nslp}; do
    RNNT_MI355X_LIB=build_dev/lib_$v.so timeout -k 10 240 python -u tools/bench_featurizer.py > $OUT/fz_${v}_$i.json 2> $OUT/fz_${v}_$i.err \
      || { echo "$v rc=$?"; tail -20 $OUT/fz_${v}_$i.err; exit 1; }
    echo "$v $i $(tail -c 300 $OUT/fz_${v}_$i.json)"
  done
done
