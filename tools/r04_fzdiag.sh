#!/bin/bash
# Featurizer corruption beside the decode, re-checked on the round-4 decode kernels:
# the shipped featurizer (CU-owning LDS request), the round-2 workgroup shape without it (one
# 4-wave chunk per workgroup, 3 per CU: decode workgroups can share its CU) and the round-3 shape
# without it.  tools/diag_fz_concurrency.py repeats one featurizer batch beside each co-runner and
# counts batches that differ from the quiet result.
OUT=${OUT:-gpurun_out/r04fz}
mkdir -p $OUT
for v in ${VARIANTS:-fz1np fzbase fz3np}; do
  RNNT_MI355X_LIB=build_dev/lib_$v.so timeout -k 10 240 python -u tools/diag_fz_concurrency.py --seconds 20 \
    --modes ${MODES:-none,decode,featurize} --out $OUT/diag_$v.json > $OUT/diag_$v.log 2>&1 || { echo "$v rc=$?"; tail -20 $OUT/diag_$v.log; exit 1; }
  echo "== $v"; grep -v "^\s*$" $OUT/diag_$v.log | tail -4
done
