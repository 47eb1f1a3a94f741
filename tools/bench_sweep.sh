#!/bin/bash
# Runs bench.py once per argument set (each a quoted string) and collects the JSON lines.
# Stops at the first failing run.  Usage: tools/bench_sweep.sh OUTDIR "args1" "args2" ...
# An argument set may start with lib=<variant> to run build_dev/lib_<variant>.so.
set -e
OUT=$1; shift
mkdir -p $OUT
i=0
for A in "$@"; do
  i=$((i+1))
  echo "== $A" | tee -a $OUT/sweep.txt
  LIBV=""
  if [[ "$A" == lib=* ]]; then LIBV=${A%% *}; LIBV=${LIBV#lib=}; A=${A#* }; fi
  if [ -n "$LIBV" ]; then export RNNT_MI355X_LIB=build_dev/lib_$LIBV.so; else unset RNNT_MI355X_LIB; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline $A > $OUT/b$i.json 2> $OUT/b$i.err || { tail -20 $OUT/b$i.err; exit 1; }
  python - $OUT/b$i.json <<'PY' | tee -a $OUT/sweep.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"value {d['value']:.0f} ms/step {d['ms_per_step']:.1f} frac {r['frac']} enc {r['encode_ms_per_query']} "
      f"greedy {r['greedy_ms_per_query']} jt {r['joint_trans_ms_per_query']} iso_enc {r['isolated']['encode_ms_per_query']} "
      f"iso_greedy {r['isolated']['greedy_ms_per_query']}")
PY
done
