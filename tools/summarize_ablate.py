"""Condense tools/enc_ablate.sh output: per variant, the tick kernel's LDS bank-conflict share
(SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE), LDS / VALU / MFMA instruction counts per dispatch and
the K2048 layer-step time from bench_kernels.py.

    python tools/summarize_ablate.py gpurun_out/ablate > summary.json
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    src = sys.argv[1]
    out = {}
    for v in ("base", "notab", "noimg", "both", "noc"):
        rec = {}
        try:
            rec["time"] = json.load(open(os.path.join(src, f"time_{v}.json")))
        except Exception as ex:  # keep the other variants
            rec["time_error"] = str(ex)
        agg = collections.defaultdict(list)
        for f in glob.glob(os.path.join(src, f"pmc_{v}", "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "lstm_i8_tick_kernel" not in r["Kernel_Name"] or "4, 8, 2" not in r["Kernel_Name"].replace("4,8,2", "4, 8, 2"):
                    continue
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        d = {c: sum(x) / len(x) for c, x in agg.items()}
        if d.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_conflict_frac"] = d.get("SQ_LDS_BANK_CONFLICT", 0.0) / d["SQ_LDS_IDX_ACTIVE"]
        rec["pmc"] = d
        out[v] = rec
    json.dump(out, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
