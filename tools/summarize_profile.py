"""Condense a tools/profile_round.sh output directory into profiles/ artefacts.

    python tools/summarize_profile.py gpurun_out/prof_round profiles/r01
writes <prefix>_kernel_stats.csv (rocprofv3 --stats, copied), <prefix>_pmc_summary.json
(per-kernel mean counters per dispatch, derived HBM bytes/launch with the gfx950 FETCH_SIZE x2
correction) and tools/roofline_traffic.json (read by bench.py's roofline.traffic; tools/ travels to the GPU
box, profiles/ does not).
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys


def main():
    src, prefix = sys.argv[1], sys.argv[2]
    os.makedirs(os.path.dirname(prefix) or ".", exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], prefix + "_kernel_stats.csv")
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(src, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    summary = {}
    for k, cs in agg.items():
        if k.startswith("void at::") or k.startswith("__amd"):
            continue
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        d["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes_per_launch"] = (2.0 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024.0
        if "SQ_VALU_MFMA_BUSY_CYCLES" in d and "GRBM_GUI_ACTIVE" in d:
            # GRBM_GUI_ACTIVE sums the 8 XCDs; 1024 SIMDs on the chip
            d["mfma_busy_frac"] = d["SQ_VALU_MFMA_BUSY_CYCLES"] / (d["GRBM_GUI_ACTIVE"] / 8.0 * 1024.0)
        summary[k] = d
    json.dump(summary, open(prefix + "_pmc_summary.json", "w"), indent=1, sort_keys=True)
    # the dominant tick kernel: the tile-shape instantiation with the most dispatches (the 256 x 256 one)
    ticks = [d for k, d in summary.items() if "lstm_i8_tick_kernel" in k]
    tick = max(ticks, key=lambda d: d.get("dispatches", 0)) if ticks else {}
    if "hbm_bytes_per_launch" in tick:
        json.dump({"lstm_i8_step_bytes_per_launch": tick["hbm_bytes_per_launch"], "source": prefix + "_pmc_summary.json"},
                  open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "roofline_traffic.json"), "w"), indent=1)
    for k, d in summary.items():
        print(k, {c: round(v, 3) for c, v in d.items() if c in ("dispatches", "hbm_bytes_per_launch", "mfma_busy_frac", "SQ_INSTS_VALU", "SQ_INSTS_MFMA")})


if __name__ == "__main__":
    main()
