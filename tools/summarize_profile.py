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
    per_query(src, stats[0] if stats else None, prefix)


def per_query(src, stats_csv, prefix):
    """Encoder kernel-time fraction per query from the traced bench run: the bench line (printed to
    trace.log) gives the int8 ops of one query (roofline.achieved x encode_ms_per_query) and the
    step count; the traced run holds warmup + timed + one isolated query (bench.py), so the tick
    kernels' total time / that many queries is the kernel time per query."""
    try:
        line = [x for x in open(os.path.join(src, "trace.log")) if x.startswith('{"metric"')][-1]
        b = json.loads(line)
    except (OSError, IndexError, ValueError):
        return
    r = b["roofline"]
    ops = r["achieved"] * 1e12 * r["encode_ms_per_query"] * 1e-3
    queries = b["steps"] + b["warmup"] + 1
    tick_ns = 0.0
    if stats_csv:
        for row in csv.DictReader(open(stats_csv)):
            if "lstm_i8_tick_kernel" in row["Name"]:
                tick_ns += float(row["TotalDurationNs"])
    if not tick_ns:
        return
    t = tick_ns * 1e-9 / queries
    out = {"queries_in_trace": queries, "note": "bench.py --warmup W --steps K traced: W + K queries + 1 isolated pass",
           "int8_ops_per_query": ops, "tick_kernel_ms_per_query": round(t * 1e3, 3),
           "tick_launches_per_query": r.get("tick_launches_per_query"),
           "encoder_kernel_time_frac": round(ops / t / 5.0e15, 4), "peak_tops": 5000.0,
           "bench_value": b["value"], "bench_roofline_frac_event_time": r["frac"]}
    json.dump(out, open(prefix + "_per_query.json", "w"), indent=1)
    print("per query:", out)


if __name__ == "__main__":
    main()
