"""Per-batch timeline of bench.py queries from a rocprofv3 --kernel-trace CSV (measurement tooling).

    python tools/trace_query.py <dir with *_kernel_trace.csv>
Tick kernels are also binned by grid size (workgroups: one CU each), so the time spent in
sparse ticks (fewer tiles than CUs) can be read off.
A batch on a queue = quantize_kernel, the tick kernels (encode), joint_trans_kernel and the
greedy loop's kernels (decode).  Prints, per batch in start order, the encode and decode spans
relative to the first kernel of the trace (ms), so the overlap of one batch's decode with the
next batch's encode and the decode tail of a query can be read off directly.
"""
import csv
import glob
import sys


def main():
    files = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("rnnt::", "").replace("void ", "")
            q = r.get("Queue_Id") or r.get("Stream_Id") or "0"
            g = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0) // max(1, int(r.get("Workgroup_Size") or r.get("Workgroup_Size_X") or 1))
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, q, g))
    rows.sort()
    t0 = rows[0][0]
    batches, cur = [], {}
    dec_cur = {}  # decode queue -> batch (a decode may run on its own stream: RNNT_SUT_DEC_PRIORITY / ENC_RESERVE)
    buckets = (256, 512, 1024, 1 << 30)
    for s, e, n, q, g in rows:
        if n.startswith("quantize"):
            b = {"q": q, "enc": [s, e], "dec": None, "ticks": 0, "hist": [[0, 0.0] for _ in buckets]}
            batches.append(b)
            cur[q] = b
            continue
        if n.startswith("lstm_i8_tick_kernel"):
            b = cur.get(q)
            if b is None:
                continue
            b["enc"][1] = e
            b["ticks"] += 1
            k = next(i for i, lim in enumerate(buckets) if g <= lim)
            b["hist"][k][0] += 1
            b["hist"][k][1] += (e - s) / 1e6
        elif n.startswith(("joint_trans", "dec_")):
            if n.startswith("joint_trans"):
                # a decode starts: the batch encoded on this queue if it has none yet, else (a decode
                # on its own stream) the oldest encoded batch still without one
                b = cur.get(q)
                if b is None or b["dec"] is not None:
                    b = next((x for x in batches if x["dec"] is None and x["enc"][1] <= s), None)
                if b is None:
                    continue
                dec_cur[q] = b
            b = dec_cur.get(q)
            if b is None:
                continue
            if b["dec"] is None:
                b["dec"] = [s, e]
            b["dec"][1] = e
    for i, b in enumerate(batches):
        d = b["dec"] or [0, 0]
        print(f"batch {i:3d} q{b['q']}: encode {(b['enc'][0] - t0) / 1e6:9.2f} .. {(b['enc'][1] - t0) / 1e6:9.2f} "
              f"({(b['enc'][1] - b['enc'][0]) / 1e6:6.2f} ms, {b['ticks']} ticks) | decode {(d[0] - t0) / 1e6:9.2f} .. "
              f"{(d[1] - t0) / 1e6:9.2f} ({(d[1] - d[0]) / 1e6:6.2f} ms)")
        print("      ticks by workgroups  <=256: %d / %.1f ms  <=512: %d / %.1f ms  <=1024: %d / %.1f ms  more: %d / %.1f ms"
              % tuple(x for h in b["hist"] for x in h))


if __name__ == "__main__":
    main()
