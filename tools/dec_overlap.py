"""Decode step kernels overlapped with the encoder vs alone, from a rocprofv3 --kernel-trace CSV
(measurement tooling).

    python tools/dec_overlap.py <dir with *_kernel_trace.csv>

For every dec_pred / dec_g / dec_joint dispatch: its duration (start -> end of the kernel) and the
gap since the previous decode kernel on the same queue ended (launch + dispatch wait).  Dispatches
are split by whether any lstm_i8_tick_kernel was running at their start.  Prints per kernel kind
and regime: count, mean / p50 / p90 duration and gap (us)."""
import bisect
import csv
import glob
import json
import sys


def main():
    rows = []
    for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            q = r.get("Queue_Id") or r.get("Stream_Id") or "0"
            g = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0) // max(1, int(r.get("Workgroup_Size") or r.get("Workgroup_Size_X") or 1))
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, q, g))
    rows.sort()
    ticks = [(s, e) for s, e, n, _, _ in rows if "lstm_i8_tick_kernel" in n]
    starts = [s for s, _ in ticks]
    # running[t] = any tick active at time t: ticks on one queue do not overlap each other, but several
    # queues may encode; a prefix max of ends answers "some tick started before t and ends after t"
    pmax, m = [], 0
    for s, e in ticks:
        m = max(m, e)
        pmax.append(m)

    def tick_active(t):
        i = bisect.bisect_right(starts, t) - 1
        return i >= 0 and pmax[i] > t

    kinds = {"dec_pred_kernel<0": "pred0", "dec_pred_kernel<1": "pred1", "dec_g_kernel": "g", "dec_joint_kernel": "joint"}
    last_end = {}
    stats = {}
    for s, e, n, q, g in rows:
        k = next((v for key, v in kinds.items() if key in n), None)
        if k is None:
            if "joint_trans" in n or "dec_init" in n:
                last_end[q] = e
            continue
        gap = s - last_end[q] if q in last_end else None
        last_end[q] = e
        # grid size: the step kernels launch one row group (pred 20, G 8 workgroups; joint <= 16 rows
        # per workgroup) once few rows are live
        size = "tail" if (k in ("pred0", "pred1") and g <= 20) or (k == "g" and g <= 8) or (k == "joint" and g <= 4) else "bulk"
        reg = ("overlapped" if tick_active(s) else "alone") + "/" + size
        d = stats.setdefault(reg, {}).setdefault(k, {"dur": [], "gap": []})
        d["dur"].append((e - s) / 1e3)
        if gap is not None and gap < 5e6:
            d["gap"].append(gap / 1e3)
    out = {}
    for reg, ks in stats.items():
        for k, d in ks.items():
            def summ(v):
                if not v:
                    return None
                v = sorted(v)
                return {"mean": round(sum(v) / len(v), 2), "p50": round(v[len(v) // 2], 2), "p90": round(v[int(len(v) * 0.9)], 2)}
            out[f"{reg}/{k}"] = {"n": len(d["dur"]), "dur_us": summ(d["dur"]), "gap_us": summ(d["gap"])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
