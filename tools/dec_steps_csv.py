"""Per-step decode times from a rocprofv3 --kernel-trace CSV (development tool).

    python tools/dec_steps_csv.py <kernel_trace.csv> [more.csv ...]

Splits the trace into decode calls (each starts with dec_init_kernel / dec_init_stream_kernel),
a step ending at each dec_joint_kernel; the step's span is from the previous step's joint end (or
the call's init end) to its joint end, so launch gaps are included.  Prints, per call and per
step-index bucket, the mean step span and the mean kernel time per kernel kind, so that step
structures (four launches: pred<0>, pred<1>, G, joint; three: pred<1>, G, joint) can be compared
on the early (many rows) and the tail (few rows) steps.
"""
import csv
import json
import sys

KINDS = {"dec_pred_kernel<0": "pred0", "dec_pred_kernel<1": "pred1", "dec_g_kernel": "g", "dec_joint_kernel": "joint"}
BUCKETS = [(0, 25), (25, 50), (50, 100), (100, 200), (200, 300), (300, 400), (400, 600), (600, 1000)]


def kind(name):
    for k, v in KINDS.items():
        if k in name:
            return v
    if "dec_init" in name:
        return "init"
    return None


def main():
    rows = []
    for f in sys.argv[1:]:
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name") or r.get("Name") or ""
            k = kind(name)
            if k is None:
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    calls, cur = [], None
    for s, e, k in rows:
        if k == "init":
            cur = {"t": e, "steps": [], "acc": {}}
            calls.append(cur)
            continue
        if cur is None:
            continue
        cur["acc"][k] = cur["acc"].get(k, 0.0) + (e - s) / 1e3
        if k == "joint":
            cur["steps"].append({"span": (e - cur["t"]) / 1e3, **cur["acc"]})
            cur["t"], cur["acc"] = e, {}
    out = []
    for i, c in enumerate(calls):
        st = c["steps"]
        rec = {"call": i, "steps": len(st), "span_ms": round(sum(x["span"] for x in st) / 1e3, 3), "buckets": {}}
        for lo, hi in BUCKETS:
            part = st[lo:hi]
            if not part:
                continue
            m = {k: round(sum(x.get(k, 0.0) for x in part) / len(part), 2) for k in ("span", "pred0", "pred1", "g", "joint")}
            rec["buckets"][f"{lo}-{hi}"] = m
        out.append(rec)
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
