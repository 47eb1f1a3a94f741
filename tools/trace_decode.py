"""Decode timeline from a rocprofv3 --kernel-trace CSV (test/measurement tooling).

    python tools/trace_decode.py <dir with *_kernel_trace.csv> [label]
Per kernel: dispatch count, mean duration; for the greedy loop's kernels also the mean gap
between the end of one decode kernel and the start of the next on the same queue (launch /
dependency latency), split by whether an encoder tick kernel was running at the time.
"""
import collections
import csv
import glob
import json
import sys


def main():
    d = sys.argv[1]
    files = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("rnnt::", "")
            q = r.get("Queue_Id") or r.get("Stream_Id") or "0"
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, q))
    rows.sort()
    ticks = [(s, e) for s, e, n, _ in rows if n == "lstm_i8_tick_kernel"]
    # merge tick intervals for an "encoder busy" test
    busy = []
    for s, e in ticks:
        if busy and s <= busy[-1][1]:
            busy[-1][1] = max(busy[-1][1], e)
        else:
            busy.append([s, e])
    import bisect
    starts = [b[0] for b in busy]

    def enc_busy(t):
        i = bisect.bisect_right(starts, t) - 1
        return i >= 0 and busy[i][1] >= t

    dur = collections.defaultdict(lambda: [[], []])
    gaps = [[], []]
    last_end = {}
    dec = {"dec_pred_kernel", "dec_g_kernel", "dec_joint_kernel"}
    for s, e, n, q in rows:
        ov = 1 if enc_busy(s) else 0
        dur[n][ov].append(e - s)
        if n in dec:
            if q in last_end and s - last_end[q] < 1_000_000:
                gaps[ov].append(s - last_end[q])
            last_end[q] = e

    def m(v):
        return round(sum(v) / len(v) / 1000.0, 2) if v else None

    out = {"label": sys.argv[2] if len(sys.argv) > 2 else d}
    for n, (a, b) in sorted(dur.items(), key=lambda kv: -sum(kv[1][0]) - sum(kv[1][1])):
        if n.startswith("void at::") or n.startswith("__amd"):
            continue
        out[n] = {"alone_n": len(a), "alone_us": m(a), "beside_enc_n": len(b), "beside_enc_us": m(b),
                  "total_ms": round((sum(a) + sum(b)) / 1e6, 2)}
    out["decode_gap_us"] = {"alone": m(gaps[0]), "beside_enc": m(gaps[1]), "n": [len(gaps[0]), len(gaps[1])]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
