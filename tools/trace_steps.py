"""Per-step decode timeline from a rocprofv3 --kernel-trace CSV (measurement tooling).

    python tools/trace_steps.py <dir with *_kernel_trace.csv>
Splits the trace into greedy steps (one dec_pred_kernel<0> starts each) and prints, for step
ranges, the mean duration of each decode kernel and the mean step span (first start to last
end), so the early (throughput) and tail (latency) regimes can be told apart.
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
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    steps, cur = [], None
    for s, e, n in rows:
        if n.startswith("dec_pred_kernel<0"):
            cur = {"start": s, "k": {}}
            steps.append(cur)
        if cur is not None and n.startswith(("dec_pred", "dec_g", "dec_joint")):
            cur["k"][n] = (s, e)
            cur["end"] = e
    # split into decodes: a gap > 1 ms between steps starts a new decode
    decs, d = [], []
    for st in steps:
        if d and st["start"] - d[-1]["end"] > 1_000_000:
            decs.append(d)
            d = []
        d.append(st)
    if d:
        decs.append(d)
    for di, d in enumerate(decs[:6]):
        n = len(d)
        print(f"decode {di}: {n} steps, span {(d[-1]['end'] - d[0]['start']) / 1e6:.2f} ms")
        for lo, hi in ((0, 10), (10, 50), (50, 200), (200, 400), (400, 600), (600, 10000)):
            seg = d[lo:min(hi, n)]
            if not seg:
                continue
            span = sum(x["end"] - x["start"] for x in seg) / len(seg) / 1e3
            ks = {}
            for x in seg:
                for k, (s, e) in x["k"].items():
                    ks.setdefault(k, []).append((e - s) / 1e3)
            kd = " ".join(f"{k.split('_')[1]}{k[-3:] if 'pred' in k else ''}={sum(v) / len(v):.1f}" for k, v in sorted(ks.items()))
            print(f"  steps {lo:4d}-{min(hi, n):4d}: step {span:6.1f} us | {kd}")


if __name__ == "__main__":
    main()
