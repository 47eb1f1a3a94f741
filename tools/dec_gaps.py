"""Where the decode loop's time between kernels goes (development tool).

    python tools/dec_gaps.py <rocprofv3 output dir with *kernel_trace.csv>

Per decode call (from dec_init_kernel to the next) the step kernels (pred0, pred1, G, joint) are
split into steps; every gap between consecutive kernels is attributed to one of:
  intra     -- inside a step (pred0 -> pred1 -> G -> joint): dependent launch boundaries;
  step      -- joint -> next pred0 with no other kernel between;
  chunk     -- joint -> next pred0 across the host loop's poll (the live-count copy kernel the
               host enqueues after each chunk, __amd_rocclr_copyBuffer, lies between).
Reported for the early steps and for the tail (the last TAIL steps of each call), as microseconds
per step, next to the kernel time per step.  A chunk gap much larger than a step gap says the
GPU waited for the host to enqueue the next chunk.
"""
import csv
import glob
import json
import os
import sys

TAIL = 200
KINDS = (("dec_pred_kernel<0", "pred0"), ("dec_pred_kernel<1", "pred1"), ("dec_g_kernel", "g"),
         ("dec_joint_kernel", "joint"), ("copyBuffer", "copy"), ("dec_init", "init"), ("dec_finish", "finish"))


def kind(name):
    for k, v in KINDS:
        if k in name:
            return v
    return None


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kind(r.get("Kernel_Name") or r.get("Name") or "")
            if k is not None:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    return rows


def calls_of(rows):
    calls, cur = [], None
    for s, e, k in rows:
        if k == "init":
            cur = []
            calls.append(cur)
        elif k == "finish":
            cur = None
        elif cur is not None:
            cur.append((s, e, k))
    return calls


def analyse(call):
    steps, cur, pending_copy, prev_end = [], None, False, None
    for s, e, k in call:
        if k == "copy":
            pending_copy = True
            continue
        if k == "pred0":
            if cur is not None:
                steps.append(cur)
            cur = {"kern": 0.0, "intra": 0.0, "step": 0.0, "chunk": 0.0}
            if prev_end is not None:
                steps[-1]["chunk" if pending_copy else "step"] += (s - prev_end) / 1e3 if steps else 0.0
            pending_copy = False
        elif cur is not None and prev_end is not None:
            cur["intra"] += (s - prev_end) / 1e3
        if cur is not None:
            cur["kern"] += (e - s) / 1e3
        prev_end = e
    if cur is not None:
        steps.append(cur)
    return steps


def mean(part, key):
    return round(sum(x[key] for x in part) / len(part), 2) if part else None


def main():
    rows = load(sys.argv[1])
    out = []
    for i, c in enumerate(calls_of(rows)):
        st = analyse(c)
        if not st:
            continue
        rec = {"call": i, "steps": len(st)}
        for name, part in (("early", st[:-TAIL] if len(st) > TAIL else []), ("tail", st[-TAIL:])):
            rec[name] = {k: mean(part, k) for k in ("kern", "intra", "step", "chunk")}
            rec[name]["chunk_boundaries"] = sum(1 for x in part if x["chunk"] > 0)
            rec[name]["ms"] = round(sum(x["kern"] + x["intra"] + x["step"] + x["chunk"] for x in part) / 1e3, 3)
        out.append(rec)
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
