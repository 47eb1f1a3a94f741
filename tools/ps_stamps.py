"""Where a persistent decode step's time goes (development tool; needs a stamps build:
tools/build_variants.sh "stamps:-DRNNT_DEV_STAMPS", then RNNT_MI355X_LIB=build_dev/lib_stamps.so).

Decodes BATCH-row batches of the bench query with the persistent tail from step 32 on
(RNNT_DEC_PERSIST_ROWS, default 64) and reads the per-step records ps_loop writes (role, workgroup,
step: ready / body end / stores drained / published, s_memrealtime at 100 MHz).  Per phase and step:
  handoff  = the phase's first workgroup ready - the previous phase's last publish
  body     = the phase's last body end - its first ready
  drain    = last drained - last body end (write-through stores landing)
Printed as medians / p90 over the steps of all batches, in microseconds.
"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rnnt-inference_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from rnnt_amd import dist, weights  # noqa: E402
from rnnt_amd.engine import Engine, pad_batch  # noqa: E402
from rnnt_amd.sut import make_batches  # noqa: E402

ROLES = ["pred0", "pred1", "g", "joint"]


def analyse(rec):
    """rec: [n, 6] int64 records of kid 16..19 -> per (phase, step) timings."""
    out = {f"{r}_{m}": [] for r in ROLES for m in ("handoff", "body", "drain")}
    kid, k = rec[:, 0] - 16, rec[:, 1] >> 16
    steps = np.unique(k)
    agg = {}
    for r in range(4):
        for s in steps:
            m = (kid == r) & (k == s)
            if m.any():
                x = rec[m]
                agg[r, s] = (x[:, 2].min(), x[:, 3].max(), x[:, 4].max(), x[:, 5].max())
    for (r, s), (ready, bend, drained, pub) in agg.items():
        prev = agg.get((r - 1, s)) if r > 0 else agg.get((3, s - 1))
        if prev is not None:
            out[f"{ROLES[r]}_handoff"].append((ready - prev[3]) * 0.01)
        out[f"{ROLES[r]}_body"].append((bend - ready) * 0.01)
        out[f"{ROLES[r]}_drain"].append((drained - bend) * 0.01)
    step_t = [(agg[3, s][3] - agg[3, s - 1][3]) * 0.01 for s in steps if (3, s) in agg and (3, s - 1) in agg]
    res = {key: {"n": len(v), "p50": round(float(np.median(v)), 2), "p90": round(float(np.percentile(v, 90)), 2)}
           for key, v in out.items() if v}
    res["step_us"] = {"n": len(step_t), "p50": round(float(np.median(step_t)), 2),
                      "p90": round(float(np.percentile(step_t, 90)), 2)}
    return res


def main():
    torch.cuda.set_device(0)
    pm, _ = weights.build_model()
    qsl = bench.build_qsl(2513, seed=4, device="cuda:0")
    bsz = int(os.environ.get("BATCH", "64"))
    ids, idx = dist.query_arrays(2513, 24576)
    batches = make_batches(qsl, ids, idx, bsz)[: int(os.environ.get("NBATCH", "24"))]
    eng = Engine(pm, device=0, max_batch=bsz, max_frames=500)
    eng.set_decode_persist(int(os.environ.get("RNNT_DEC_PERSIST_ROWS", "64")))
    stamps = eng._lib.rnnt_dev_read_stamps
    stamps.restype = C.c_int
    buf = np.zeros((1 << 22) // 6 * 6, np.uint64)
    recs = []
    for bids, bidx in batches:
        n = len(bids)
        b = qsl.batch_inputs(bidx, pad_batch(n), torch.device("cuda", 0))
        res = torch.empty((n, eng.max_res), dtype=torch.int32, device="cuda")
        rl = torch.empty(n, dtype=torch.int32, device="cuda")
        eng.encode_gather(b["store"], b["offsets"], b["lens"], b["lens_host"], b["T"], n, pad_batch(n))
        eng.decode(res, rl)
        torch.cuda.synchronize()
        stamps(None, 0)
        eng.decode(res, rl)
        torch.cuda.synchronize()
        m = stamps(C.c_void_p(buf.ctypes.data), len(buf) // 6)
        rec = buf[: 6 * m].reshape(m, 6).astype(np.int64)
        rec = rec[rec[:, 0] >= 16]
        if len(rec):
            # steps of different batches must not mix: offset the step field per batch
            rec[:, 1] += (len(recs) * 100000) << 16
            recs.append(rec)
    rec = np.concatenate(recs)
    print(json.dumps({"batch": bsz, "batches": len(recs), "records": int(len(rec)), **analyse(rec)}, indent=1))
    eng.close()


if __name__ == "__main__":
    main()
