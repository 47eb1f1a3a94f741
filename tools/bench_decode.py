"""Greedy-decode microbenchmark (development tool): encode each batch of the bench query
once, then time rnnt_engine_decode alone (it re-runs from the kept encoder output).

    RNNT_MI355X_LIB=build_dev/lib_<variant>.so python tools/bench_decode.py
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rnnt-inference_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from rnnt_amd import dist, weights  # noqa: E402
from rnnt_amd.engine import Engine, pad_batch  # noqa: E402
from rnnt_amd.sut import make_batches  # noqa: E402


def main():
    torch.cuda.set_device(0)
    pm, _ = weights.build_model()
    qsl = bench.build_qsl(2513, seed=4, device="cuda:0")
    bsz = int(os.environ.get("RNNT_BENCH_BATCH", "4096"))  # the bench's default batch
    ids, idx = dist.query_arrays(2513, 24576)
    batches = make_batches(qsl, ids, idx, bsz)
    eng = Engine(pm, device=0, max_batch=bsz, max_frames=500)
    out = {"lib": os.path.basename(os.environ.get("RNNT_MI355X_LIB", "default"))}
    tot = 0.0
    for i, (bids, bidx) in enumerate(batches):
        n = len(bids)
        b = qsl.batch_inputs(bidx, pad_batch(n), torch.device("cuda", 0))
        res = torch.empty((n, eng.max_res), dtype=torch.int32, device="cuda")
        rl = torch.empty(n, dtype=torch.int32, device="cuda")
        eng.encode_gather(b["store"], b["offsets"], b["lens"], b["lens_host"], b["T"], n, pad_batch(n))
        eng.decode(res, rl)
        torch.cuda.synchronize()
        eng.stats(reset=True)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            eng.decode(res, rl)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        st = eng.stats(reset=True)
        stamps = getattr(eng._lib, "rnnt_dev_read_stamps", None)
        if stamps is not None and i == 0:
            import ctypes as C
            import numpy as np
            stamps.restype = C.c_int
            stamps(None, 0)  # reset
            eng.decode(res, rl)
            torch.cuda.synchronize()
            buf = np.zeros((1 << 22) // 6 * 6, np.uint64)
            n = stamps(C.c_void_p(buf.ctypes.data), len(buf) // 6)
            rec = buf[: 6 * n].reshape(n, 6).astype(np.int64)
            names = {0: "pred0", 1: "pred1", 2: "g", 3: "joint"}
            summ = {}
            for kid, nm in names.items():
                r = rec[rec[:, 0] == kid]
                if len(r) == 0:
                    continue
                d = lambda a, b: np.round(np.percentile((r[:, b] - r[:, a]) * 0.01, [50, 90]), 2).tolist()
                summ[nm] = {"n": int(len(r)), "entries_us": d(2, 3), "staging_us": d(3, 4), "compute_us": d(4, 5),
                            "total_us": d(2, 5)}
            out["stamps_batch0_p50_p90"] = summ
        out[f"batch{i}"] = {"decode_ms": round(min(ts), 2), "steps": int(st["decode_steps"] // 3),
                            "emitted": int(rl.sum())}
        tot += min(ts)
    out["total_ms"] = round(tot, 2)
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
