"""Where a persistent dataflow encode (lstm_i8_flow_kernel, encoder.hip) spends its time: config 3
(N=128, U{47..500}) on a -DRNNT_DEV_STAMPS build, one record per task (development tool).

    RNNT_MI355X_LIB=build_dev/lib_stamps.so python tools/flow_stamps.py

Per task (s_memrealtime, 100 MHz): dequeued, input frame ready (after its wait + acquire), first
stage landed, recurrent state ready (after its wait + acquire), main loop done, epilogue + copy-out
done.  Per layer: mean phase times; per layer-step chain: from the last task of step (l, t)
finishing to the first task of (l, t+1) seeing its state ready (the hand-off latency).
"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rnnt-inference_amd"))
import torch  # noqa: E402

from rnnt_amd import synthetic, weights  # noqa: E402
from rnnt_amd.engine import Engine, pad_batch  # noqa: E402


def step_layers(T):
    """(layer, frame) of each flow step, in the host's order (engine.hip run_flow; every step of
    config 3 has one batch tile)."""
    Tp = (T + 1) // 2
    out = []
    for tau in range(max(T + 1, 2 * Tp + 4)):
        jobs = []
        if tau < T:
            jobs.append((0, tau, 256))
        if 1 <= tau <= T:
            jobs.append((1, tau - 1, 1024))
        for l in range(2, 5):
            d = tau - (l + 1)
            if d >= 0 and d % 2 == 0 and d // 2 < Tp:
                jobs.append((l, d // 2, 2048 if l == 2 else 1024))
        jobs.sort(key=lambda j: -j[2])  # stable, like the host
        out += [(l, t) for l, t, _ in jobs]
    return out


def main():
    pm, _ = weights.build_model()
    n = 128
    n_pad = pad_batch(n)
    lens = np.sort(synthetic.uniform_lengths(n, seed=3))[::-1].astype(np.int32).copy()
    T = int(lens.max())
    e = Engine(pm, device=0, max_batch=n_pad, max_frames=T)
    e.set_tile("flow")
    lp = np.zeros(n_pad, np.int32)
    lp[:n] = lens
    x = torch.from_numpy(synthetic.make_features(T, n_pad, seed=3, lens=lp)).cuda()
    ld = torch.from_numpy(lp).cuda()
    res = torch.empty((n, e.max_res), dtype=torch.int32, device="cuda")
    rl = torch.empty(n, dtype=torch.int32, device="cuda")
    rd = e._lib.rnnt_dev_read_enc_stamps
    rd.restype = C.c_int
    rd.argtypes = [C.c_void_p, C.c_int]
    buf = np.zeros((1 << 18, 16), np.uint64)  # 16-word tile records (encoder.hip EST_W)
    for _ in range(2):
        e.infer(x, ld, lens, res, rl, n=n)
        torch.cuda.synchronize()
        k = rd(buf.ctypes.data, buf.shape[0])
    r = buf[:k].astype(np.int64)
    e.close()
    steps = step_layers(T)
    si = r[:, 1]
    deq, st0, lend, epi, xr, hr = r[:, 2], r[:, 3], r[:, 4], r[:, 5], r[:, 6], r[:, 7]
    t0 = deq.min()
    us = lambda v: v / 100.0  # noqa: E731  (100 MHz ticks -> us)
    out = {"tasks": int(k), "span_us": round(us(epi.max() - t0), 1), "steps": len(steps)}
    lay = np.array([steps[int(s)][0] for s in si])
    for l in range(5):
        m = lay == l
        if not m.any():
            continue
        hw = np.maximum(hr[m], xr[m])
        out[f"layer{l}"] = {
            "tasks": int(m.sum()),
            "deq_to_x_ready": round(us(np.mean(xr[m] - deq[m])), 2),
            "x_ready_to_stage0": round(us(np.mean(st0[m] - xr[m])), 2),
            "h_wait_after_x": round(us(np.mean(hr[m] - xr[m])), 2),
            "h_ready_to_loop_end": round(us(np.mean(lend[m] - hw)), 2),
            "epilogue": round(us(np.mean(epi[m] - lend[m])), 2),
            "task_total": round(us(np.mean(epi[m] - deq[m])), 2)}
    # hand-off chain of each layer: (l, t) all done -> (l, t+1) first sees its state ready
    done = {}
    first_h = {}
    for j in range(k):
        key = steps[int(si[j])]
        done[key] = max(done.get(key, 0), int(epi[j]))
        first_h[key] = min(first_h.get(key, 1 << 62), int(hr[j]))
    for l in range(5):
        gaps, per = [], []
        ts = sorted(t for (ll, t) in done if ll == l)
        for a, b in zip(ts, ts[1:]):
            gaps.append(first_h[(l, b)] - done[(l, a)])
            per.append(done[(l, b)] - done[(l, a)])
        if gaps:
            out[f"chain{l}"] = {"handoff_us": round(us(np.median(gaps)), 2), "step_us": round(us(np.median(per)), 2)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
