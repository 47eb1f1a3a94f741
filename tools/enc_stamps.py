"""Per-tile timeline of the int8 tick kernel from in-kernel stamps (development tool).

    RNNT_MI355X_LIB=build_dev/lib_stamps.so python tools/enc_stamps.py [--n 8192] [--first 1] [--T 4]
Runs T layer-steps of one layer (op-level ABI, full batch) on a library built with
-DRNNT_DEV_STAMPS and splits every tile's time into: dispatch lag (the previous tile on the same
CU ended -> this workgroup started), prologue (start -> stage 0 landed), main loop (-> after
the last MFMA + cell-state DMA) and epilogue (-> copy-out issued).  Times in us (100 MHz
s_memrealtime).
"""
import argparse
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rnnt-inference_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rnnt_amd import weights  # noqa: E402
from rnnt_amd.engine import Engine, pad_batch  # noqa: E402


def pct(v, q):
    return round(float(np.percentile(v, q)), 2) if len(v) else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--first", type=int, default=1, help="0: K1280, 1: K2048, 2: K3072")
    ap.add_argument("--T", type=int, default=4)
    ap.add_argument("--encode", action="store_true",
                    help="time a whole dense encode (every tick carries all its layer-steps) instead of one layer")
    args = ap.parse_args()
    pm, _ = weights.build_model()
    n_pad = pad_batch(args.n)
    eng = Engine(pm, device=0, max_batch=n_pad, max_frames=64)
    rd = getattr(eng._lib, "rnnt_dev_read_enc_stamps", None)
    if rd is None:
        raise SystemExit("library built without -DRNNT_DEV_STAMPS")
    rd.argtypes = [C.c_void_p, C.c_int]
    rd.restype = C.c_int
    I = {0: 256, 1: 1024, 2: 2048}[args.first]
    T = args.T
    if args.encode:
        T = max(T, 16)
        feats = torch.randn((T, n_pad, 256), device="cuda")
        lens_h = np.full(args.n, T, np.int32)
        lens = torch.zeros(n_pad, dtype=torch.int32, device="cuda")
        lens[: args.n] = T
        run = lambda: eng.encode(feats, lens, lens_h, n=args.n)  # noqa: E731
    else:
        x = (torch.randn((T, n_pad, 256), device="cuda") if args.first == 0 else
             torch.randint(-128, 127, (T, n_pad, I), dtype=torch.int8, device="cuda"))
        hx = torch.zeros((1, n_pad, 1024), dtype=torch.int8, device="cuda")
        cx = torch.zeros((1, n_pad, 1024), dtype=torch.int16, device="cuda")
        y = torch.empty((T, n_pad, 1024), dtype=torch.int8, device="cuda")
        run = lambda: eng.lstm_int8(args.first, 1, x, hx, cx, y)  # noqa: E731
    run()  # warm
    torch.cuda.synchronize()
    rd(None, 0)
    run()
    torch.cuda.synchronize()
    W = 16  # words per tile record (encoder.hip EST_W)
    buf = np.zeros(W * (1 << 18), np.uint64)
    n = rd(C.c_void_p(buf.ctypes.data), len(buf) // W)
    r = buf[: W * n].reshape(n, W).astype(np.int64)
    # HW_ID bits 8-15 (cu_id, sh_id, se_id) + XCC_ID: one value per CU
    cu = ((r[:, 0] >> 40) & 0xFF) | ((r[:, 1] & 0xFF) << 8)
    clk = (r[:, 7] - r[:, 6]).astype(np.float64)  # shader clocks over the main loop (s_memtime)
    t0, t1, t2, t3 = r[:, 2], r[:, 3], r[:, 4], r[:, 5]
    order = np.argsort(t0)
    # launches: consecutive tiles whose start precedes the running max end belong together
    launch = np.zeros(n, np.int64)
    cur_end, lid = -1, -1
    for i in order:
        if t0[i] > cur_end:
            lid += 1
        launch[i] = lid
        cur_end = max(cur_end, t3[i])
    out = {"tiles": int(n), "launches": int(lid + 1), "K": int(r[0, 0] & 0xFFFF)}
    per = []
    lag = []
    util, gaps, prev_end = [], [], None
    for L in range(lid + 1):
        idx = np.where(launch == L)[0]
        s0, e1 = t0[idx].min(), t3[idx].max()
        per.append((e1 - s0) / 100.0)
        # CU occupancy inside the launch (tile time / (CUs x span)) and the gap since the last one
        util.append(float((t3[idx] - t0[idx]).sum()) / (256.0 * max(1, e1 - s0)))
        if prev_end is not None:
            gaps.append((s0 - prev_end) / 100.0)
        prev_end = e1
        # dispatch lag: tiles that started after another tile ended on the same CU slot
        for c in np.unique(cu[idx]):
            ii = idx[cu[idx] == c]
            ii = ii[np.argsort(t0[ii])]
            for a, b in zip(ii[:-1], ii[1:]):
                lag.append((t0[b] - t3[a]) / 100.0)
        first_round = idx[t0[idx] - s0 < 50]  # started within 0.5 us of the launch's first tile
        out.setdefault("first_round_tiles", []).append(int(len(first_round)))
    # position of each tile in its CU's sequence within the launch (0 = first)
    pos = np.zeros(n, np.int64)
    for L in range(lid + 1):
        idx = np.where(launch == L)[0]
        for c in np.unique(cu[idx]):
            ii = idx[cu[idx] == c]
            pos[ii[np.argsort(t0[ii])]] = np.arange(len(ii))
    pro, main_, epi = (t1 - t0) / 100.0, (t2 - t1) / 100.0, (t3 - t2) / 100.0
    for ps in (0, 1):
        m = pos == ps
        out[f"tile{ps}_prologue_main_epilogue_us_p50"] = [pct(pro[m], 50), pct(main_[m], 50), pct(epi[m], 50)]
    out.update({
        "launch_span_us_p50": pct(per, 50),
        "launch_cu_occupancy_p10_p50_p90": [pct(util, 10), pct(util, 50), pct(util, 90)],
        "gap_between_launches_us_p50": pct(gaps, 50) if gaps else None,
        "launch_span_us": [round(v, 1) for v in per[:8]],
        "prologue_us_p10_p50_p90": [pct(pro, 10), pct(pro, 50), pct(pro, 90)],
        "main_us_p10_p50_p90": [pct(main_, 10), pct(main_, 50), pct(main_, 90)],
        "epilogue_us_p10_p50_p90": [pct(epi, 10), pct(epi, 50), pct(epi, 90)],
        "tile_us_p10_p50_p90": [pct(t3 - t0, 10) / 100.0, pct(t3 - t0, 50) / 100.0, pct(t3 - t0, 90) / 100.0],
        "dispatch_lag_us_p10_p50_p90": [pct(lag, 10), pct(lag, 50), pct(lag, 90)],
        "main_loop_clock_ghz_p10_p50_p90": [pct(clk / (main_ * 1e3), 10), pct(clk / (main_ * 1e3), 50),
                                            pct(clk / (main_ * 1e3), 90)],
        # per stage, shader clocks: at the stage barrier (wait for the stage's DMA + the other waves)
        # and from the barrier to the end of the stage's MFMA issue (fragment waits + issue), wave 0
        "stage_clk_barrier_p50": pct(r[:, 8] / np.maximum(r[:, 10], 1), 50),
        "stage_clk_reads_mfma_issue_p50": pct(r[:, 9] / np.maximum(r[:, 10], 1), 50),
        "stage_clk_total_p50": pct(clk / np.maximum(r[:, 10], 1), 50),
        "tiles_per_cu_slot": int(np.bincount(np.unique(cu, return_inverse=True)[1]).max()),
        "cu_slots": int(len(np.unique(cu))),
    })
    print(json.dumps(out))


if __name__ == "__main__":
    main()
