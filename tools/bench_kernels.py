"""Kernel-level microbenchmarks of the HIP engine (development tool, not the bench contract).

    python tools/bench_kernels.py [--n 1024] [--T 32]
Times the int8 LSTM step kernel per layer width (full batch, no tile skipping) through the
op-level C ABI, and one full encode+decode of a dev-clean-shaped batch with the engine's
event stats.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rnnt-inference_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rnnt_amd import synthetic, weights  # noqa: E402
from rnnt_amd.engine import Engine, pad_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--T", type=int, default=32)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--skip-decode", action="store_true")
    ap.add_argument("--layers", default="1,2,0", help="first-layer ids to time (0: K1280, 1: K2048, 2: K3072)")
    args = ap.parse_args()
    pm, _ = weights.build_model()
    n_pad = pad_batch(args.n)
    eng = Engine(pm, device=0, max_batch=n_pad, max_frames=500)
    out = {}
    T = args.T
    widths = {0: 256, 1: 1024, 2: 2048}
    for first in [int(v) for v in args.layers.split(",") if v != ""]:
        I = widths[first]
        if first == 0:
            x = torch.randn((T, n_pad, 256), device="cuda")
        else:
            x = torch.randint(-128, 127, (T, n_pad, I), dtype=torch.int8, device="cuda")
        hx = torch.zeros((1, n_pad, 1024), dtype=torch.int8, device="cuda")
        cx = torch.zeros((1, n_pad, 1024), dtype=torch.int16, device="cuda")
        y = torch.empty((T, n_pad, 1024), dtype=torch.int8, device="cuda")
        eng.lstm_int8(first, 1, x, hx, cx, y)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            eng.lstm_int8(first, 1, x, hx, cx, y)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / T)
        K = I + 1024
        ms = min(ts)
        tops = 2 * 4096 * K * n_pad / (ms * 1e-3) / 1e12
        out[f"step_K{K}"] = {"us_per_launch": round(ms * 1e3, 2), "TOPS": round(tops, 1)}
    if not args.skip_decode:
        lens = np.sort(synthetic.devclean_lengths(args.n, seed=4))[::-1].astype(np.int32)
        lp = np.zeros(n_pad, np.int32)
        lp[: args.n] = lens
        Tm = int(lens.max())
        x = torch.from_numpy(synthetic.make_features(Tm, n_pad, seed=5, lens=lp)).cuda()
        ld = torch.from_numpy(lp).cuda()
        res = torch.empty((args.n, eng.max_res), dtype=torch.int32, device="cuda")
        rl = torch.empty(args.n, dtype=torch.int32, device="cuda")
        eng.infer(x, ld, lens, res, rl, n=args.n)
        torch.cuda.synchronize()
        eng.set_profiling(True)
        eng.stats(reset=True)
        t0 = time.perf_counter()
        eng.infer(x, ld, lens, res, rl, n=args.n)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        st = eng.stats(reset=True)
        U = rl.cpu().numpy().astype(np.int64)
        Tp = (lens.astype(np.int64) + 1) // 2
        out["infer_batch"] = {"n": args.n, "wall_ms": round(wall * 1e3, 2), **{k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.items()},
                              "emitted": int(U.sum()),
                              "U_pct": [int(np.percentile(U, p)) for p in (50, 90, 99, 100)],
                              "Tp_pct": [int(np.percentile(Tp, p)) for p in (50, 90, 99, 100)],
                              "TpU_max": int((Tp + U).max()), "U_over_Tp_max": round(float((U / Tp).max()), 2),
                              "top_U_rows": [[int(U[i]), int(Tp[i])] for i in np.argsort(-U)[:8]]}
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
