"""Throughput of BASELINE configs 2 and 3 on one MI355X (measurement tool; the bench contract's
line is config 4, `bench.py`).

    python tools/bench_configs.py [--reps 5]
config 2: fp32 encoder LSTM stack only, N=32 synthetic 15 s utterances (T=500 feature frames),
          the f32 path (encoder_f32.hip) -> utt/s and the fraction of the fp32 MFMA peak
          (157.3 TF, MI355X_MICROARCH.md) for SURVEY 8d's encoder work E(T).
config 3: int8 encoder + bf16 prediction/joint greedy decode, N=128, lengths U{47..500}
          sorted descending (the GPU parity test's shape) -> utt/s, encode/decode split.
Random-init weights (synthetic checkpoint), synthetic N(0,1) features; one JSON line.
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

FP32_MFMA_PEAK_TF = 157.3


def enc_ops(T):
    return 27_131_904 * T + 58_720_256 * ((T + 1) // 2)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return min(ts), float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--concurrent", type=int, default=8,
                    help="config 3 also with this many 128-row batches in flight (one engine, HIP stream and host "
                         "thread each, like the reference's concurrent SUT instances); 0: skip")
    ap.add_argument("--tiles", default="auto",
                    help="config 3 encoder settings to time, comma-separated (rnnt_engine_set_tile: auto, ticks = "
                         "one launch per tick, flow = the persistent dataflow launch); tokens must agree")
    ap.add_argument("--skip-config2", action="store_true")
    args = ap.parse_args()
    pm, ckpt = weights.build_model()
    out = {}
    # ---- config 2: fp32 encoder, N=32, T=500
    if not args.skip_config2:
        config2(pm, ckpt, args, out)
    config3(pm, args, out)
    if args.concurrent > 0:
        out["config3_int8_full_n128_concurrent"] = concurrent_config3(pm, args.concurrent, args.reps)
    print(json.dumps(out))


def config2(pm, ckpt, args, out):
    sd = weights.migrate_state_dict(ckpt)
    n, T = 32, 500
    n_pad = pad_batch(n)
    e = Engine(pm, device=0, max_batch=n_pad, max_frames=T)
    e.load_f32_encoder([weights.enc_layer_params(sd, l) for l in range(5)])
    lens = np.full(n, T, np.int32)
    lp = np.zeros(n_pad, np.int32)
    lp[:n] = lens
    x = torch.from_numpy(synthetic.make_features(T, n_pad, seed=21, lens=lp)).cuda()
    ld = torch.from_numpy(lp).cuda()
    f = torch.empty(((T + 1) // 2, n_pad, 1024), dtype=torch.float32, device="cuda")
    best, med = timed(lambda: e.encode_f32(x, ld, n, f), args.reps)
    tf = n * enc_ops(T) / best / 1e12
    out["config2_fp32_encoder_n32_T500"] = {"utt_per_s": round(n / best, 1), "ms_per_batch": round(best * 1e3, 2),
                                           "ms_median": round(med * 1e3, 2), "achieved_tflops": round(tf, 2),
                                           "frac_fp32_mfma_peak": round(tf / FP32_MFMA_PEAK_TF, 4)}
    e.close()


def config3(pm, args, out):
    """int8 enc + bf16 pred/joint greedy, N=128, U{47..500}, under each --tiles setting."""
    n = 128
    n_pad = pad_batch(n)
    lens = np.sort(synthetic.uniform_lengths(n, seed=3))[::-1].astype(np.int32).copy()
    T = int(lens.max())
    e = Engine(pm, device=0, max_batch=n_pad, max_frames=T)
    lp = np.zeros(n_pad, np.int32)
    lp[:n] = lens
    x = torch.from_numpy(synthetic.make_features(T, n_pad, seed=3, lens=lp)).cuda()
    ld = torch.from_numpy(lp).cuda()
    res = torch.empty((n, e.max_res), dtype=torch.int32, device="cuda")
    rl = torch.empty(n, dtype=torch.int32, device="cuda")
    ref = None
    for tile in args.tiles.split(","):
        e.set_tile(tile)
        best, med = timed(lambda: e.infer(x, ld, lens, res, rl, n=n), args.reps)
        e.set_profiling(True)
        e.stats(reset=True)
        encs = []
        for _ in range(max(3, args.reps)):  # encode time: the best of a few profiled passes
            e.infer(x, ld, lens, res, rl, n=n)
            torch.cuda.synchronize()
            encs.append(e.stats(reset=True))
        e.set_profiling(False)
        st = min(encs, key=lambda d: d["encode_ms"])
        ops = float(sum(enc_ops(int(t)) for t in lens))
        toks = (res.cpu().numpy().copy(), rl.cpu().numpy().copy())
        if ref is None:
            ref = toks
        same = bool(np.array_equal(ref[0], toks[0]) and np.array_equal(ref[1], toks[1]))
        key = "config3_int8_full_n128" + ("" if tile == "auto" else "_" + tile)
        out[key] = {"utt_per_s": round(n / best, 1), "ms_per_batch": round(best * 1e3, 2),
                    "ms_median": round(med * 1e3, 2), "encode_ms": round(st["encode_ms"], 3),
                    "joint_trans_ms": round(st["joint_trans_ms"], 3), "greedy_ms": round(st["greedy_ms"], 3),
                    "encoder_int8_frac": round(ops / (st["encode_ms"] * 1e-3) / 5e15, 4),
                    "emitted": int(toks[1].sum()), "tokens_equal_first_setting": same}
    e.close()


def concurrent_config3(pm, k, reps):
    """k config-3 batches (N=128, U{47..500}, their own features) in flight on one GPU: one engine,
    stream and host thread each, every engine running its batch reps times; tokens checked against
    the same batch run alone first."""
    import threading
    n = 128
    n_pad = pad_batch(n)
    lens = np.sort(synthetic.uniform_lengths(n, seed=3))[::-1].astype(np.int32).copy()
    T = int(lens.max())
    lp = np.zeros(n_pad, np.int32)
    lp[:n] = lens
    ld = torch.from_numpy(lp).cuda()
    engs, xs, ress, rls, refs = [], [], [], [], []
    for i in range(k):
        e = Engine(pm, device=0, max_batch=n_pad, max_frames=T)
        x = torch.from_numpy(synthetic.make_features(T, n_pad, seed=100 + i, lens=lp)).cuda()
        res = torch.empty((n, e.max_res), dtype=torch.int32, device="cuda")
        rl = torch.empty(n, dtype=torch.int32, device="cuda")
        e.infer(x, ld, lens, res, rl, n=n)  # alone: the reference answer (and warm-up)
        torch.cuda.synchronize()
        refs.append((res.cpu().numpy().copy(), rl.cpu().numpy().copy()))
        engs.append(e)
        xs.append(x)
        ress.append(res)
        rls.append(rl)
    streams = [torch.cuda.Stream() for _ in range(k)]
    start = threading.Barrier(k + 1)

    def worker(i):
        with torch.cuda.stream(streams[i]):
            start.wait()
            for _ in range(reps):
                engs[i].infer(xs[i], ld, lens, ress[i], rls[i], n=n, stream=streams[i])
            streams[i].synchronize()

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(k)]
    for t in ths:
        t.start()
    torch.cuda.synchronize()
    start.wait()
    t0 = time.perf_counter()
    for t in ths:
        t.join()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    same = all(np.array_equal(ress[i].cpu().numpy(), refs[i][0]) and np.array_equal(rls[i].cpu().numpy(), refs[i][1])
               for i in range(k))
    ops = float(sum(enc_ops(int(t)) for t in lens)) * k * reps
    for e in engs:
        e.close()
    return {"batches_in_flight": k, "reps_per_batch": reps, "utt_per_s": round(k * n * reps / wall, 1),
            "wall_ms": round(wall * 1e3, 2), "int8_encoder_work_per_wall_frac": round(ops / wall / 5e15, 4),
            "tokens_equal_alone_run": bool(same),
            "note": "chip-level rate: encoder int8 work over wall time while the batches' decodes share the GPU"}


if __name__ == "__main__":
    main()
