#!/usr/bin/env python3
"""MLPerf Server scenario on one MI355X (BASELINE config 5, per GPU): Poisson arrivals of
single-sample queries at a target QPS over a dev-clean-shaped QSL, served by
rnnt_amd.sut.ServerSUT (continuous batching: slots carrying LSTM / greedy state across split_len
chunks, refilled as samples finish -- the reference's PipelineState) or, with --mode dynamic,
DynamicBatchServerSUT (whole utterances, dynamic batches); reports latency percentiles
and, with --search, the largest QPS whose p99 latency meets the Server bound
(rnnt.Server.target_latency = 1000 ms, reference configs/mlperf.conf).

    python tools/server_bench.py --qps 20000 --duration 10 [--slots 4096 --split-len 128]
    python tools/server_bench.py --search [--mode dynamic]
Latency = completion (tokens on the host) - scheduled arrival time.  8 GPUs = 8 independent
processes (queries are dealt per GPU; no collective), so per-GPU QPS x 8 is the node figure.
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
from rnnt_amd.engine import Engine, cu_mask_words  # noqa: E402
from rnnt_amd.sut import DynamicBatchServerSUT, GpuQSL, GpuWavQSL, QuerySample, ServerSUT, WavFeed  # noqa: E402

TARGET_LATENCY_S = 1.0   # mlperf.conf rnnt.Server.target_latency (ms) / 1000
PERCENTILE = 99.0        # mlperf.conf *.Server.target_latency_percentile


def run_point(engines, qsl, qps, duration, max_batch, seed, args, feeds=None):
    if args.mode == "dynamic":
        sut = DynamicBatchServerSUT(engines, qsl, max_batch=max_batch)
    else:
        sut = ServerSUT(engines, None if feeds else qsl, slots=max_batch, split_len=args.split_len, qos_len=args.qos_len,
                        pipelined=args.pipelined, feeds=feeds,
                        engine_cu_mask=cu_mask_words(args.fz_cus) if feeds and args.fz_cus else None, refill=args.refill)
    sut.start()
    rng = np.random.default_rng(seed)
    n = max(1, int(qps * duration))
    arrivals = np.cumsum(rng.exponential(1.0 / qps, size=n))
    index = rng.integers(0, len(qsl), size=n)
    t0 = time.perf_counter()
    i = 0
    while i < n:
        now = time.perf_counter() - t0
        j = int(np.searchsorted(arrivals, now, side="right"))
        if j > i:
            for k in range(i, j):  # scheduled arrival time = the sample's issue timestamp
                sut.issue_query([QuerySample(id=k, index=int(index[k]))], now=t0 + arrivals[k])
            i = j
        else:
            time.sleep(min(0.0005, arrivals[i] - now))
    if hasattr(sut, "flush_queries"):
        sut.flush_queries()  # LoadGen's FlushQueries after the last issue: deferred QoS samples run
    deadline = time.perf_counter() + 60.0
    while len(sut.latency) < n and time.perf_counter() < deadline and not sut.errors:
        time.sleep(0.005)
    sut.stop()
    if sut.errors:
        raise sut.errors[0]
    lat = np.array([sut.latency.get(k, np.inf) for k in range(n)])
    span = time.perf_counter() - t0
    return dict(target_qps=qps, samples=n, achieved_qps=round(n / max(span, 1e-9), 1),
                rounds=getattr(sut, "rounds", None), batches=getattr(sut, "batches", None),
                p50_ms=round(float(np.percentile(lat, 50)) * 1e3, 2), p90_ms=round(float(np.percentile(lat, 90)) * 1e3, 2),
                p99_ms=round(float(np.percentile(lat, PERCENTILE)) * 1e3, 2),
                max_ms=round(float(lat.max()) * 1e3, 2), valid=bool(np.percentile(lat, PERCENTILE) <= TARGET_LATENCY_S))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qps", type=float, default=20000.0)
    ap.add_argument("--duration", type=float, default=10.0)
    ap.add_argument("--mode", choices=["continuous", "dynamic"], default="continuous")
    ap.add_argument("--max-batch", "--slots", type=int, default=4096, help="slots per engine (continuous) / max batch")
    ap.add_argument("--split-len", type=int, default=128,
                    help="continuous: frames per chunk (the reference's LEN; its CPU Server runs LEN=8, run.sh:74; "
                         "on the GPU 128-frame chunks measured best: 50k QPS p99 253 ms vs 32-frame chunks invalid)")
    ap.add_argument("--qos-len", type=int, default=None, help="continuous: defer samples longer than this (frames)")
    ap.add_argument("--inflight", type=int, default=4,
                    help="engines (continuous: 4096 slots each); 4 measured best valid 80k QPS target vs 70k with 2 "
                         "(profiles/r02z_server_search_continuous*.json)")
    ap.add_argument("--pipelined", action="store_true",
                    help="continuous: each engine encodes round k+1 while it decodes round k")
    ap.add_argument("--refill", choices=["fcfs", "tile"], default="fcfs",
                    help="continuous: free slots take the oldest samples (fcfs), or whole free 128-row tiles take "
                         "groups of similar lengths (tile)")
    ap.add_argument("--qsl", type=int, default=2513)
    ap.add_argument("--search", action="store_true", help="largest QPS with p99 <= 1000 ms")
    ap.add_argument("--burst", type=int, default=0,
                    help="capacity instead of latency: issue this many samples at once and report samples / s until "
                         "the last completes (the saturated throughput, free of the Poisson points' queueing noise)")
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--wav", action="store_true",
                    help="continuous, audio input (the reference's processor=true Server): --feeds WAV feeds, each "
                         "with its own audio copy and feature store, featurize arriving samples (ServerSUT feeds)")
    ap.add_argument("--feeds", type=int, default=2, help="--wav: producer lanes on the GPU (engines dealt round-robin)")
    ap.add_argument("--pro-batch", type=int, default=512,
                    help="--wav: at most this many queued samples featurized per launch (64: the producers fall "
                         "behind under load, 70k QPS target -> 39.5k completed; 512: 57k; profiles/r03/server_wav_*)")
    ap.add_argument("--fz-cus", type=int, default=0,
                    help="--wav: reserve this many CUs per XCD for the featurizer and keep the engines off them "
                         "(CU-masked streams); 0: shared CUs")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    pm, _ = weights.build_model()
    engines = [Engine(pm, device=0, max_batch=args.max_batch, max_frames=500) for _ in range(args.inflight)]
    feeds = None
    if args.wav:
        if args.mode != "continuous":
            raise SystemExit("--wav runs the continuous ServerSUT")
        frames = synthetic.devclean_lengths(args.qsl, seed=args.seed)
        wavs = synthetic.make_wavs(synthetic.wav_lengths_for_frames(frames, seed=args.seed), seed=args.seed,
                                   device="cuda")
        fz_mask = cu_mask_words(args.fz_cus, reserved=True) if args.fz_cus else None
        feeds = [WavFeed(GpuWavQSL(wavs), pro_batch=args.pro_batch, cu_mask=fz_mask) for _ in range(args.feeds)]
        del wavs
        qsl = feeds[0].qsl
    else:
        qsl = GpuQSL(synthetic.devclean_lengths(args.qsl, seed=args.seed), seed=args.seed)
    rp = lambda q, d, s: run_point(engines, qsl, q, d, args.max_batch, s, args, feeds)  # noqa: E731
    rp(2000.0, 1.0, 1)  # warm-up
    points = []
    if args.burst:
        rng = np.random.default_rng(args.seed)
        index = rng.integers(0, len(qsl.lengths), size=args.burst)
        sut = ServerSUT(engines, None if feeds else qsl, slots=args.max_batch, split_len=args.split_len,
                        qos_len=args.qos_len, pipelined=args.pipelined, feeds=feeds, refill=args.refill)
        sut.start()
        t0 = time.perf_counter()
        sut.issue_query([QuerySample(id=k, index=int(index[k])) for k in range(args.burst)], now=t0)
        sut.flush_queries()
        deadline = t0 + 300.0
        while len(sut.latency) < args.burst and time.perf_counter() < deadline and not sut.errors:
            time.sleep(0.005)
        span = time.perf_counter() - t0
        sut.stop()
        if sut.errors:
            raise sut.errors[0]
        frames = int(qsl.lengths[index].sum())
        print(json.dumps({"scenario": "Server capacity (burst)", "refill": args.refill, "samples": args.burst,
                          "seconds": round(span, 3), "samples_per_s": round(args.burst / span, 1),
                          "frames_per_s": round(frames / span, 1), "rounds": sut.rounds,
                          "stream_prefix": os.environ.get("RNNT_STREAM_PREFIX", "0")}), flush=True)
        for e in engines:
            e.close()
        return
    if not args.search:
        points.append(rp(args.qps, args.duration, args.seed))
    else:
        lo, hi, q = 0.0, None, 10000.0
        while hi is None and q < 1e6:
            p = rp(q, args.duration, args.seed)
            points.append(p)
            print(json.dumps(p), flush=True)
            if p["valid"]:
                lo, q = q, q * 2
            else:
                hi = q
        for _ in range(4 if hi else 0):
            q = 0.5 * (lo + hi)
            p = rp(q, args.duration, args.seed)
            points.append(p)
            print(json.dumps(p), flush=True)
            lo, hi = (q, hi) if p["valid"] else (lo, q)
    best = max((p for p in points if p["valid"]), key=lambda p: p["target_qps"], default=None)
    print(json.dumps({"scenario": "Server", "target_latency_ms": TARGET_LATENCY_S * 1e3, "percentile": PERCENTILE,
                      "duration_s": args.duration, "mode": args.mode, "slots_or_max_batch": args.max_batch,
                      "split_len": args.split_len if args.mode == "continuous" else None, "inflight": args.inflight,
                      "pipelined": args.pipelined, "input": (f"wav ({args.feeds} feeds, pro_batch {args.pro_batch}, featurizer CUs/XCD {args.fz_cus or 'shared'})"
                                                             if args.wav else "features (GpuQSL store)"),
                      "best_valid_qps_per_gpu": best["target_qps"] if best else None, "points": points}))
    for e in engines:
        e.close()


if __name__ == "__main__":
    main()
