#!/usr/bin/env python3
"""MLPerf-Offline-style throughput of the MI355X RNN-T engine (utterances/s).

Workload (BASELINE.json metric / config 4): LoadGen's Offline scenario.  Each GPU holds a
LibriSpeech-dev-clean-shaped QSL of 2513 synthetic utterances (mlperf.conf:13) and serves one
Offline query of --query samples (default 24576 = *.Offline.min_query_count, mlperf.conf:63;
LoadGen fills it by repeating the QSL), weak scaling: one process per GPU, each with its own
query, no data-path collective.  The SUT sorts the query longest-first (rnnt_qsl.cpp:104-133)
and runs it in batches of --batch through the int8 encoder + bf16 prediction/joint +
device-side greedy decode.  One step = one whole query, features already resident in HBM;
the host gather of each utterance's int32 tokens (QuerySamplesComplete payload) is inside
the timed region.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "rnnt-inference_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rnnt_amd import synthetic, weights  # noqa: E402
from rnnt_amd.config import encoder_frames, encoder_ops  # noqa: E402
from rnnt_amd.engine import Engine, PartitionedStream, cu_mask_words, pad_batch  # noqa: E402

METRIC = "MLPerf Offline utterances/sec at 1/2/4/8 MI355X; WER vs fp32 ref"
INT8_DENSE_PEAK_TOPS = 5000.0  # MI355X_MICROARCH.md: I8 MFMA = 2x the ~2.5 PF dense bf16 rate
BF16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA
DECODE_OPS_PER_STEP = 4_682_752  # (2*2*4P*2P + 2*J*(H+P) + 2*K*J) per frame or emitted symbol


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--qsl", type=int, default=2513, help="QSL utterances per GPU (mlperf.conf:13)")
    ap.add_argument("--query", type=int, default=24576, help="samples per Offline query per GPU (mlperf.conf:63)")
    ap.add_argument("--batch", type=int, default=8192, help="utterances per encode+decode call")
    ap.add_argument("--batch-sizes", default=None,
                    help="comma-separated batch sizes over the sorted query (the last repeats), e.g. 8192,8192,4096,2048")
    ap.add_argument("--inflight", type=int, default=3,
                    help="batches in flight per GPU: one engine + HIP stream + host thread each, so one "
                         "batch's latency-bound greedy decode overlaps the next batch's encoder")
    ap.add_argument("--decode-priority", type=int, default=0,
                    help="run each engine's decode on a separate stream of this priority (torch: lower = higher; "
                         "0 = decode on the encode stream)")
    ap.add_argument("--enc-concurrency", type=int, default=1,
                    help="encoders allowed on the GPU at once (1: encoders take turns, each batch's decode beside "
                         "the next encoder; 2+: the next encoder also fills the CUs a finishing encoder's short "
                         "length-sorted tail ticks leave idle)")
    ap.add_argument("--enc-reserve", type=int, default=0,
                    help="CUs per XCD kept off the encoder streams (CU-masked HIP streams, rnnt_stream_create); "
                         "each engine's decode then runs on its own unrestricted stream and always finds free CUs")
    ap.add_argument("--dec-cus", type=int, default=0,
                    help="CUs per XCD the decode streams may use (CU-masked; 0 = all): bounds how many CUs the "
                         "overlapped greedy decode takes from the encoder")
    ap.add_argument("--cpu-sample", type=int, default=256, help="utterances timed on the CPU restatement")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--wav", action="store_true",
                    help="WAV=true path (launch_sut.sh:53-55): the QSL holds 16 kHz audio and every batch runs the "
                         "GPU featurizer (FilterbankFeatures.forward) inside the timed region")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic_latest.json"),
                    help="per-launch HBM bytes from a rocprofv3 --pmc pass (profiles/), if present")
    return ap.parse_args()


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    return rank, local, world


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def all_max(x, world):
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def build_qsl(count, seed):
    """QSL: per-utterance features [T_i, 240] ~ N(0,1) (normalised log-mel stand-in), stored
    ragged in HBM (LoadSamplesToRam), lengths dev-clean-shaped."""
    lens = synthetic.devclean_lengths(count, seed=seed)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    feats = torch.randn((int(lens.sum()), 240), device="cuda", generator=g)
    return dict(lens=lens, offs=offs, feats=feats)


def build_wav_qsl(count, seed):
    """WAV QSL: speech-shaped synthetic 16 kHz audio stored ragged in HBM, with sample counts
    drawn so the feature lengths follow the same dev-clean shape as build_qsl."""
    lens = synthetic.devclean_lengths(count, seed=seed)
    wav_lens = synthetic.wav_lengths_for_frames(lens, seed=seed)
    store = torch.cat(synthetic.make_wavs(wav_lens, seed=seed, device="cuda"))
    offs = np.concatenate([[0], np.cumsum(wav_lens.astype(np.int64))[:-1]]).astype(np.int64)
    return dict(lens=lens, wav_lens=wav_lens, wav_offs=offs, store=store)


def batch_bounds(n, batch, sizes=None):
    """Start/end of each batch over the sorted query: --batch-sizes (cycled; the last entry
    repeats) or uniform --batch."""
    out, i, k = [], 0, 0
    while i < n:
        b = sizes[min(k, len(sizes) - 1)] if sizes else batch
        out.append((i, min(n, i + b)))
        i += b
        k += 1
    return out


def make_wav_batches(qsl, query, batch, sizes=None):
    """As make_batches, but each batch keeps only its samples' offsets into the ragged audio;
    its feature buffer [T_max, n_pad, 256] is filled by the featurizer inside every step."""
    count = len(qsl["lens"])
    ids = np.arange(query) % count
    ids = ids[np.argsort(-qsl["lens"][ids], kind="stable")]
    out = []
    for i, e in batch_bounds(len(ids), batch, sizes):
        idx = ids[i:e]
        n = len(idx)
        n_pad = pad_batch(n)
        bl = qsl["lens"][idx].astype(np.int32)
        wl = qsl["wav_lens"][idx].astype(np.int32)
        T = int(bl.max())
        out.append(dict(n=n, n_pad=n_pad, T=T, lens_host=bl, wav_lens_host=wl, idx=idx,
                        wav_lens=torch.from_numpy(wl).cuda(), wav_off=torch.from_numpy(qsl["wav_offs"][idx]).cuda(),
                        lens=torch.zeros(n_pad, dtype=torch.int32, device="cuda"),
                        x=torch.zeros((T, n_pad, 256), dtype=torch.float32, device="cuda")))
    torch.cuda.synchronize()
    return out


def make_batches(qsl, query, batch, sizes=None):
    """The Offline query (sample i -> QSL index i % count, as LoadGen repeats the QSL),
    sorted longest-first and split into batches; each batch assembled in HBM as
    [T_max, n_pad, 256] fp32, zero padded (AssembleSamples, rnnt_qsl.cpp:150-188)."""
    count = len(qsl["lens"])
    ids = np.arange(query) % count
    ids = ids[np.argsort(-qsl["lens"][ids], kind="stable")]
    out = []
    for i, e in batch_bounds(len(ids), batch, sizes):
        idx = ids[i:e]
        bl = qsl["lens"][idx].astype(np.int32)
        n = len(idx)
        n_pad = pad_batch(n)
        lp = np.zeros(n_pad, np.int32)
        lp[:n] = bl
        T = int(bl.max())
        t = torch.arange(T, device="cuda")[:, None]
        ln = torch.from_numpy(bl).cuda()[None, :]
        rows = torch.from_numpy(qsl["offs"][idx]).cuda()[None, :] + t
        valid = t < ln
        x = torch.zeros((T, n_pad, 256), dtype=torch.float32, device="cuda")
        x[:, :n, :240] = qsl["feats"][torch.where(valid, rows, 0)] * valid[..., None]
        out.append(dict(n=n, n_pad=n_pad, T=T, lens_host=bl, lens=torch.from_numpy(lp).cuda(), x=x, idx=idx))
    torch.cuda.synchronize()
    return out


def run_step(engines, streams, batches, featurizers=None, store=None, dec_streams=None, enc_concurrency=1):
    """One Offline query.  Batch i runs on engine i % inflight, each engine with its own HIP
    stream and host thread (ctypes releases the GIL).  Encoders take turns (a lock held until
    the encode has finished on the GPU), so each batch's latency-bound greedy decode overlaps
    the next batch's encoder instead of competing with another encoder.  Then the responses
    are gathered to the host."""
    import threading
    k = len(engines)
    enc_lock = threading.Semaphore(enc_concurrency)

    def worker(j):
        for b in batches[j::k]:
            if featurizers is not None:  # audio -> features on this batch's stream
                featurizers[j].featurize(store, b["wav_lens"], b["wav_lens_host"], n=b["n"], n_pad=b["n_pad"],
                                         T_out=b["T"], offsets=b["wav_off"], out=b["x"], feat_lens=b["lens"],
                                         stream=streams[j])
            ds = streams[j] if dec_streams is None else dec_streams[j]
            if ds is not streams[j]:
                streams[j].wait_stream(ds)  # the engine's previous decode has consumed its state
            with enc_lock:
                engines[j].encode(b["x"], b["lens"], b["lens_host"], n=b["n"], stream=streams[j])
                streams[j].synchronize()
            engines[j].decode(b["res"], b["rl"], stream=ds)

    if k == 1:
        worker(0)
    else:
        ths = [threading.Thread(target=worker, args=(j,)) for j in range(k)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
    for s in streams + (dec_streams or []):
        s.synchronize()
    # host gather of the responses: lengths, then each batch's used token columns
    lens = [b["rl"].cpu() for b in batches]
    toks = [b["res"][:, : max(1, int(l.max()))].cpu() for b, l in zip(batches, lens)]
    return lens, toks


def sample_timed_rows(batches, n_sample, inflight):
    """Rows of the timed query to re-check on the CPU: evenly spaced rows (first = longest,
    last = shortest) of the first batch each engine ran and of the query's last batch, so the
    sample spans every engine in flight and both ends of the length-sorted query."""
    picks = sorted(set(list(range(min(inflight, len(batches)))) + [len(batches) - 1]))
    per = max(2, -(-n_sample // len(picks)))
    out = []
    for b in picks:
        n = batches[b]["n"]
        rows = np.unique(np.linspace(0, n - 1, min(per, n)).round().astype(np.int64))
        out += [(b, int(r)) for r in rows]
    return out


def cpu_baseline(pm, qsl, batches, timed_lens, timed_toks, n_sample, inflight):
    """The C restatement (oracle/, TEST INFRASTRUCTURE) timed on this host's cores on a bounded
    sample of the timed query's own utterances, and the parity check of the tokens the GPU
    produced for those rows INSIDE the timed region (last timed step) against it."""
    from oracle import oracle
    picks = sample_timed_rows(batches, n_sample, inflight)
    order = sorted(range(len(picks)), key=lambda i: -int(batches[picks[i][0]]["lens_host"][picks[i][1]]))
    picks = [picks[i] for i in order]  # longest first, as the SUT sorts
    qidx = np.array([batches[b]["idx"][r] for b, r in picks], np.int64)
    sl = qsl["lens"][qidx].astype(np.int32)
    n = len(sl)
    T = int(sl.max())
    x = np.zeros((T, n, 256), np.float32)
    feats = qsl["feats"]
    for i, q in enumerate(qidx):
        o = int(qsl["offs"][q])
        x[: sl[i], i, :240] = feats[o: o + int(sl[i])].cpu().numpy()
    oracle.lib()
    t0 = time.perf_counter()
    f = oracle.encoder_i8(pm, x, sl)
    res, rl, _ = oracle.greedy_decode(pm, f, (sl + 1) // 2, max_res=(500 // 2) * 30)
    dt = time.perf_counter() - t0
    mism = 0
    gpu_res = np.full_like(res, -1)
    gpu_rl = np.zeros_like(rl)
    for i, (b, r) in enumerate(picks):
        gl = int(timed_lens[b][r])
        gpu_rl[i] = gl
        gpu_res[i, :gl] = timed_toks[b][r, :gl].numpy()
        if gl != int(rl[i]) or not np.array_equal(gpu_res[i, :gl], res[i, :gl]):
            mism += 1
    engines_hit = sorted({b % inflight for b, _ in picks})
    return dict(value=n / dt, seconds=dt, n=n, sl=sl, x=x, res=res, rl=rl, cores=oracle.lib().oracle_num_threads(),
                frames=int(sl.sum()), mismatches=mism, gpu_res=gpu_res, gpu_rl=gpu_rl, batches=sorted({b for b, _ in picks}), engines=engines_hit)


def wer_vs_fp32(n=256, seed=44):
    """BASELINE metric's second half ("WER vs fp32 ref"), measured on the well-conditioned
    planted model (rnnt_amd.planted: contractive encoder, confident joint -- the regime of a
    trained network; the random-init throughput model's decisions sit at bf16-rounding margins,
    see DESIGN.md section 2).  n dev-clean-shaped utterances of the planted task; hypothesis =
    the int8 encoder + bf16 decoder (the timed path's kernels), reference = the fp32 encoder +
    fp32 decoder, both on the GPU through GreedyDecoder; plus both against the planted truth."""
    from rnnt_amd import accuracy, planted
    from rnnt_amd.decoder import GreedyDecoder
    from rnnt_amd.model import RNNT
    ckpt, task = planted.make_planted_checkpoint()
    lens = synthetic.devclean_lengths(n, seed=seed)
    feats, truth = planted.planted_features(task, lens, seed=seed + 1)
    x = np.zeros((int(lens.max()), n, 240), np.float32)
    for i, fe in enumerate(feats):
        x[: len(fe), i] = fe
    amax = weights.calibrate_amax(weights.migrate_state_dict(ckpt), x[:, :8], lens[:8])
    xd, ld = torch.from_numpy(x).cuda(), torch.from_numpy(lens)
    hyp = {}
    for mode in ("quant", "f32"):
        m = RNNT(ckpt, mode, enable_bf16=(mode == "quant"), amax=amax)
        dec = GreedyDecoder(m, mode, mode == "quant", batch_size=n, device=torch.cuda.current_device())
        res, rl = dec(xd, ld)
        res, rl = res.cpu().numpy(), rl.cpu().numpy()
        hyp[mode] = [accuracy.seq_to_sen(res[i], rl[i]) for i in range(n)]
        dec.close()
    ref = ["".join(accuracy.LABELS[c] for c in t) for t in truth]

    def w(h, r):
        wer, errs, words = accuracy.word_error_rate(h, r)
        return {"wer": round(wer, 5), "word_errors": errs, "words": words}

    return {"utterances": n, "model": "planted (well-conditioned) RNN-T, rnnt_amd/planted.py",
            "int8_bf16_vs_fp32": w(hyp["quant"], hyp["f32"]),
            "fp32_vs_planted_truth": w(hyp["f32"], ref), "int8_bf16_vs_planted_truth": w(hyp["quant"], ref),
            "target": "int8_bf16_vs_fp32 WER <= 0.01 (north_star)",
            "hypothesis": "int8 encoder + bf16 prediction/joint (GPU)", "reference": "fp32 encoder + fp32 decoder (GPU)",
            "note": "synthetic planted task (no checkpoint / LibriSpeech offline); teacher-forced joint-logit tolerance "
                    "on both models: tests/test_accuracy_gpu.py"}


def main():
    args = parse()
    rank, local, world = dist_setup()
    pm, _ = weights.build_model()
    qsl = (build_wav_qsl if args.wav else build_qsl)(args.qsl, seed=4 + 1000 * rank)
    lens = qsl["lens"]
    sizes = [int(v) for v in args.batch_sizes.split(",")] if args.batch_sizes else None
    engines = [Engine(pm, device=local, max_batch=min(max(sizes or [args.batch]), args.query), max_frames=500)
               for _ in range(args.inflight)]
    engine = engines[0]
    owned = []
    if args.dec_cus:
        owned = [PartitionedStream(local, cu_mask_words(args.dec_cus, reserved=True)) for _ in engines]
        streams = [torch.cuda.Stream() for _ in engines]
        dec_streams = [p.stream for p in owned]
    elif args.enc_reserve:
        owned = [PartitionedStream(local, cu_mask_words(args.enc_reserve)) for _ in engines]
        owned += [PartitionedStream(local) for _ in engines]
        streams = [p.stream for p in owned[: len(engines)]]
        dec_streams = [p.stream for p in owned[len(engines):]]
    else:
        streams = [torch.cuda.Stream() for _ in engines]
        dec_streams = ([torch.cuda.Stream(priority=args.decode_priority) for _ in engines] if args.decode_priority
                       else None)
    iso_stream = torch.cuda.Stream()
    batches = (make_wav_batches if args.wav else make_batches)(qsl, args.query, args.batch, sizes)
    fzs, store = None, None
    if args.wav:
        from rnnt_amd.featurizer import FilterbankFeatures
        fzs = [FilterbankFeatures(sample_rate=16000, window="hann", n_fft=512, nfilt=80, frame_splicing=3,
                                  pad_out_feat=True, device=local) for _ in engines]
        store = qsl["store"]
    for b in batches:  # response buffers, allocated once (the engine fills them every call)
        b["res"] = torch.empty((b["n"], engine.max_res), dtype=torch.int32, device="cuda")
        b["rl"] = torch.empty(b["n"], dtype=torch.int32, device="cuda")

    for _ in range(args.warmup):
        run_step(engines, streams, batches, fzs, store, dec_streams, args.enc_concurrency)
    torch.cuda.synchronize()
    for e in engines:  # HIP events around every encode / joint_trans / greedy call, on its stream
        e.set_profiling(True)
        e.stats(reset=True)
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        lens_out, toks_out = run_step(engines, streams, batches, fzs, store, dec_streams, args.enc_concurrency)
    torch.cuda.synchronize()
    barrier(world)
    elapsed = time.perf_counter() - t0
    elapsed_max = all_max(elapsed, world)
    sts = [e.stats(reset=True) for e in engines]
    st = {k: sum(x[k] for x in sts) for k in sts[0]}
    # isolated pass (untimed): the same query once more, batches back to back on one engine,
    # so the encoder's event time is not shared with an overlapping decode
    run_step([engine], [iso_stream], batches)
    iso = engine.stats(reset=True)
    for e in engines:
        e.set_profiling(False)
    utts = args.query * world * args.steps
    value = utts / elapsed_max
    emitted = int(sum(int(l.sum()) for l in lens_out))
    qlens = np.concatenate([b["lens_host"] for b in batches])
    enc_frames = int(sum(encoder_frames(l) for l in qlens))
    enc_ops = float(sum(encoder_ops(int(l)) for l in qlens))  # SURVEY 8d E(T), valid frames, one query
    achieved = enc_ops * args.steps / (st["encode_ms"] * 1e-3) / 1e12 if st["encode_ms"] > 0 else 0.0
    achieved_iso = enc_ops / (iso["encode_ms"] * 1e-3) / 1e12 if iso["encode_ms"] > 0 else 0.0
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            traffic = json.load(open(args.traffic_json)).get("lstm_i8_step_bytes_per_launch")
        except Exception:
            traffic = None
    # decode work: D = (T' + U) * 4,682,752 bf16 ops per utterance, summed over the query
    dec_ops = float(enc_frames + emitted) * DECODE_OPS_PER_STEP
    dec_ms = (st["greedy_ms"] + st["joint_trans_ms"]) / args.steps
    dec_ms_iso = iso["greedy_ms"] + iso["joint_trans_ms"]
    dec_ach = dec_ops / (dec_ms * 1e-3) / 1e12 if dec_ms > 0 else 0.0
    dec_ach_iso = dec_ops / (dec_ms_iso * 1e-3) / 1e12 if dec_ms_iso > 0 else 0.0
    ticks_q = st["step_launches"] / args.steps
    roofline = {
        "bound": "mfma", "kernel": "lstm_i8_tick_kernel (int8 encoder, up to 5 layer-steps per launch)",
        "achieved": round(achieved, 2), "peak": INT8_DENSE_PEAK_TOPS, "unit": "TFLOP/s",
        "frac": round(achieved / INT8_DENSE_PEAK_TOPS, 4), "traffic": traffic,
        "measured_on": "HIP events around every encode call on its own stream, timed region (encode overlaps "
                       "other batches' decode)",
        "encode_ms_per_query": round(st["encode_ms"] / args.steps, 3),
        "joint_trans_ms_per_query": round(st["joint_trans_ms"] / args.steps, 3),
        "greedy_ms_per_query": round(st["greedy_ms"] / args.steps, 3),
        "tick_launches_per_query": int(st["step_launches"] // args.steps),
        "encode_us_per_tick_events": round(st["encode_ms"] / args.steps / ticks_q * 1e3, 2) if ticks_q else None,
        "encode_us_per_tick_note": "event time per encode call / tick launches (includes the quantize kernel and "
                                   "the gaps between ticks; rocprofv3 kernel stats give the kernel alone)",
        "decode": {"kernels": "joint_trans_gemm_kernel + dec_pred/g/joint step kernels (bf16 MFMA)",
                   "ops_per_query": dec_ops, "achieved": round(dec_ach, 2), "peak": BF16_DENSE_PEAK_TFLOPS,
                   "unit": "TFLOP/s", "frac": round(dec_ach / BF16_DENSE_PEAK_TFLOPS, 4),
                   "isolated_achieved": round(dec_ach_iso, 2),
                   "isolated_frac": round(dec_ach_iso / BF16_DENSE_PEAK_TFLOPS, 4),
                   "note": "latency-bound lock-step greedy loop; time = joint_trans + greedy event time"},
        "isolated": {"achieved": round(achieved_iso, 2), "frac": round(achieved_iso / INT8_DENSE_PEAK_TOPS, 4),
                     "encode_ms_per_query": round(iso["encode_ms"], 3),
                     "greedy_ms_per_query": round(iso["greedy_ms"], 3),
                     "note": "untimed pass, batches back to back on one engine (no overlap)"},
    }
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "utterances/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed_max / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int8",
        "data": ("synthetic (seeded dev-clean-shaped speech-like 16 kHz audio, random-init RNN-T weights)" if args.wav
                 else "synthetic (seeded dev-clean-shaped lengths, N(0,1) features, random-init RNN-T weights)"),
        "config": {"workload": "MLPerf Offline query over a LibriSpeech-dev-clean-shaped QSL (BASELINE config 4)",
                   "qsl_per_gpu": args.qsl, "query_samples_per_gpu": args.query, "batch_size": args.batch,
                   "batches_in_flight": args.inflight, "encoder_concurrency": args.enc_concurrency,
                   "encoder_cu_reserve_per_xcd": args.enc_reserve, "decode_cus_per_xcd": args.dec_cus or 32,
                   "input": ("16 kHz audio: GPU featurizer (FilterbankFeatures.forward) in the timed region" if args.wav
                             else "log-mel features resident in HBM"),
                   "encoder": "int8 (lstm_amx_int8)",
                   "decoder": "bf16 prediction/joint, fp32 accumulate, greedy (device loop)",
                   "parallelism": f"dp{world} (one process per GPU, sharded queries)",
                   "encoder_frames_per_query": enc_frames, "emitted_symbols_per_query": emitted},
        "roofline": roofline,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.wav:
        cb = cpu_baseline(pm, qsl, batches, lens_out, toks_out, args.cpu_sample, args.inflight)
        out["cpu_baseline"] = {"value": round(cb["value"], 3), "unit": "utterances/s", "cores": cb["cores"],
                               "kind": "port",
                               "sample": f"{cb['n']} utterances ({cb['frames']} frames) of the timed query (batches "
                                         f"{cb['batches']}, longest to shortest rows), int8 encoder + greedy decode, "
                                         f"{cb['seconds']:.1f} s"}
        out["parity_spot_check"] = {"utterances": cb["n"], "source": "token rows produced inside the last timed step",
                                    "batches": cb["batches"], "engines": cb["engines"],
                                    "mismatched_rows": cb["mismatches"], "tokens_identical": cb["mismatches"] == 0}
        out["wer_vs_fp32"] = wer_vs_fp32()
    if rank == 0:
        print(json.dumps(out), flush=True)
    for e in engines:
        e.close()
    for p in owned:
        p.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
