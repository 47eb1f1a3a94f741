#!/usr/bin/env python3
"""MLPerf-Offline-style throughput of the MI355X RNN-T engine (utterances/s).

Workload (BASELINE.json metric / config 4): LoadGen's Offline scenario over a
LibriSpeech-dev-clean-shaped QSL of 2513 synthetic utterances (mlperf.conf:13), features resident
in HBM on every GPU.  One step = one Offline query of --query samples per GPU (default 300000 =
the reference's own Offline.min_query_count, configs/user.conf:6, which launch_sut.sh:46 passes to
LoadGen; mlperf.conf:63's rule minimum is 24576; LoadGen repeats the QSL), issued exactly as the
SUT serves it, all inside the timed region:
  * sort the query longest first (rnnt_qsl.cpp:104-133) and split it into batches of --batch;
    with several ranks (one process per GPU) every rank claims the next batch from one shared
    counter whenever its encoder is free (rnnt_amd.dist.BatchClaim; --deal static: snake deal);
  * per rank, rnnt_amd.sut.OfflineSUT: --inflight engines, one host thread + HIP stream each,
    pulling batches from a shared list; per batch AssembleSamples fused into the int8 encoder's
    quantize pass (gathered straight from the ragged QSL store), the wavefront-tick int8 encoder,
    bf16 prediction/joint + device-side greedy decode, and the D2H copy of the token rows
    (QuerySamplesComplete payloads);
  * the responses of all ranks streamed to rank 0's host per completed batch (rnnt_amd.dist.ResponseStream).
Weak scaling: the query grows with the GPU count (--query per GPU), one query served by all.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
``--gpus N`` without a torchrun environment starts the N ranks itself (torch.distributed.run as a
child process, before anything touches HIP), so both command lines measure N GPUs.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "rnnt-inference_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rnnt_amd import dist, synthetic, weights  # noqa: E402
from rnnt_amd.config import encoder_frames, encoder_ops  # noqa: E402
from rnnt_amd.engine import Engine  # noqa: E402
from rnnt_amd.sut import GpuQSL, GpuWavQSL, OfflineSUT, make_batches  # noqa: E402

METRIC = "MLPerf Offline utterances/sec at 1/2/4/8 MI355X; WER vs fp32 ref"
INT8_DENSE_PEAK_TOPS = 5000.0  # MI355X_MICROARCH.md: I8 MFMA = 2x the ~2.5 PF dense bf16 rate
BF16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA
DECODE_OPS_PER_STEP = 4_682_752  # (2*2*4P*2P + 2*J*(H+P) + 2*K*J) per frame or emitted symbol


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--qsl", type=int, default=2513, help="QSL utterances (mlperf.conf:13)")
    ap.add_argument("--query", type=int, default=300000,
                    help="Offline query samples per GPU (default: the reference's user.conf:6 Offline.min_query_count; "
                         "mlperf.conf:63's rule minimum is 24576)")
    ap.add_argument("--batch", type=int, default=6144,
                    help="utterances per encode+decode call (300000-sample query, 4 in flight, one box: 6144 "
                         "123.1-124.9k utt/s, 4096 121.4-122.6k, 8192 x 3 122.0-123.3k, 8192 x 2 105.5k: with two "
                         "engines the encoder waits for a free one; MEASUREMENTS.md section 8)")
    ap.add_argument("--inflight", type=int, default=4,
                    help="engines per GPU (one HIP stream + host thread each): one batch's latency-bound greedy "
                         "decode overlaps the next batch's encoder")
    ap.add_argument("--batch-sizes", default=None,
                    help="comma-separated batch sizes over the sorted query (the last repeats); default: --batch")
    ap.add_argument("--early-decodes", type=int, default=None,
                    help="only the first K batches decode beside the next encoder; the others wait for every encode "
                         "(default: all decode right after their encode)")
    ap.add_argument("--batch-order", default=None,
                    help="development: this rank's batches in another order, a permutation of their indices "
                         "(e.g. 0,5,1,4,2,3; default: longest first)")
    ap.add_argument("--cpu-sample", type=int, default=256, help="utterances timed on the CPU restatement")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--wav", action="store_true",
                    help="WAV=true path (launch_sut.sh:53-55): the QSL holds 16 kHz audio and every batch runs the "
                         "GPU featurizer (FilterbankFeatures.forward) inside the timed region")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "tools", "roofline_traffic.json"),
                    help="per-launch HBM bytes from a rocprofv3 --pmc pass (profiles/), if present")
    ap.add_argument("--deal", choices=("dynamic", "static"), default="dynamic",
                    help="several ranks: claim batches from one shared counter when the encoder is free (dynamic), or "
                         "deal them in snake order up front (static)")
    ap.add_argument("--sut-warmup", type=int, default=0,
                    help="OfflineSUT.warmup iterations on dummy samples before the --warmup steps (default 0: the "
                         "--warmup steps on real batches already take the first-call costs; DESIGN section 5)")
    ap.add_argument("--sut-warmup-frames", type=int, default=500, help="frames per dummy sample (MAX_FEA_LEN)")
    ap.add_argument("--share-device", action="store_true",
                    help="multi-rank rehearsal on a 1-GPU box: every rank on cuda:0, control plane on gloo (RCCL refuses "
                         "two ranks on one device); the line checks the multi-process path, it is not a measurement")
    ap.add_argument("--dump-responses", default=None,
                    help="rank 0 writes the last timed query's gathered responses (ids, lens, toks) to this .npz")
    ap.add_argument("--control-backend", choices=("gloo", "nccl"), default="gloo",
                    help="torch.distributed backend of the control plane (barriers, max-over-ranks timing, batch "
                         "claims) for --gpus N: the data path has no collective (DESIGN section 6), and gloo is the "
                         "backend the multi-rank hardware rehearsal (--share-device) ran; nccl (RCCL) is opt-in")
    ap.add_argument("--mock", action="store_true",
                    help="launcher / sharding check without a GPU: gloo ranks deal and gather a query of stand-in "
                         "responses (no engine, no HIP); the line it prints is not a measurement")
    return ap.parse_args()


def control_backend(args):
    """Backend of the multi-rank control plane: gloo unless --control-backend nccl (RCCL refuses two
    ranks on one device, so --share-device is always gloo).  Utterances are independent, so no
    device-side collective is on the data path; barriers and the max-over-ranks timing
    are host scalars."""
    if args.share_device or args.mock:
        return "gloo"
    return args.control_backend


def launch_ranks(args):
    """``--gpus N`` (N > 1) outside a torchrun environment: run this script as N ranks under
    torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) in a child process and
    return its exit code.  The parent never initialises HIP (only argparse has run), so the ranks
    own the GPUs.  None when this process is already a rank (WORLD_SIZE set) or N == 1."""
    if "WORLD_SIZE" in os.environ or args.gpus <= 1:
        return None
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def mock_main(args):
    """CPU rehearsal of the multi-rank step (--mock): the same shard / gather / barrier / max-over-ranks
    timing as main() over gloo, with stand-in token rows instead of the engine."""
    rank, _, world, group = dist.setup(control_backend(args))
    lens = synthetic.devclean_lengths(args.qsl, seed=4)
    from rnnt_amd.sut import RNNTQSL
    qsl = RNNTQSL([None] * len(lens), lens)
    query = args.query * world
    ids, idx = dist.query_arrays(args.qsl, query)

    qno = [0]

    def step():
        if args.deal == "static" or world == 1:
            mine = dist.shard_query(qsl, ids, idx, args.batch, rank, world)
        else:
            batches = make_batches(qsl, ids, idx, args.batch)
            claim = dist.claim_for_query(qno[0], len(batches))
            mine = []
            while (i := claim()) is not None:
                mine.append(batches[i])
        stream = dist.ResponseStream(world, group, tag=qno[0]) if world > 1 else None
        qno[0] += 1
        got = []
        for b_ids, b_idx in mine:  # stand-in responses, shipped batch by batch like the SUT's completions
            # the timed workload's volume: ~0.55 symbols per encoder frame (64.6 per sample in BENCH_r05)
            rl = (((lens[b_idx] + 1) // 2) * (45 + b_ids % 21) // 100).astype(np.int32)
            toks = np.repeat((b_ids % 29).astype(np.int32), rl)
            if stream:
                stream.push(b_ids, rl, toks)
            else:
                got.append((b_ids, rl, toks))
        if stream:
            return stream.finish()
        return tuple(np.concatenate([g[k] for g in got]) for k in range(3))

    for _ in range(args.warmup):
        step()
    dist.barrier(group)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        got = step()
    dist.barrier(group)
    elapsed = dist.reduce_max(time.perf_counter() - t0, group)
    if rank == 0:
        assert len(got[0]) == query and len(np.unique(got[0])) == query, "gathered responses do not cover the query"
        if args.dump_responses:
            np.savez_compressed(args.dump_responses, ids=got[0], lens=got[1], toks=got[2])
        print(json.dumps({"metric": METRIC, "value": None, "unit": "utterances/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
                          "rows_per_s_gathered": round(query * args.steps / elapsed, 1),
                          "tokens_per_query": int(got[1].sum()),
                          "data": "mock: no engine, stand-in responses (launcher / sharding check, not a measurement)",
                          "control_plane": dist.backend_name(),
                          "config": {"query_samples": query, "gathered": int(len(got[0]))}}), flush=True)
    if world > 1:
        import torch.distributed as tdist
        tdist.destroy_process_group()


def build_qsl(count, seed, device, wav=False):
    """The QSL on this rank's GPU: dev-clean-shaped lengths; N(0,1) features ragged in HBM, or
    speech-shaped synthetic 16 kHz audio (--wav).  Same seed on every rank: the same samples."""
    lens = synthetic.devclean_lengths(count, seed=seed)
    if not wav:
        return GpuQSL(lens, seed=seed, device=device)
    wav_lens = synthetic.wav_lengths_for_frames(lens, seed=seed)
    q = GpuWavQSL(synthetic.make_wavs(wav_lens, seed=seed, device=device), device=device)
    assert np.array_equal(q.lengths, lens)
    return q


def sample_timed_rows(batches, batch_engine, n_sample, inflight):
    """Rows of the timed query to re-check on the CPU: evenly spaced rows (first = longest,
    last = shortest) of the first batch each engine ran and of the query's last batch, so the
    sample spans every engine in flight and both ends of the length-sorted query."""
    firsts = {}
    for i, e in enumerate(batch_engine):
        firsts.setdefault(e, i)
    picks = sorted(set(firsts.values()) | {len(batches) - 1})
    per = max(2, -(-n_sample // len(picks)))
    out = []
    for b in picks:
        n = len(batches[b][0])
        rows = np.unique(np.linspace(0, n - 1, min(per, n)).round().astype(np.int64))
        out += [(b, int(r)) for r in rows]
    return out


def cpu_baseline(pm, qsl, batches, batch_engine, responses, n_sample, inflight):
    """The C restatement (oracle/, TEST INFRASTRUCTURE) timed on this host's cores on a bounded
    sample of the timed query's own utterances, and the parity check of the tokens the GPU
    produced for those samples INSIDE the timed region (last timed step) against it."""
    from oracle import oracle
    picks = sample_timed_rows(batches, batch_engine, n_sample, inflight)
    sid = np.array([batches[b][0][r] for b, r in picks], np.int64)
    qidx = np.array([batches[b][1][r] for b, r in picks], np.int64)
    order = np.argsort(-qsl.lengths[qidx], kind="stable")  # longest first, as the SUT sorts
    sid, qidx = sid[order], qidx[order]
    sl = qsl.lengths[qidx].astype(np.int32)
    n, T = len(sl), int(sl.max())
    x = np.zeros((T, n, 256), np.float32)
    for i, q in enumerate(qidx):
        o = int(qsl.offsets[q])
        x[: sl[i], i, :240] = qsl.feats[o: o + int(sl[i])].cpu().numpy()
    import ctypes
    lib = oracle.lib()
    cpus, meta = host_cpu_budget()
    arr = (ctypes.c_int * len(cpus))(*cpus)
    lib.oracle_pin_threads.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    pinned = lib.oracle_pin_threads(len(cpus), arr)
    lib.oracle_bind_master(cpus[0])
    try:
        t0 = time.perf_counter()
        f = oracle.encoder_i8(pm, x, sl)
        res, rl, _ = oracle.greedy_decode(pm, f, (sl + 1) // 2, max_res=(500 // 2) * 30)
        dt = time.perf_counter() - t0
    finally:
        lib.oracle_bind_master(-1)
    meta["threads_pinned"] = int(pinned)
    mism = 0
    for i, s in enumerate(sid):
        row = responses.get(int(s))
        if row is None or len(row) != int(rl[i]) or not np.array_equal(row, res[i, : rl[i]]):
            mism += 1
    return dict(value=n / dt, seconds=dt, n=n, cores=lib.oracle_num_threads(), frames=int(sl.sum()),
                mismatches=mism, batches=sorted({b for b, _ in picks}),
                engines=sorted({batch_engine[b] for b, _ in picks}), host=meta)


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def cgroup_cpu_quota():
    """The cgroup CPU bandwidth limit of this process in CPUs (quota / period), or None when
    unlimited / unreadable.  cgroup v2 (`cpu.max`) and v1 (`cpu.cfs_quota_us` / `cpu.cfs_period_us`),
    at the namespace root and at the process's own cgroup path."""
    paths = []
    for line in (_read("/proc/self/cgroup") or "").splitlines():
        parts = line.split(":", 2)
        if len(parts) == 3:
            ctl, rel = parts[1], parts[2]
            if ctl == "":
                paths.append(("v2", "/sys/fs/cgroup" + rel))
            elif "cpu" in ctl.split(","):
                for mnt in ("/sys/fs/cgroup/cpu", "/sys/fs/cgroup/cpu,cpuacct"):
                    paths.append(("v1", mnt + rel))
    paths += [("v2", "/sys/fs/cgroup"), ("v1", "/sys/fs/cgroup/cpu"), ("v1", "/sys/fs/cgroup/cpu,cpuacct")]
    for kind, d in paths:
        if kind == "v2":
            v = _read(os.path.join(d, "cpu.max"))
            if v:
                q, _, per = v.partition(" ")
                if q == "max":
                    return None
                return int(q) / int(per or 100000)
        else:
            q, per = _read(os.path.join(d, "cpu.cfs_quota_us")), _read(os.path.join(d, "cpu.cfs_period_us"))
            if q is not None and per is not None:
                return None if int(q) < 0 else int(q) / int(per)
    return None


def host_cpu_budget():
    """The host CPUs this process can actually use: its affinity set, capped by the cgroup quota
    (a GPU box grants a share of a many-core host: affinity may list every CPU while the quota
    allows 16).  -> (cpus to pin one OpenMP thread each to, metadata).  CPUs are taken one per
    physical core first (SMT siblings last), in affinity order."""
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    quota = cgroup_cpu_quota()
    n = len(aff) if quota is None else max(1, min(len(aff), int(quota)))
    env_threads = os.environ.get("OMP_NUM_THREADS")
    seen, first, second = set(), [], []
    for c in aff:
        key = (_read(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id"),
               _read(f"/sys/devices/system/cpu/cpu{c}/topology/core_id"))
        (second if key in seen and key != (None, None) else first).append(c)
        seen.add(key)
    cpus = (first + second)[:n]
    meta = {"affinity_cpus": len(aff), "machine_cpus": os.cpu_count(),
            "cgroup_cpu_quota": round(quota, 3) if quota is not None else None,
            "omp_num_threads_env": env_threads, "threads": n,
            "pinning": f"one OpenMP thread per CPU (sched_setaffinity), CPUs {cpus[0]}..{cpus[-1]}" if len(cpus) > 1
                       else f"one thread on CPU {cpus[0]}"}
    return cpus, meta


def host_cpu_model():
    for line in (_read("/proc/cpuinfo") or "").splitlines():
        if line.startswith("model name"):
            return line.split(":", 1)[1].strip()
    return None


def wer_vs_fp32(n=1024, seed=44):
    """BASELINE metric's second half ("WER vs fp32 ref"), measured on the well-conditioned
    planted model (rnnt_amd.planted: contractive encoder, confident joint -- the regime of a
    trained network; the random-init throughput model's decisions sit at bf16-rounding margins,
    see DESIGN.md section 2).  n dev-clean-shaped utterances of the planted task; hypothesis =
    the int8 encoder + bf16 decoder (the timed path's kernels), reference = the fp32 encoder +
    fp32 decoder, both on the GPU through GreedyDecoder.  The criterion is MLPerf's: each path's
    WER against the transcripts, the quantised one within 1 point of fp32 (wer_delta); the
    pairwise transcript disagreement is reported beside it (a few utterances whose greedy decode
    cascades after one flipped decision dominate it)."""
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

    w32, w8 = w(hyp["f32"], ref), w(hyp["quant"], ref)
    differ = sum(a != b for a, b in zip(hyp["quant"], hyp["f32"]))
    return {"utterances": n, "seed": seed, "model": "planted (well-conditioned) RNN-T, rnnt_amd/planted.py",
            "fp32_vs_planted_truth": w32, "int8_bf16_vs_planted_truth": w8,
            "wer_delta": round(w8["wer"] - w32["wer"], 5),
            "target": "wer_delta <= 0.01 (north_star 'WER within 1% of fp32 reference', MLPerf-style: each path's WER "
                      "vs the transcripts)",
            "int8_bf16_vs_fp32": w(hyp["quant"], hyp["f32"]), "utterances_differing": differ,
            "hypothesis": "int8 encoder + bf16 prediction/joint (GPU)", "reference": "fp32 encoder + fp32 decoder (GPU)",
            "note": "synthetic planted task (no checkpoint / LibriSpeech offline); teacher-forced joint-logit tolerance "
                    "on both models: tests/test_accuracy_gpu.py"}


def responses_dict(ids, lens, toks):
    out, off = {}, 0
    for i, L in zip(ids, lens):
        out[int(i)] = toks[off: off + int(L)]
        off += int(L)
    return out


def summarize(args, world, query, elapsed_max, st, iso, lengths, mine, got, my_emitted, sizes):
    """The JSON line of a measured run (everything but the rank-0-only extras): value, roofline (this
    rank's share of the query: a rank may run no batch at all -- a query of fewer batches than ranks, or
    claims taken by faster ranks), config.  st / iso: summed rnnt_engine_get_stats of the timed steps /
    of the isolated pass; lengths: the QSL's lengths; mine: this rank's (ids, qsl indices) batches."""
    value = query * args.steps / elapsed_max
    # this rank's share (a rank may run no batch: a query of fewer batches than ranks, or claims
    # taken by faster ranks)
    qlens = np.concatenate([lengths[b[1]] for b in mine]) if mine else np.zeros(0, np.int64)
    enc_frames = int(sum(encoder_frames(l) for l in qlens))
    enc_ops = float(sum(encoder_ops(int(l)) for l in qlens))  # SURVEY 8d E(T), valid frames
    emitted = int(got[1].sum()) if got is not None else 0  # whole query (rank 0 holds the gathered responses)
    achieved = enc_ops * args.steps / (st["encode_ms"] * 1e-3) / 1e12 if st["encode_ms"] > 0 else 0.0
    achieved_iso = enc_ops / (iso["encode_ms"] * 1e-3) / 1e12 if iso["encode_ms"] > 0 else 0.0
    traffic, traffic_src = None, None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            traffic, traffic_src = tj.get("lstm_i8_step_bytes_per_launch"), tj.get("source")
        except Exception:
            traffic = None
    # decode work: D = (T' + U) * 4,682,752 bf16 ops per utterance (this rank's share)
    dec_ops = float(enc_frames + my_emitted) * DECODE_OPS_PER_STEP
    dec_ms = (st["greedy_ms"] + st["joint_trans_ms"]) / args.steps
    dec_ms_iso = iso["greedy_ms"] + iso["joint_trans_ms"]
    dec_ach = dec_ops / (dec_ms * 1e-3) / 1e12 if dec_ms > 0 else 0.0
    dec_ach_iso = dec_ops / (dec_ms_iso * 1e-3) / 1e12 if dec_ms_iso > 0 else 0.0
    ticks_q = st["step_launches"] / args.steps
    roofline = {
        "bound": "mfma", "kernel": "lstm_i8_tick_kernel (int8 encoder, up to 5 layer-steps per launch)",
        "achieved": round(achieved, 2), "peak": INT8_DENSE_PEAK_TOPS, "unit": "TFLOP/s",
        "frac": round(achieved / INT8_DENSE_PEAK_TOPS, 4), "traffic": traffic,
        "traffic_source": ("HBM bytes per tick launch, rocprofv3 PMC pass of this round's profile "
                           "(tools/gpu.sh profile; (2 FETCH_SIZE + WRITE_SIZE) x 1024): " + str(traffic_src))
        if traffic is not None else None,
        "measured_on": "HIP events around every encode call on its own stream, timed region (encode overlaps "
                       "other batches' decode); rank 0's share of the query",
        "encode_ms_per_query": round(st["encode_ms"] / args.steps, 3),
        "joint_trans_ms_per_query": round(st["joint_trans_ms"] / args.steps, 3),
        "greedy_ms_per_query": round(st["greedy_ms"] / args.steps, 3),
        "tick_launches_per_query": int(st["step_launches"] // args.steps),
        "encode_us_per_tick_events": round(st["encode_ms"] / args.steps / ticks_q * 1e3, 2) if ticks_q else None,
        "encode_us_per_tick_note": "event time per encode call / tick launches (includes the gather-quantize kernel "
                                   "and the gaps between ticks; rocprofv3 kernel stats give the kernel alone)",
        "decode": {"kernels": "joint_trans_gemm_kernel + dec_pred/g/joint step kernels (bf16 MFMA)",
                   "ops_per_query": dec_ops, "achieved": round(dec_ach, 2), "peak": BF16_DENSE_PEAK_TFLOPS,
                   "unit": "TFLOP/s", "frac": round(dec_ach / BF16_DENSE_PEAK_TFLOPS, 4),
                   "isolated_achieved": round(dec_ach_iso, 2),
                   "isolated_frac": round(dec_ach_iso / BF16_DENSE_PEAK_TFLOPS, 4),
                   "note": "latency-bound lock-step greedy loop; time = joint_trans + greedy event time"},
        "isolated": {"achieved": round(achieved_iso, 2), "frac": round(achieved_iso / INT8_DENSE_PEAK_TOPS, 4),
                     "encode_ms_per_query": round(iso["encode_ms"], 3),
                     "greedy_ms_per_query": round(iso["greedy_ms"], 3),
                     "note": "untimed pass, this rank's batches back to back on one engine (no overlap)"},
    }
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "utterances/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed_max / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int8",
        "data": ("synthetic (seeded dev-clean-shaped speech-like 16 kHz audio, random-init RNN-T weights)" if args.wav
                 else "synthetic (seeded dev-clean-shaped lengths, N(0,1) features, random-init RNN-T weights)"),
        "config": {"workload": "MLPerf Offline query over a LibriSpeech-dev-clean-shaped QSL (BASELINE config 4)",
                   "qsl": args.qsl, "query_samples": query, "query_samples_per_gpu": args.query,
                   "query_source": ("configs/user.conf:6 Offline.min_query_count (the reference's run setting, "
                                    "launch_sut.sh:46)" if args.query == 300000 else "--query"),
                   "batch_size": args.batch, "batch_sizes": sizes, "batches_in_flight_per_gpu": args.inflight,
                   "input": ("16 kHz audio: GPU featurizer (FilterbankFeatures.forward) in the timed region" if args.wav
                             else "log-mel features resident in HBM, gathered by the encoder's quantize pass"),
                   "encoder": "int8 (lstm_amx_int8)",
                   "decoder": "bf16 prediction/joint, fp32 accumulate, greedy (device loop)",
                   "parallelism": f"dp{world}: one query sorted and batched; {world} process(es), one per GPU, "
                                  + ("claim batches from one shared counter when their encoder is free" if world > 1 and
                                     args.deal == "dynamic" else "batches dealt in snake order")
                                  + "; responses streamed to rank 0's host (gloo) inside the timed region",
                   "batches_run_rank0": len(mine),
                   "encoder_frames_per_query_rank0": enc_frames, "emitted_symbols_per_query": emitted},
        "roofline": roofline,
        "control_plane": dist.backend_name(),
    }
    return out


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    _, local, world = dist.env_rank()
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the torchrun world has {world} rank(s)")
    if args.mock:
        return mock_main(args)
    from rnnt_amd import _lib
    # a fatal signal names the shared object of every frame (round 5's exit-time fault named none)
    _lib.check(_lib.lib().rnnt_install_crash_report(), "rnnt_install_crash_report")
    dev = 0 if args.share_device else local
    torch.cuda.set_device(dev)
    rank, local, world, ggroup = dist.setup(control_backend(args))
    device = f"cuda:{dev}"
    pm, _ = weights.build_model()
    qsl = build_qsl(args.qsl, seed=4, device=device, wav=args.wav)
    query = args.query * world
    ids, idx = dist.query_arrays(args.qsl, query)
    max_b = max([args.batch] + ([int(v) for v in args.batch_sizes.split(",")] if args.batch_sizes else []))
    engines = [Engine(pm, device=dev, max_batch=min(max_b, query), max_frames=500) for _ in range(args.inflight)]
    sut = OfflineSUT(engines, qsl, early_decodes=args.early_decodes)
    if args.sut_warmup:  # OfflineSUT::warmup (torch_sut.cpp:124-138), before any query
        sut.warmup(iters=args.sut_warmup, batch_size=args.batch, frames=args.sut_warmup_frames)
    sizes = [int(v) for v in args.batch_sizes.split(",")] if args.batch_sizes else None

    qno = [0]

    def step():
        """One Offline query: sort + batch, this rank's batches through the SUT (claimed from the
        shared counter, or dealt), every batch's responses streamed to rank 0 as it completes
        (dist.ResponseStream, tagged with the query number)."""
        if world > 1 and args.deal == "dynamic":
            batches = make_batches(qsl, ids, idx, args.batch, sizes)
            claim = dist.claim_for_query(qno[0], len(batches))
        else:
            batches, claim = dist.shard_query(qsl, ids, idx, args.batch, rank, world, sizes), None
            if args.batch_order:
                order = [int(v) for v in args.batch_order.split(",")]
                if sorted(order) != list(range(len(batches))):
                    raise SystemExit(f"--batch-order must permute 0..{len(batches) - 1}")
                batches = [batches[i] for i in order]
        stream = dist.ResponseStream(world, ggroup, tag=qno[0]) if world > 1 else None
        qno[0] += 1
        sut.on_batch = stream.push if stream else None
        sut.issue_batches(batches, claim=claim)
        local = sut.take_completed()
        got = stream.finish() if stream else local
        return sut.ran_batches(batches), got, int(local[1].sum())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    for e in engines:  # HIP events around every encode / joint_trans / greedy call, on its stream
        e.set_profiling(True)
        e.stats(reset=True)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        mine, got, my_emitted = step()
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed_max = dist.reduce_max(elapsed)
    sts = [e.stats(reset=True) for e in engines]
    st = {k: sum(x[k] for x in sts) for k in sts[0]}
    batch_engine = [e for e in sut.batch_engine if e is not None]  # aligned with `mine` (the batches this rank ran)
    # isolated pass (untimed): this rank's batches once more on one engine, back to back, so the
    # encoder's event time is not shared with an overlapping decode
    iso_sut = OfflineSUT([engines[0]], qsl)
    iso_sut.issue_batches(mine)
    iso_sut.take_completed()
    iso = engines[0].stats(reset=True)
    for e in engines:
        e.set_profiling(False)
    out = summarize(args, world, query, elapsed_max, st, iso, qsl.lengths, mine, got, my_emitted, sizes)
    if rank == 0 and got is not None:
        assert len(got[0]) == query and len(np.unique(got[0])) == query, "gathered responses do not cover the query"
        if args.dump_responses:
            np.savez_compressed(args.dump_responses, ids=got[0], lens=got[1], toks=got[2])
    if args.share_device:
        out["rehearsal"] = (f"{world} ranks share cuda:0 (gloo control plane): multi-process path check, not a "
                            "measurement")
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.wav:
        resp = responses_dict(*got)
        cb = cpu_baseline(pm, qsl, mine, batch_engine, resp, args.cpu_sample, args.inflight)
        out["cpu_baseline"] = {"value": round(cb["value"], 3), "unit": "utterances/s", "cores": cb["cores"],
                               "kind": "port", "cpu_model": host_cpu_model(), **cb["host"],
                               "sample": f"{cb['n']} utterances ({cb['frames']} frames) of the timed query (batches "
                                         f"{cb['batches']}, longest to shortest rows), int8 encoder + greedy decode, "
                                         f"{cb['seconds']:.1f} s"}
        out["parity_spot_check"] = {"utterances": cb["n"], "source": "responses completed inside the last timed step",
                                    "batches": cb["batches"], "engines": cb["engines"],
                                    "mismatched_rows": cb["mismatches"], "tokens_identical": cb["mismatches"] == 0}
        out["wer_vs_fp32"] = wer_vs_fp32()
    if rank == 0:
        print(json.dumps(out), flush=True)
    # teardown in a fixed order, before interpreter exit: the SUTs' threads have all joined (issue_batches),
    # then every engine is destroyed and the QSL freed while torch's HIP runtime is fully up, the device
    # drained, and the process group closed; nothing of ours is left to a __del__ or a static destructor
    del sut, iso_sut
    for e in engines:
        e.close()
    del engines, qsl
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    if world > 1:
        import torch.distributed as tdist
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
