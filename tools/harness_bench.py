#!/usr/bin/env python3
"""Throughput of the compiled TorchModel drop-in under the harness's restated reference SUT
(rnnt_sut_harness --scenario offline) on bench.py's workload: the same 2513-sample QSL (identical
features: GpuQSL's seeded generator on the GPU, copied to host memory as the reference QSL holds
them), the same query (ids 0..Q-1, QSL index id % 2513).  Unlike bench.py's `value`, the inputs start
in host memory: the harness assembles each batch on the host (AssembleSamples) and the model copies it
to the GPU, so the rate is PCIe- and host-inclusive.

    python tools/harness_bench.py --query 300000 --batch 6144 --threads 4 [--compare bench_dump.npz]

--compare: a bench.py --dump-responses file of the same query; every response must match.
Prints one JSON line (the harness's, plus the workload)."""
import argparse
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rnnt-inference_amd"))

import numpy as np  # noqa: E402

HARNESS = os.path.join(REPO, "rnnt-inference_amd", "rnnt_amd", "rnnt_sut_harness")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qsl", type=int, default=2513)
    ap.add_argument("--query", type=int, default=300000)
    ap.add_argument("--batch", type=int, default=6144)
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--split-len", type=int, default=-1)
    ap.add_argument("--intra", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--pinned", type=int, default=0, help="1: the harness assembles batches in pinned memory")
    ap.add_argument("--check-fill", type=int, default=0,
                    help="1: the harness also scans every answered row's SOS fill (the tests do; 184 MB per 6144-row "
                         "batch, not part of the reference's response path)")
    ap.add_argument("--preassemble", type=int, default=0,
                    help="1: every batch assembled before the timed region (the model's own rate, host assembly excluded)")
    ap.add_argument("--wav", action="store_true",
                    help="WAV=true: bench.py --wav's audio QSL in host memory, featurized by the AudioProcessor drop-in")
    ap.add_argument("--compare", default=None)
    ap.add_argument("--workdir", default=None)
    args = ap.parse_args()

    import torch
    from rnnt_amd import synthetic, weights
    from rnnt_amd.sut import GpuQSL
    work = args.workdir or tempfile.mkdtemp(prefix="rnnt_harness_", dir="/tmp")
    os.makedirs(work, exist_ok=True)
    lens = synthetic.devclean_lengths(args.qsl, seed=4)
    if args.wav:  # bench.py's build_qsl(wav=True): the same audio
        from rnnt_amd.featurizer import write_processor_file
        wav_lens = synthetic.wav_lengths_for_frames(lens, seed=4)
        wavs = synthetic.make_wavs(wav_lens, seed=4, device="cuda:0")
        with open(os.path.join(work, "wav.bin"), "wb") as f:
            for w in wavs:
                f.write(w.cpu().numpy().astype(np.float32).tobytes())
        del wavs
        torch.cuda.empty_cache()
        wav_lens.astype(np.int32).tofile(os.path.join(work, "wav_lens.bin"))
        write_processor_file(os.path.join(work, "rnnt.processor"))
    else:
        q = GpuQSL(lens, seed=4, device="cuda:0")  # bench.py's build_qsl: the same features
        print(f"[harness_bench] QSL {args.qsl} samples, query {args.query}", file=sys.stderr, flush=True)
        q.feats.cpu().numpy().tofile(os.path.join(work, "feats.bin"))
        del q
        torch.cuda.empty_cache()
        lens.astype(np.int32).tofile(os.path.join(work, "lens.bin"))
    (np.arange(args.query, dtype=np.int64) % args.qsl).astype(np.int32).tofile(os.path.join(work, "query.bin"))
    pm, _ = weights.build_model()
    eng = weights.save_engine_file(pm, os.path.join(work, "rnnt.engine"))
    out = os.path.join(work, "responses.bin")
    src = (["--processor", os.path.join(work, "rnnt.processor"), "--wav", os.path.join(work, "wav.bin"), "--wav-lens",
            os.path.join(work, "wav_lens.bin")] if args.wav else
           ["--feats", os.path.join(work, "feats.bin"), "--lens", os.path.join(work, "lens.bin")])
    cmd = [HARNESS, "--engine", eng] + src + [
           "--query", os.path.join(work, "query.bin"), "--scenario", "offline", "--threads", str(args.threads),
           "--batch", str(args.batch), "--split-len", str(args.split_len), "--intra", str(args.intra),
           "--warmup", str(args.warmup), "--pinned", str(args.pinned), "--preassemble", str(args.preassemble),
           "--check-fill", str(args.check_fill), "--out", out]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True)  # progress lines pass through on stderr
    if r.returncode != 0:
        sys.exit(r.returncode)
    res = json.loads(r.stdout.strip().splitlines()[-1])
    res["workload"] = {"qsl": args.qsl, "query_samples": args.query,
                       "features": ("bench.py --wav's audio (seed 4) in host memory, AudioProcessor drop-in" if args.wav
                                    else "bench.py's GpuQSL (seed 4) in host memory"),
                       "rate": "host- and PCIe-inclusive: AssembleSamples on the host, the model's staged copy to HBM"}
    res["intra"] = args.intra
    if args.compare:
        d = np.load(args.compare)
        want, off = {}, 0
        for i, L in zip(d["ids"], d["lens"]):
            want[int(i)] = d["toks"][off: off + int(L)]
            off += int(L)
        b = open(out, "rb").read()
        got, off, bad = 0, 0, 0
        while off < len(b):
            sid, size = np.frombuffer(b, np.int32, 2, off)
            off += 8
            row = np.frombuffer(b, np.int32, int(size) // 4, off)
            off += int(size)
            got += 1
            w = want.get(int(sid))
            bad += int(w is None or not np.array_equal(row, w))
        res["compare_with_bench"] = {"responses": got, "mismatched": bad, "bench_rows": len(want)}
    os.remove(out)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
