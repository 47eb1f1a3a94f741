#!/usr/bin/env python3
"""Throughput of the HIP featurizer on one batch of dev-clean-shaped synthetic audio.

    python tools/bench_featurizer.py --batch 8192 --iters 10
Prints one JSON line: utterances/s, audio seconds/s, and the HBM roofline of the pair of kernels
with algorithmic bytes = 4 B per input sample + 4 B x 256 per output frame row written
(feats [T_out][n_pad][256], including the zero padding the layout requires); the
intermediate write + re-read of the valid rows is not counted.  Samples are stored ragged (offsets).
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rnnt-inference_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rnnt_amd import synthetic  # noqa: E402
from rnnt_amd.featurizer import FilterbankFeatures, feature_frames  # noqa: E402

HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--distinct", type=int, default=512, help="distinct synthetic utterances (repeated)")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--seed", type=int, default=4)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    fz = FilterbankFeatures(sample_rate=16000, window="hann", n_fft=512, nfilt=80, frame_splicing=3,
                            pad_out_feat=True)
    frames = synthetic.devclean_lengths(args.distinct, seed=args.seed)
    lens_d = synthetic.wav_lengths_for_frames(frames, seed=args.seed)
    wavs = synthetic.make_wavs(lens_d, seed=args.seed, device="cuda")
    store = torch.cat(wavs)
    off_d = np.concatenate([[0], np.cumsum(lens_d.astype(np.int64))[:-1]])
    pick = np.random.default_rng(args.seed).integers(0, args.distinct, args.batch)
    pick = pick[np.argsort(-lens_d[pick], kind="stable")]  # sorted like the Offline batches
    lens = lens_d[pick].astype(np.int32)
    off = torch.from_numpy(off_d[pick]).cuda()
    lens_dev = torch.from_numpy(lens).cuda()
    T_out = max(feature_frames(int(v)) for v in lens)
    out = torch.empty((T_out, args.batch, 256), dtype=torch.float32, device="cuda")
    fl = torch.empty(args.batch, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    for _ in range(2):
        fz.featurize(store, lens_dev, lens, n_pad=args.batch, T_out=T_out, offsets=off, out=out, feat_lens=fl)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(args.iters):
        fz.featurize(store, lens_dev, lens, n_pad=args.batch, T_out=T_out, offsets=off, out=out, feat_lens=fl)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    samples = int(lens.sum())
    valid_rows = int(sum(feature_frames(int(v)) for v in lens))
    algo = 4.0 * samples + 1024.0 * T_out * args.batch  # compulsory: samples in, feature rows out
    print(json.dumps({"kernel": "featurizer (fz_logmel + fz_norm)", "batch": args.batch, "T_out": T_out,
                      "valid_frames": valid_rows,
                      "ms_per_batch": round(ms, 3), "utterances_per_s": round(args.batch / ms * 1e3, 1),
                      "audio_seconds_per_s": round(samples / 16000.0 / ms * 1e3, 1),
                      "roofline": {"bound": "hbm", "achieved": round(algo / ms / 1e6, 1), "peak": HBM_PEAK_GBS,
                                   "unit": "GB/s", "frac": round(algo / ms / 1e6 / HBM_PEAK_GBS, 4),
                                   "algorithmic_bytes": algo}}))
    fz.close()


if __name__ == "__main__":
    main()
