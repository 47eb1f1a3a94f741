#!/usr/bin/env python3
"""Calibrate + quantise + export a packed model file (the reference's calibration and save_jit
stages, models/main.py:21-58, calib_model.sh / save_model.sh, in one offline step).

    python tools/export_model.py --checkpoint rnnt.pt --calib-features calib.npz --out rnnt_quant.npz
    python tools/export_model.py --synthetic --out rnnt_synth.npz
--checkpoint: the MLPerf RNN-T state dict (.pt loaded with weights_only=True, .safetensors or .npz).
--calib-features: .npz with "feats" [T][N][>=240] fp32 (normalised log-mel, the calibration set's
featurizer output) and "lens" [N]; default: the synthetic calibration batch build_model uses.
--amax: five comma-separated values to skip calibration (e.g. from an earlier export).
The output (rnnt_amd.weights.save_prepared) is read by rnnt_amd.weights.load_prepared and handed
to rnnt_amd.engine.Engine; --engine-file also writes the flat container the C ABI loads directly
(rnnt_engine_create_from_file, for the C++ SUT) and --processor-file the audio processor's (window +
filterbank, rnnt_featurizer_create_from_file).  One JSON line (amax, scales, digest) goes to stdout.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rnnt-inference_amd"))

import numpy as np  # noqa: E402

from rnnt_amd import synthetic, weights  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    src = ap.add_mutually_exclusive_group(required=True)
    src.add_argument("--checkpoint")
    src.add_argument("--synthetic", action="store_true", help="the seeded random-init checkpoint (synthetic.py)")
    ap.add_argument("--seed", type=int, default=synthetic.DEFAULT_SEED)
    ap.add_argument("--calib-features")
    ap.add_argument("--calib-n", type=int, default=2)
    ap.add_argument("--calib-T", type=int, default=120)
    ap.add_argument("--amax")
    ap.add_argument("--fp32-decoder", action="store_true", help="keep prediction/joint fp32 (enable_bf16 off)")
    ap.add_argument("--out", required=True)
    ap.add_argument("--engine-file", help="also write the C-loadable engine model file (RNNTMI01)")
    ap.add_argument("--processor-file", help="also write the audio processor file the C++ AudioProcessor drop-in "
                                             "loads (configs/rnnt.toml [input_eval] geometry; RNNTMI01)")
    args = ap.parse_args()

    ckpt = weights.load_checkpoint(args.checkpoint) if args.checkpoint else synthetic.make_checkpoint(args.seed)
    sd = weights.migrate_state_dict(ckpt)
    if args.amax:
        amax = np.array([float(v) for v in args.amax.split(",")], np.float32)
        calib = "given"
    elif args.calib_features:
        with np.load(args.calib_features, allow_pickle=False) as z:
            feats, lens = z["feats"], z["lens"]
        amax = weights.calibrate_amax(sd, feats, lens)
        calib = f"{args.calib_features}: {feats.shape[1]} utterances"
    else:  # build_model's synthetic calibration batch
        lens = np.full(args.calib_n, args.calib_T, np.int32)
        feats = synthetic.make_features(args.calib_T, args.calib_n, seed=args.seed ^ 0xCA1B, lens=lens)
        amax = weights.calibrate_amax(sd, feats, lens)
        calib = f"synthetic {args.calib_n} x {args.calib_T} frames"
    pm = weights.prepare_model(ckpt, amax, bf16=not args.fp32_decoder)
    meta = weights.save_prepared(pm, args.out, extra={"calibration": calib,
                                                      "source": args.checkpoint or f"synthetic seed {args.seed}"})
    if args.engine_file:
        weights.save_engine_file(pm, args.engine_file)
        meta["engine_file"] = args.engine_file
    if args.processor_file:
        from rnnt_amd.featurizer import write_processor_file
        write_processor_file(args.processor_file)
        meta["processor_file"] = args.processor_file
    print(json.dumps({"out": args.out, "amax": [float(v) for v in amax], "in_scale": [float(v) for v in pm.enc_in_s],
                      "rb_scale": [float(v) for v in pm.enc_rb], **meta}))


if __name__ == "__main__":
    main()
