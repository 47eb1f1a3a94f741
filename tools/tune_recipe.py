#!/usr/bin/env python3
"""Development: emission statistics of synthetic-checkpoint recipes on the CPU restatement.

    python tools/tune_recipe.py blank_bias=13 post_emit_blank=0.1 ...
Runs the fp32 encoder + greedy decode (oracle/, test infrastructure) on a dev-clean-shaped
sample and prints symbols per 30 ms frame and the per-utterance U/T' distribution.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rnnt-inference_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

from oracle import oracle  # noqa: E402
from rnnt_amd import synthetic, weights  # noqa: E402


def stats(recipe, n=48, tmax=200, seed=7):
    ck = synthetic.make_checkpoint(synthetic.DEFAULT_SEED, recipe)
    sd = weights.migrate_state_dict(ck)
    layers = [weights.enc_layer_params(sd, l) for l in range(5)]
    pm = weights.prepare_model(ck, np.ones(5, np.float32) * 6.0, bf16=False)
    lens = np.minimum(synthetic.devclean_lengths(n, seed=seed), tmax).astype(np.int32)
    T = int(lens.max())
    x = synthetic.make_features(T, n, seed=seed + 1, lens=lens)[:, :, :240]
    f = oracle.encoder_f32(layers, x, lens)
    tp = (lens + 1) // 2
    res, rl, steps = oracle.greedy_decode(pm, f, tp)
    r = rl / tp
    labels = np.concatenate([res[i, : rl[i]] for i in range(n)])
    return dict(sym_per_frame=float(rl.sum() / lens.sum()), u_tp_pct=np.percentile(r, [10, 50, 90, 99, 100]).round(2).tolist(),
                labels_used=int(len(np.unique(labels))), zero_rows=int((rl == 0).sum()))


if __name__ == "__main__":
    rc = {}
    for a in sys.argv[1:]:
        k, v = a.split("=")
        rc[k] = float(v)
    oracle.lib()
    print(rc, stats(rc))
