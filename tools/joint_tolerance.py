#!/usr/bin/env python3
"""Teacher-forced joint logits: the bf16 GPU decoder vs the fp32 decoder on the same inputs.

north_star: "joint logits within a stated fp tolerance".  For a batch of utterances the int8
encoder output f is computed once on the GPU.  The fp32 greedy decode of f (CPU restatement,
pm32) is the teacher: at every step both decoders see the same frame f[t] and the same
emitted-label history; the bf16 side (the engine's lstm_amx_bf16 / amx_linear_bf16_accum_relu /
amx_linear_i16o32 operators, bf16 weights, its own bf16 prediction state) and the fp32 side
(fp32 weights and state) each produce the 29 logits.  Reports |dL| statistics and, per step,
whether the argmax agrees, binned by the fp32 top-2 margin.

TEST / MEASUREMENT TOOL: uses oracle/ as the fp32 reference.
    python tools/joint_tolerance.py [--model planted|throughput] [--n 32]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rnnt-inference_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402


def teacher_forced(engine, pm, pm32, f, lens, max_steps=None):
    """f: int8 encoder output [Tp, N, 1024] fp32 (host); lens: feature lengths [N].  The bf16
    side runs the torch.ops.intel_mlperf operators on pm's reference-format weights; pm32 should
    be ops.op_model-consistent (its b_hh is the fp32 one, a <= 1 ulp bias difference).
    Returns dict of per-step arrays over active (row, step) pairs: L16, L32 [M, 29]."""
    import torch
    from oracle import oracle
    from rnnt_amd import ops
    from rnnt_amd.config import RNNTParam as R
    W = ops.reference_weights(pm)
    Tp, N, _ = f.shape
    fl = (np.asarray(lens) + 1) // 2
    t = np.zeros(N, np.int64)
    added = np.zeros(N, np.int64)
    fin = fl <= 0
    pre_g = np.full(N, R.SOS, np.int32)
    h32 = np.zeros((2, N, 320), np.float32)
    c32 = np.zeros((2, N, 320), np.float32)
    h16 = torch.zeros((2, N, 320), dtype=torch.bfloat16, device="cuda")
    c16 = torch.zeros((2, N, 320), dtype=torch.float32, device="cuda")
    embed = torch.from_numpy(np.asarray(pm.embed, np.float32)).cuda().to(torch.bfloat16)
    fd = torch.from_numpy(np.ascontiguousarray(f)).cuda()
    out16, out32 = [], []
    steps = 0
    while not fin.all() and (max_steps is None or steps < max_steps):
        steps += 1
        g32, h32n, c32n = oracle.prediction(pm32, pre_g, h32, c32)
        fi = np.stack([f[min(t[n], max(fl[n] - 1, 0)), n] for n in range(N)])
        L32 = oracle.joint(pm32, fi, g32)
        pg = torch.from_numpy(pre_g).cuda()
        sos = pg.eq(R.SOS)
        xg = embed[pg.clamp(min=0).long()].masked_fill(sos[:, None], 0.0)
        g16, hl, cl = ops.lstm_amx_bf16(xg.unsqueeze(0), [h16[0], h16[1]], [c16[0], c16[1]], W["pred"])
        tix = torch.from_numpy(np.minimum(t, np.maximum(fl - 1, 0))).cuda()
        fi16 = fd[tix, torch.arange(N, device="cuda")]
        y1 = ops.amx_linear_bf16_accum_relu(fi16, W["w1_trans"], g16[0], W["w1_pred"], W["bias"])
        L16 = ops.amx_linear_i16o32(y1, W["w2"], W["b2"])[:, : R.num_labels].float().cpu().numpy()
        act = ~fin
        out16.append(L16[act])
        out32.append(L32[act])
        sym = L32.argmax(1)
        emit = act & (sym != R.BLANK) & (added != R.max_symbols_per_step)
        adv = act & ~emit
        if emit.any():
            e = torch.from_numpy(emit).cuda()
            pre_g = np.where(emit, sym, pre_g).astype(np.int32)
            h32[:, emit] = h32n[:, emit]
            c32[:, emit] = c32n[:, emit]
            for l in range(2):
                h16[l][e] = hl[l][e]
                c16[l][e] = cl[l][e]
            added = np.where(emit, added + 1, added)
        t = np.where(adv, t + 1, t)
        added = np.where(adv, 0, added)
        fin = fin | (adv & (t >= fl))
    return dict(L16=np.concatenate(out16), L32=np.concatenate(out32), steps=steps)


def stats(L16, L32, tol_abs, tol_rel):
    d = np.abs(L16 - L32)
    scale = np.abs(L32).max(1, keepdims=True)
    s = np.sort(L32, 1)
    margin = s[:, -1] - s[:, -2]
    tol = tol_abs + tol_rel * scale[:, 0]
    agree = L16.argmax(1) == L32.argmax(1)
    clear = margin > 2 * tol
    return {"pairs": int(len(d)), "max_abs": float(d.max()), "p99_abs": float(np.quantile(d.max(1), 0.99)),
            "max_rel_to_row_scale": float((d / np.maximum(scale, 1e-6)).max()),
            "within_tolerance_frac": float((d.max(1) <= tol).mean()),
            "argmax_agree_frac": float(agree.mean()), "clear_margin_frac": float(clear.mean()),
            "argmax_agree_where_margin_gt_2tol": float(agree[clear].mean()) if clear.any() else None}


def main():
    import torch
    from rnnt_amd import planted, synthetic, weights
    from rnnt_amd.engine import Engine
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="planted", choices=["planted", "throughput"])
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--tol-abs", type=float, default=0.1)
    ap.add_argument("--tol-rel", type=float, default=0.01)
    args = ap.parse_args()
    if args.model == "planted":
        ckpt, task = planted.make_planted_checkpoint()
        lens = np.minimum(synthetic.devclean_lengths(args.n, seed=5), 300)
        feats, _ = planted.planted_features(task, lens, seed=6)
        x = np.zeros((int(lens.max()), args.n, 256), np.float32)
        for i, fe in enumerate(feats):
            x[: len(fe), i, :240] = fe
        amax = weights.calibrate_amax(weights.migrate_state_dict(ckpt), x[:, :8], lens[:8])
    else:
        ckpt = synthetic.make_checkpoint(synthetic.DEFAULT_SEED)
        lens = np.minimum(synthetic.devclean_lengths(args.n, seed=5), 300)
        x = synthetic.make_features(int(lens.max()), args.n, seed=6, lens=lens)
        amax = None
    pm, _ = (weights.prepare_model(ckpt, amax, bf16=True), None) if amax is not None else weights.build_model()
    pm32 = weights.prepare_model(ckpt, pm.amax, bf16=False)
    n_pad = 256
    e = Engine(pm, device=0, max_batch=n_pad, max_frames=int(lens.max()))
    xp = np.zeros((x.shape[0], n_pad, 256), np.float32)
    xp[:, : args.n] = x
    lp = np.zeros(n_pad, np.int32)
    lp[: args.n] = lens
    Tp = (x.shape[0] + 1) // 2
    f = torch.empty((Tp, n_pad, 1024), dtype=torch.float32, device="cuda")
    e.encode(torch.from_numpy(xp).cuda(), torch.from_numpy(lp).cuda(), lens, n=args.n, f_out=f)
    torch.cuda.synchronize()
    r = teacher_forced(e, pm, pm32, f.cpu().numpy()[:, : args.n], lens)
    out = {"model": args.model, "utterances": args.n, "steps": r["steps"], "tol_abs": args.tol_abs,
           "tol_rel": args.tol_rel, **stats(r["L16"], r["L32"], args.tol_abs, args.tol_rel)}
    print(json.dumps(out))
    e.close()


if __name__ == "__main__":
    main()
