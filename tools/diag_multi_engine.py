"""Diagnostic: the round-2 intermittent token mismatch of tests/test_featurizer_gpu.py::
test_server_sut_over_wav_qsl (two engines on one GPU, DynamicBatchServerSUT over GpuWavQSL).

Runs the test's scenario many times in one process and compares EVERY answer -- the Server's
and the single-batch engine.infer's -- with the CPU restatement (oracle) on the same features,
so a mismatch names the wrong side, its sample, batch, engine and repetition.  Variants isolate
the suspects VERDICT r02 lists: (a) two engines overlapping on one device, (b) the 4-deep-ring
tick tiles (RNNT_ENC_TILE=small forces the 2-deep 128x128 tile), (c) the featurizer running on
the worker streams (precomputed features instead).

python tools/diag_multi_engine.py [--reps 12] [--out gpurun_out/diag.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rnnt-inference_amd"))
sys.path.insert(0, REPO)


class PreQSL:
    """QSL over precomputed features [T, n, 256] (cuda): assemble gathers rows on the caller's stream."""

    def __init__(self, x, lens_host):
        self.x, self.lengths = x, np.asarray(lens_host, np.int32)

    def assemble(self, indices, n_pad=None):
        import torch
        from rnnt_amd.engine import pad_batch
        n = len(indices)
        n_pad = n_pad or pad_batch(n)
        bl = self.lengths[list(indices)]
        T = max(int(bl.max()), 1)
        out = torch.zeros((T, n_pad, 256), dtype=torch.float32, device=self.x.device)
        out[:, :n] = self.x[:T].index_select(1, torch.tensor(list(indices), device=self.x.device))
        lp = np.zeros(n_pad, np.int32)
        lp[:n] = bl
        return out, torch.from_numpy(lp).to(self.x.device), bl


def capturing_server(base, warm="none"):
    """DynamicBatchServerSUT whose worker also keeps, per batch, the features the engine encoded
    and the encoder output (host copies), so a wrong answer can be localised to the featurizer,
    the encoder or the decode."""
    import time as _t

    import torch

    class Cap(base):
        def start(self):
            self.captured = {}
            self.seen = set()
            self.first_batch = set()
            super().start()

        def _worker(self, j):
            eng = self.engines[j]
            st = torch.cuda.Stream()
            if warm == "create":  # this thread's featurizer exists (constants uploaded) before its first batch
                self.qsl._featurizer()
                torch.cuda.synchronize()
            elif warm == "full":  # ... and its plan buffer is already at the largest size the test needs
                with torch.cuda.stream(st):
                    self.qsl.assemble(list(range(len(self.qsl.lengths))))
                torch.cuda.synchronize()
            while True:
                batch = self._take()
                if batch is None:
                    return
                try:
                    batch.sort(key=lambda b: -int(self.qsl.lengths[b[1].index]))
                    n = len(batch)
                    with self._cv:
                        bi = len(self.batch_log)
                        self.batch_log.append((j, [s.id for _, s in batch]))
                        first = j not in self.seen
                        self.seen.add(j)
                    with torch.cuda.stream(st):
                        if warm == "nanfill":  # GpuWavQSL.assemble with the output pre-filled with NaN
                            from rnnt_amd.engine import pad_batch
                            q_ = self.qsl
                            idx = np.asarray([b[1].index for b in batch], np.int64)
                            bl = q_.lengths[idx].astype(np.int32)
                            wl = q_.wav_lengths[idx].astype(np.int32)
                            off = torch.from_numpy(q_.offsets[idx]).to(q_.device)
                            xo = torch.full((max(int(bl.max()), 1), pad_batch(n), 256), float("nan"), device="cuda")
                            x, lens = q_._featurizer().featurize(q_.store, torch.from_numpy(wl).to(q_.device), wl, n=n,
                                                                 n_pad=pad_batch(n), T_out=xo.shape[0], offsets=off,
                                                                 out=xo)
                        else:
                            x, lens, bl = self.qsl.assemble([b[1].index for b in batch])
                        res = torch.empty((n, eng.max_res), dtype=torch.int32, device="cuda")
                        rl = torch.empty(n, dtype=torch.int32, device="cuda")
                        f = torch.zeros(((x.shape[0] + 1) // 2, x.shape[1], 1024), dtype=torch.float32, device="cuda")
                    with self._enc_lock:
                        eng.encode(x, lens, bl, n=n, f_out=f, stream=st)
                        st.synchronize()
                    eng.decode(res, rl, stream=st)
                    with torch.cuda.stream(st):
                        rlh = rl.cpu()
                        toks = res[:, : max(1, int(rlh.max()))].cpu().numpy()
                        self.captured[bi] = (x[:, :n].cpu().numpy(), f[:, :n].cpu().numpy(), bl.copy())
                    if first:
                        self.first_batch.add(bi)
                    done = _t.perf_counter()
                    rlh = rlh.numpy()
                    for i, (t0, s) in enumerate(batch):
                        self.responses[s.id] = toks[i, : rlh[i]].copy()
                        self.latency[s.id] = done - t0
                    self.batches += 1
                except Exception as ex:
                    self.errors.append(ex)
                    for t0, s in batch:
                        self.latency[s.id] = float("inf")
    return Cap


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--out", default="gpurun_out/diag.json")
    ap.add_argument("--variants", default="test,one_engine,small_tile,prefeat,infer_only")
    args = ap.parse_args()
    import torch
    from oracle import oracle
    from rnnt_amd import synthetic, weights
    from rnnt_amd.engine import Engine
    from rnnt_amd.sut import DynamicBatchServerSUT, GpuWavQSL, QuerySample

    pm, _ = weights.build_model()
    frames = np.minimum(synthetic.devclean_lengths(24, seed=61), 120)
    wavs = synthetic.make_wavs(synthetic.wav_lengths_for_frames(frames, seed=61), seed=61, device="cuda")
    qsl = GpuWavQSL(wavs)
    n = len(frames)
    x_full, lens_full, bl_full = qsl.assemble(list(range(n)))
    torch.cuda.synchronize()
    feats = np.ascontiguousarray(x_full.cpu().numpy()[:, :n])
    t0 = time.time()
    engines = [Engine(pm, device=0, max_batch=64, max_frames=128) for _ in range(2)]
    max_res = engines[0].max_res
    fo = oracle.encoder_i8(pm, feats, bl_full)
    ro, rlo, _ = oracle.greedy_decode(pm, fo, (bl_full + 1) // 2, max_res=max_res)
    print(f"oracle: {time.time() - t0:.1f} s, res_len {rlo.tolist()}", flush=True)
    oracle_rows = [ro[i, : rlo[i]] for i in range(n)]
    # featurizer batch invariance at these lengths: every 8-row sub-batch's features equal the full batch's
    fz_mismatch = []
    for k in range(0, n, 8):
        idx = list(range(k, min(n, k + 8)))
        xs, _, bls = qsl.assemble(idx)
        torch.cuda.synchronize()
        a = xs.cpu().numpy()
        for r, i in enumerate(idx):
            L = int(bls[r])
            if not np.array_equal(a[:L, r].view(np.uint32), feats[:L, i].view(np.uint32)):
                fz_mismatch.append(i)
    print(f"featurizer sub-batch vs full batch mismatching samples: {fz_mismatch}", flush=True)
    pre = PreQSL(x_full[:, :n].contiguous(), bl_full)

    def first_diff(a, b):
        m = min(len(a), len(b))
        d = np.nonzero(a[:m] != b[:m])[0]
        return int(d[0]) if len(d) else m

    summary = dict(oracle_res_len=rlo.tolist(), featurizer_batch_mismatch=fz_mismatch, variants={})
    for var in args.variants.split(","):
        for e in engines:
            e.set_tile("small" if var == "small_tile" else "auto")
        engs = engines[:1] if var == "one_engine" else engines
        q = pre if var == "prefeat" else qsl
        warm = {"warm_create": "create", "warm_full": "full", "nanfill": "nanfill"}.get(var, "none")
        bad_srv, bad_inf = [], []
        for rep in range(args.reps):
            if var != "infer_only":
                srv = capturing_server(DynamicBatchServerSUT, warm)(engs, q, max_batch=8)
                srv.start()
                samples = [QuerySample(id=i, index=i) for i in range(n)]
                rng = np.random.default_rng(rep)
                for k in range(0, n, 5):
                    srv.issue_query(samples[k:k + 5])
                    time.sleep(float(rng.uniform(0.0, 0.004)))
                deadline = time.time() + 60
                while len(srv.latency) < n and time.time() < deadline:
                    time.sleep(0.005)
                srv.stop()
                if srv.errors or len(srv.responses) != n:
                    bad_srv.append(dict(rep=rep, error=repr(srv.errors[:1]), got=len(srv.responses)))
                    continue
                where = {}
                for bi, (j, ids) in enumerate(srv.batch_log):
                    for r, i in enumerate(ids):
                        where[i] = (bi, j, r, ids)
                for i in range(n):
                    if not np.array_equal(srv.responses[i], oracle_rows[i]):
                        bi, j, r, ids = where[i]
                        xc, fc, blc = srv.captured[bi]
                        L = int(frames[i])
                        Lp = (L + 1) // 2
                        xd = np.nonzero(np.any(xc[:L, r].view(np.uint32) != feats[:L, i].view(np.uint32), axis=1))[0]
                        fd = np.nonzero(np.any(fc[:Lp, r].view(np.uint32) != fo[:Lp, i].view(np.uint32), axis=1))[0]
                        info = dict(rep=rep, sample=i, batch=bi, engine=j, row=r, batch_ids=ids,
                                    workers_first_batch=bi in srv.first_batch,
                                    batches=[(jj, len(ii)) for jj, ii in srv.batch_log],
                                    frames=L, got_len=len(srv.responses[i]), want_len=int(rlo[i]),
                                    first_diff=first_diff(srv.responses[i], oracle_rows[i]),
                                    feat_bad_frames=xd[:8].tolist(), n_feat_bad=int(len(xd)),
                                    enc_bad_frames=fd[:8].tolist(), n_enc_bad=int(len(fd)))
                        if len(xd):
                            xr = xc[:L, r]
                            info["feat_max_abs_err"] = float(np.nanmax(np.abs(xr - feats[:L, i])))
                            nanp = np.argwhere(np.isnan(xc[:, r]))
                            info["nan_count"] = int(len(nanp))
                            info["nan_frames"] = sorted(set(int(v) for v in nanp[:, 0]))[:40]
                            info["nan_channels"] = sorted(set(int(v) for v in nanp[:, 1]))[:40]
                            info["feat_like_sample"] = [int(k) for k in range(n) if int(frames[k]) >= L and
                                                        np.abs(xr - feats[:L, k]).max() < 1e-4]
                            # per 16-frame STFT chunk (frames 16c.. -> spliced rows 16c/3..): which spliced rows differ most
                            e = np.nanmax(np.abs(xr - feats[:L, i]), axis=1)
                            info["feat_worst_frames"] = np.argsort(-e)[:12].tolist()
                            dif = xr.view(np.uint32) != feats[:L, i].view(np.uint32)
                            bch = np.nonzero(dif.any(axis=0))[0]
                            info["bad_channels"] = [int(len(bch)), bch[:12].tolist(), bch[-12:].tolist()]
                            # per corrupted channel, the affine map the normalisation applied fits every frame but
                            # the corrupted ones: the frames off the fit (robust: median slope / intercept)
                            offs = []
                            for cc in bch[:240]:
                                g, b_ = feats[:L, i, cc].astype(np.float64), xr[:, cc].astype(np.float64)
                                A = np.vstack([g, np.ones_like(g)]).T
                                sol = np.linalg.lstsq(A, b_, rcond=None)[0]
                                rsd = np.abs(b_ - A @ sol)
                                tt = int(np.argmax(rsd))
                                offs.append((int(cc), tt, round(float(rsd[tt]), 3)))
                            info["chan_frame_off"] = offs[:80]
                            info["feat_err_by_row_q"] = [float(np.quantile(e, qq)) for qq in (0.0, 0.5, 1.0)]
                        if len(fd):
                            t = int(fd[0])
                            ch = np.nonzero(fc[t, r].view(np.uint32) != fo[t, i].view(np.uint32))[0]
                            info["enc_first_frame_bad_channels"] = ch[:16].tolist()
                            info["enc_first_frame_n_bad"] = int(len(ch))
                            # other rows of the same batch at that frame
                            info["other_rows_bad"] = [int(rr) for rr, ii in enumerate(ids) if rr != r and np.any(
                                fc[:Lp, rr].view(np.uint32) != fo[:Lp, ii].view(np.uint32))]
                        else:  # encoder output right: the decode of the captured frames
                            ro1, rl1, _ = oracle.greedy_decode(pm, np.ascontiguousarray(fc[:, r:r + 1]),
                                                               np.array([Lp], np.int32), max_res=max_res)
                            info["oracle_on_captured_f_ok"] = bool(np.array_equal(ro1[0, :rl1[0]], oracle_rows[i]))
                        bad_srv.append(info)
                        print("MISMATCH", info, flush=True)
            # the test's reference side: one 24-row batch through engine 0 (null stream)
            xq, lq, bq = q.assemble(list(range(n)))
            res = torch.empty((n, max_res), dtype=torch.int32, device="cuda")
            rl = torch.empty(n, dtype=torch.int32, device="cuda")
            engs[0].infer(xq, lq, bq, res, rl, n=n)
            res, rl = res.cpu().numpy(), rl.cpu().numpy()
            for i in range(n):
                if not np.array_equal(res[i, : rl[i]], oracle_rows[i]):
                    bad_inf.append(dict(rep=rep, sample=i, got_len=int(rl[i]), want_len=int(rlo[i]),
                                        first_diff=first_diff(res[i, : rl[i]], oracle_rows[i])))
            print(f"[{var}] rep {rep}: server mismatches {len(bad_srv)}, infer mismatches {len(bad_inf)}", flush=True)
        summary["variants"][var] = dict(reps=args.reps, server_bad=bad_srv, infer_bad=bad_inf)
    for e in engines:
        e.close()
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps({k: dict(server_bad=len(v["server_bad"]), infer_bad=len(v["infer_bad"]))
                      for k, v in summary["variants"].items()}), flush=True)


if __name__ == "__main__":
    main()
