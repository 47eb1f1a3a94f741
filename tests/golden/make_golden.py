"""Generate tests/golden/golden.npz from the REFERENCE's own Python modules.

Build-container only (it imports /root/reference/models, which never travels to the GPU box):
    python -B tests/golden/make_golden.py
The committed .npz holds only data (inputs, expected outputs, quantisation parameters); the
weights are regenerated from the seed by rnnt_amd.synthetic (digest stored to catch drift).

The reference's native op library (the `mlperf_plugins` submodule, absent: reference
.gitmodules:1-3) is replaced by a stand-in `_C` providing only what the fp32 path reaches:
`prepack_lstm_weights` (identity) and `lstm` (a textbook LSTM, gates = linear(x,W_ih,b_ih) +
linear(h,W_hh,b_hh), i,f,g,o order).  Everything else exercised here -- QuantLSTMLayer
(f32 / calib / fake_quant), StackTime.forward_f32, the fp32 Joint, greedy_decode_f32, the
split_len chunking, TensorQuantizer calibration, iLSTMLayer._quant_parameters and the quant
scale propagation -- is the reference's own code.
"""
import hashlib
import os
import sys
import tempfile
import types

sys.dont_write_bytecode = True  # never write __pycache__ into /root/reference
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF_MODELS = "/root/reference/models"
OUT = os.path.join(REPO, "tests", "golden", "golden.npz")

sys.path.insert(0, os.path.join(REPO, "rnnt-inference_amd"))
from rnnt_amd import synthetic  # noqa: E402
from rnnt_amd.synthetic import DEFAULT_SEED  # noqa: E402

# ---- stand-in for the absent plugin (fp32 prediction LSTM only) ----
_stub = types.ModuleType("_C")


def _prepack_lstm_weights(w_ih, w_hh):
    return w_ih, w_hh


def _lstm(x, hx, cx, weights):
    ys = []
    hy, cy = list(hx), list(cx)
    for t in range(x.shape[0]):
        inp = x[t]
        for l, (w_ih, w_hh, b_ih, b_hh) in enumerate(weights):
            gates = F.linear(inp, w_ih, b_ih) + F.linear(hy[l], w_hh, b_hh)
            i, f, g, o = gates.chunk(4, 1)
            cy[l] = torch.sigmoid(f) * cy[l] + torch.sigmoid(i) * torch.tanh(g)
            hy[l] = torch.sigmoid(o) * torch.tanh(cy[l])
            inp = hy[l]
        ys.append(inp)
    return torch.stack(ys, 0), hy, cy


_stub.prepack_lstm_weights = _prepack_lstm_weights
_stub.lstm = _lstm
sys.modules["_C"] = _stub
sys.path.insert(0, REF_MODELS)
import decoder as ref_decoder  # noqa: E402
import modeling_rnnt as ref_model  # noqa: E402
import quant_lstm as ref_ql  # noqa: E402
import quant_modules as ref_qm  # noqa: E402


def _check_no_pycache():
    assert not os.path.exists(os.path.join(REF_MODELS, "__pycache__")), "wrote into the reference!"


def unpack_tiled_int8(packed, rows_in, cols_in, padding):
    """Invert quant_modules.transpose_tile_weight(W^T, padding) -> natural W [cols_in, rows_pad]."""
    idx = torch.arange(1, rows_in * cols_in + 1, dtype=torch.int64).reshape(rows_in, cols_in)
    pidx = ref_qm.transpose_tile_weight(idx, padding).reshape(-1)
    flat = packed.reshape(-1).to(torch.int64)
    rows_pad = ((rows_in + 63) // 64) * 64 if padding else rows_in
    wt = torch.zeros(rows_pad * cols_in, dtype=torch.int64)
    sel = pidx > 0
    src = pidx[sel] - 1  # index into the unpadded [rows_in, cols_in] W^T
    r, c = src // cols_in, src % cols_in
    wt[r * cols_in + c] = flat[sel]
    return wt.reshape(rows_pad, cols_in).t().contiguous().to(torch.int8)  # [cols_in, rows_pad]


def main():
    torch.manual_seed(0)
    torch.set_num_threads(8)
    seed = DEFAULT_SEED
    ckpt_np = synthetic.make_checkpoint(seed)
    digest = synthetic.checkpoint_digest(ckpt_np)
    tmp = tempfile.mkdtemp()
    ck_path = os.path.join(tmp, "rnnt.pt")
    torch.save({k: torch.from_numpy(v.copy()) for k, v in ckpt_np.items()}, ck_path)
    out = {"seed": np.int64(seed), "digest": np.frombuffer(digest.encode(), np.uint8)}

    # ---------------- fp32 end-to-end (config 1 style plumbing + a 4-utterance batch) -------
    T, N = 60, 4
    lens = np.array([60, 51, 33, 8], np.int32)
    x = synthetic.make_features(T, N, seed=1, lens=lens)[:, :, :240]
    out["a_x"], out["a_lens"] = x, lens
    rnnt = ref_model.RNNT(ck_path, "f32").eval()
    with torch.no_grad():
        dec = ref_decoder.GreedyDecoder(rnnt, "f32", False, -1, N)
        res, res_len = dec(torch.from_numpy(x.copy()), torch.from_numpy(lens.astype(np.int64)))
        out["a_f32_res"], out["a_f32_len"] = res.numpy().astype(np.int32), res_len.numpy().astype(np.int32)
        out["a_f32_steps"] = dec.step.numpy().astype(np.int32)  # [N,2] (advance, emit) debug counters
        z = lambda: [torch.zeros(N, 1024) for _ in range(5)]  # noqa: E731
        zs = z()
        f, *_ = rnnt.transcription(torch.from_numpy(x.copy()), torch.from_numpy(lens.astype(np.int64)),
                                   zs[:2], zs[:2], zs[2:], zs[2:])
        out["a_f32_f"] = f.numpy()
        dec2 = ref_decoder.GreedyDecoder(rnnt, "f32", False, 2, N)
        res2, len2 = dec2(torch.from_numpy(x.copy()), torch.from_numpy(lens.astype(np.int64)))
        out["a_f32_split2_res"], out["a_f32_split2_len"] = res2.numpy().astype(np.int32), len2.numpy().astype(np.int32)
        # single utterance (BASELINE config 1 shape)
        T1 = 245
        x1 = synthetic.make_features(T1, 1, seed=11)[:, :, :240]
        d1 = ref_decoder.GreedyDecoder(rnnt, "f32", False, -1, 1)
        r1, l1 = d1(torch.from_numpy(x1.copy()), torch.tensor([T1], dtype=torch.int64))
        out["c1_x"], out["c1_res"], out["c1_len"] = x1, r1.numpy().astype(np.int32), l1.numpy().astype(np.int32)
    print("f32 lens", out["a_f32_len"], "split2", out["a_f32_split2_len"], "c1", out["c1_len"])

    # ---------------- calibration (run_mode calib) ----------------
    calib_n, calib_T = 2, 120
    cl = np.full(calib_n, calib_T, np.int32)
    xc = synthetic.make_features(calib_T, calib_n, seed=seed ^ 0xCA1B, lens=cl)[:, :, :240]
    rc = ref_model.RNNT(ck_path, "calib").eval()
    with torch.no_grad():
        dc = ref_decoder.GreedyDecoder(rc, "calib", False, -1, calib_n)
        dc(torch.from_numpy(xc.copy()), torch.from_numpy(cl.astype(np.int64)))
    sd = rc.state_dict()
    amax = []
    for stack, nl in (("pre_rnn", 2), ("post_rnn", 3)):
        for l in range(nl):
            amax.append(float(sd[f"transcription.{stack}.lstm{l}.input_quantizer._amax"]))
    out["calib_amax"] = np.array(amax, np.float32)
    calib_path = os.path.join(tmp, "rnnt_calib.pt")
    torch.save(sd, calib_path)
    print("amax", out["calib_amax"])

    # ---------------- quant model parameters (run_mode quant, bf16) ----------------
    rq = ref_model.RNNT(calib_path, "quant", enable_bf16=True).eval()
    layer = 0
    for stack, nl, in0 in (("pre_rnn", 2, 240), ("post_rnn", 3, 2048)):
        m = getattr(rq.transcription, stack)
        for l in range(nl):
            w_ih_p, w_hh_p, b_ih, b_q = m.weights[l]
            isz = in0 if l == 0 else 1024
            w_ih = unpack_tiled_int8(w_ih_p, isz, 4096, padding=(layer == 0))
            w_hh = unpack_tiled_int8(w_hh_p, 1024, 4096, padding=False)
            w = torch.cat([w_ih, w_hh], 1).numpy()
            out[f"q_w{layer}_sha"] = np.frombuffer(hashlib.sha256(w.tobytes()).hexdigest().encode(), np.uint8)
            out[f"q_w{layer}_rows"] = w[::257].copy()
            out[f"q_bq{layer}"] = b_q.detach().numpy().astype(np.float32)
            layer += 1
        out[f"q_{stack}_rb"] = m.rb_scale.numpy().astype(np.float32)
        out[f"q_{stack}_in"] = m.in_scale.numpy().astype(np.float32)
        out[f"q_{stack}_out"] = m.out_scale.numpy().astype(np.float32)
    out["q_joint_b1"] = rq.joint.linear1_bias.detach().numpy().astype(np.float32)
    out["q_joint_b2"] = rq.joint.linear2.bias.detach().numpy().astype(np.float32)

    # ---------------- fake_quant end-to-end (float restatement of the int8 path) -----------
    # QuantLSTM.__init__ skips iLSTM.__init__ (quant_lstm.py:106-107), so run_mode
    # "fake_quant" dies on the missing `weights` / `rb_scale` attributes that
    # _process_parameters passes along (quant_lstm.py:56-60).  Add exactly those two
    # attributes; nothing numeric changes.
    orig_init = ref_ql.QuantLSTM.__init__

    def _init(self, *a, **k):
        orig_init(self, *a, **k)
        self.weights = []
        self.rb_scale = torch.zeros(self.num_layers)

    ref_ql.QuantLSTM.__init__ = _init
    rf = ref_model.RNNT(calib_path, "fake_quant").eval()
    ref_ql.QuantLSTM.__init__ = orig_init
    with torch.no_grad():
        df = ref_decoder.GreedyDecoder(rf, "f32", False, -1, N)
        res, res_len = df(torch.from_numpy(x.copy()), torch.from_numpy(lens.astype(np.int64)))
        out["a_fq_res"], out["a_fq_len"] = res.numpy().astype(np.int32), res_len.numpy().astype(np.int32)
        zs = z()
        f, *_ = rf.transcription(torch.from_numpy(x.copy()), torch.from_numpy(lens.astype(np.int64)),
                                 zs[:2], zs[:2], zs[2:], zs[2:])
        out["a_fq_f"] = f.numpy()
    print("fake_quant lens", out["a_fq_len"])

    # ---------------- the 30-symbols-per-frame cap (decoder.py:131-136, 153-167) ----------------
    # A checkpoint variant (synthetic.CAP_RECIPE) whose joint prefers one non-blank label on some
    # frames whatever the prediction: the reference's greedy_decode_f32 emits 30 symbols there and
    # the cap forces the advance.  The joint is wrapped to count those forced advances per row
    # (symbols_added == max_symbols_per_step, argmax non-blank, row not finished), and the
    # generator asserts that they happen, beside blank advances, on most rows.
    cap_ck = synthetic.make_checkpoint(seed, synthetic.CAP_RECIPE)
    out["cap_digest"] = np.frombuffer(synthetic.checkpoint_digest(cap_ck).encode(), np.uint8)
    cap_path = os.path.join(tmp, "rnnt_cap.pt")
    torch.save({k: torch.from_numpy(v.copy()) for k, v in cap_ck.items()}, cap_path)
    Tc, Nc = 60, 6
    cap_lens = np.array([60, 53, 40, 29, 9, 3], np.int32)
    xcap = synthetic.make_features(Tc, Nc, seed=7, lens=cap_lens)[:, :, :240]
    rcap = ref_model.RNNT(cap_path, "f32").eval()
    dcap = ref_decoder.GreedyDecoder(rcap, "f32", False, -1, Nc)
    caps = np.zeros(Nc, np.int32)
    joint = rcap.joint

    class _CountCaps(torch.nn.Module):
        def forward(self, fi, g, padded):
            y = joint(fi, g, padded)
            sym = torch.argmax(y, dim=1)
            hit = dcap.symbols_added.eq(30) & sym.ne(28) & ~dcap.finish
            caps[:] += hit.numpy()[:Nc].astype(np.int32)
            return y

    rcap.joint = _CountCaps()
    with torch.no_grad():
        res, res_len = dcap(torch.from_numpy(xcap.copy()), torch.from_numpy(cap_lens.astype(np.int64)))
        zs = [torch.zeros(Nc, 1024) for _ in range(5)]
        rcap.joint = joint
        fcap, *_ = rcap.transcription(torch.from_numpy(xcap.copy()), torch.from_numpy(cap_lens.astype(np.int64)),
                                      zs[:2], zs[:2], zs[2:], zs[2:])
    steps = dcap.step.numpy().astype(np.int32)
    assert caps.max() > 0 and (caps > 0).sum() >= 3, f"no row hits the 30-symbol cap: {caps}"
    assert (steps[:, 0] > caps).sum() >= 3, "cap rows also need blank advances (a mixed decode)"
    out["cap_x"], out["cap_lens"] = xcap, cap_lens
    out["cap_f32_res"], out["cap_f32_len"] = res.numpy().astype(np.int32), res_len.numpy().astype(np.int32)
    out["cap_f32_steps"], out["cap_f32_caps"] = steps, caps
    out["cap_f32_f"] = fcap.numpy()
    print("cap lens", out["cap_f32_len"], "caps", caps, "steps", steps.tolist())
    _check_no_pycache()
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
