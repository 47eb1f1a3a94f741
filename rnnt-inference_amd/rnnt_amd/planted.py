"""A well-conditioned synthetic RNN-T ("planted transducer") for the accuracy criterion.

The north_star asks for WER within 1 % of the fp32 reference.  No trained checkpoint or
LibriSpeech is available offline, and the throughput model of ``synthetic.make_checkpoint``
is a random-init network whose encoder recurrence is chaotic (int8 quantisation noise grows
along the utterance) and whose joint decisions sit at bf16-rounding margins -- on it no
precision comparison is meaningful.  This module builds a network of the exact reference
architecture whose behaviour resembles a trained model's, so the int8 + bf16 path can be
measured against fp32 the way the reference's accuracy run would be:

* **Speech stand-in.**  An utterance is a sequence of segments, one per character of a
  random word-like transcript (letters, apostrophes, spaces between 2-7 letter words), each
  segment 6-14 feature frames of that label's 240-d prototype plus noise, with short silence
  segments between words.  Features are ~N(0, 1) per channel like normalised log-mels.
* **Encoder: contractive.**  Small recurrent weights and a negative forget-gate bias make every
  LSTM layer forget within a few frames, so the encoder output is a smooth function of the last
  few inputs (a trained acoustic encoder is stable in this sense; a chaotic one amplifies any
  rounding).
* **Joint: confident.**  Hidden units 0..27 compute ``relu(M * s_k(f) - M * r_k(g))``: s_k is a
  ridge-regression read-out of "inside a segment of label k" from the fp32 encoder output,
  r_k a read-out of "the last emitted label is k" from the prediction output.  linear2 passes
  unit k to label k, blank has a constant logit M/2.  Inside a segment its label wins by ~M/2
  until it is emitted, then blank wins by ~M/2 -- the margins of a trained model, not of a
  random one.  The other 484 hidden units are random features with a small linear2 weight.

``make_planted_checkpoint`` returns a checkpoint in the original key format (it goes through
``migrate_state_dict`` / calibration / quantisation like any other) plus the generator of its
synthetic utterances and their ground-truth transcripts.  Everything is seeded and computed in
numpy; the read-outs are fitted on fp32 outputs, never on the quantised path being measured.
"""
from dataclasses import dataclass

import numpy as np

from .config import RNNTParam as R

LETTERS = list(range(1, 27))  # a..z
APOS, SPACE, BLANK = 27, 0, R.BLANK


def _sig(x):
    return 1.0 / (1.0 + np.exp(-x))


def lstm_layer_f32(x, wih, whh, bih, bhh, lens=None):
    """torch.nn.LSTM single layer (gate order i, f, g, o), numpy fp32: x [T, N, I] -> y [T, N, H]."""
    T, N, _ = x.shape
    H = whh.shape[1]
    h = np.zeros((N, H), np.float32)
    c = np.zeros((N, H), np.float32)
    y = np.empty((T, N, H), np.float32)
    xw = (x.reshape(T * N, -1) @ wih.T).reshape(T, N, 4 * H) + (bih + bhh)
    for t in range(T):
        g = xw[t] + h @ whh.T
        i, f, gg, o = np.split(g, 4, axis=1)
        c = _sig(f) * c + _sig(i) * np.tanh(gg)
        h = (_sig(o) * np.tanh(c)).astype(np.float32)
        y[t] = h
    return y


def transcription_f32(sd, x, lens):
    """Transcription.forward in fp32 (modeling_rnnt.py:116-144) on a migrated state dict:
    x [T, N, 240] -> f [ceil(T/2), N, 1024]."""
    from .weights import enc_layer_params
    y = np.asarray(x, np.float32)
    for layer in range(5):
        if layer == 2:  # StackTime.forward_f32 (modeling_rnnt.py:314-324)
            T, N, C = y.shape
            y = y.copy()
            for n in range(N):
                y[int(lens[n]):, n, :] = 0
            if T % 2:
                y = np.concatenate([y, np.zeros((1, N, C), np.float32)], 0)
            y = y.reshape(y.shape[0] // 2, 2, N, C).transpose(0, 2, 1, 3).reshape(y.shape[0] // 2, N, 2 * C)
        y = lstm_layer_f32(y, *enc_layer_params(sd, layer))
    return y


def prediction_f32(sd, labels):
    """Prediction.forward over a label sequence (SOS first, modeling_rnnt.py:183-205), fp32:
    labels [U, N] int (-1 = SOS) -> g [U, N, 320] (the output after consuming each label)."""
    P = R.pred_hidden_size
    emb = sd["prediction.embed.weight"]
    U, N = labels.shape
    x = np.where(labels[..., None] >= 0, emb[np.maximum(labels, 0)], 0.0).astype(np.float32)
    for l in range(R.pred_num_layers):
        p = "prediction.pred_rnn."
        x = lstm_layer_f32(x, sd[p + f"weight_ih_l{l}"], sd[p + f"weight_hh_l{l}"], sd[p + f"bias_ih_l{l}"],
                           sd[p + f"bias_hh_l{l}"])
    assert x.shape[-1] == P
    return x


@dataclass
class PlantedTask:
    protos: np.ndarray      # [29, 240] label prototypes (28 = silence)
    noise: float
    seg_frames: tuple       # (min, max) feature frames per character segment
    sil_frames: tuple       # (min, max) feature frames of a silence segment

    def transcript(self, rng, n_chars):
        """A word-like character sequence (no two equal neighbours: one segment = one emission)."""
        out = []
        while len(out) < n_chars:
            if out:
                out.append(SPACE)
            for _ in range(int(rng.integers(2, 8))):
                while True:
                    ch = int(rng.choice(LETTERS)) if rng.random() > 0.03 else APOS
                    if not out or ch != out[-1]:
                        break
                out.append(ch)
        out = out[:n_chars]
        while out and out[-1] == SPACE:
            out.pop()
        return out

    def utterance(self, rng, frames):
        """Features [frames, 240] and the ground-truth label sequence of one utterance."""
        mean_seg = 0.5 * (self.seg_frames[0] + self.seg_frames[1])
        n_chars = max(1, int(frames / (mean_seg * 1.25)))
        labels = self.transcript(rng, n_chars)
        segs = [(BLANK, int(rng.integers(*self.sil_frames)))]
        for ch in labels:
            segs.append((ch, int(rng.integers(self.seg_frames[0], self.seg_frames[1] + 1))))
            if ch == SPACE or rng.random() < 0.15:
                segs.append((BLANK, int(rng.integers(*self.sil_frames))))
        seq = np.concatenate([np.full(n, lab, np.int64) for lab, n in segs])
        if len(seq) < frames:
            seq = np.concatenate([seq, np.full(frames - len(seq), BLANK, np.int64)])
        seq = seq[:frames]
        # the characters whose segments made it into the utterance (a truncated last segment
        # shorter than 4 frames may legitimately go undetected: drop it from the truth)
        truth, run, prev = [], 0, None
        for lab in list(seq) + [None]:
            if lab == prev:
                run += 1
                continue
            if prev is not None and prev != BLANK and (run >= 4 or lab is not None):
                truth.append(int(prev))
            prev, run = lab, 1
        x = self.protos[seq] + self.noise * rng.standard_normal((frames, self.protos.shape[1])).astype(np.float32)
        return x.astype(np.float32), truth


def planted_features(task, lengths, seed):
    """-> (list of [T_i, 240] fp32 features, list of ground-truth label lists)."""
    rng = np.random.default_rng(seed)
    feats, truths = [], []
    for T in np.asarray(lengths, np.int64):
        x, tr = task.utterance(rng, int(T))
        feats.append(x)
        truths.append(tr)
    return feats, truths


def _batch(feats):
    lens = np.array([len(f) for f in feats], np.int32)
    x = np.zeros((int(lens.max()), len(feats), R.trans_input_size), np.float32)
    for i, f in enumerate(feats):
        x[: len(f), i] = f
    return x, lens


def _frame_labels(task, feats, lens):
    """Per stacked encoder frame, the label whose prototype dominates its two feature frames."""
    d = [np.argmin(((f[:, None, :] - task.protos[None]) ** 2).sum(-1), 1) for f in feats]
    Tp = (int(lens.max()) + 1) // 2
    lab = np.full((Tp, len(feats)), -1, np.int64)
    for n, dn in enumerate(d):
        for tp in range((len(dn) + 1) // 2):
            lab[tp, n] = dn[2 * tp + 1] if 2 * tp + 1 < len(dn) else dn[2 * tp]
    return lab


def make_planted_checkpoint(seed=0x504C4E54, margin=8.0, fit_utts=48, fit_frames=(120, 260)):
    """-> (checkpoint in the original key format, PlantedTask)."""
    rng = np.random.default_rng(seed)
    H, P, J, L, I0 = R.trans_hidden_size, R.pred_hidden_size, R.joint_hidden_size, R.num_labels, R.trans_input_size

    def U(shape, scale):
        return rng.uniform(-scale, scale, size=shape).astype(np.float32)

    sd = {}
    for stack, n_layers, in0 in (("pre_rnn", 2, I0), ("post_rnn", 3, 2 * H)):
        for l in range(n_layers):
            isz = in0 if l == 0 else H
            p = f"encoder.{stack}.lstm."
            sd[p + f"weight_ih_l{l}"] = U((4 * H, isz), 1.6 / np.sqrt(isz))
            sd[p + f"weight_hh_l{l}"] = U((4 * H, H), 0.35 / np.sqrt(H))
            b = U((4 * H,), 0.1)
            b[H: 2 * H] -= 2.0  # forget gate: forget within a few frames (contractive state)
            sd[p + f"bias_ih_l{l}"] = b
            sd[p + f"bias_hh_l{l}"] = U((4 * H,), 0.1)
    sd["prediction.embed.weight"] = U((L - 1, P), 1.0)
    for l in range(2):
        p = "prediction.dec_rnn.lstm."
        sd[p + f"weight_ih_l{l}"] = U((4 * P, P), 1.5 / np.sqrt(P))
        sd[p + f"weight_hh_l{l}"] = U((4 * P, P), 0.3 / np.sqrt(P))
        b = U((4 * P,), 0.1)
        b[P: 2 * P] -= 2.0
        sd[p + f"bias_ih_l{l}"] = b
        sd[p + f"bias_hh_l{l}"] = U((4 * P,), 0.1)
    task = PlantedTask(protos=(0.85 * rng.standard_normal((L, I0))).astype(np.float32), noise=0.5,
                       seg_frames=(6, 14), sil_frames=(3, 9))

    # --- s_k: "inside a segment of label k" read-out of the fp32 encoder output (ridge)
    from .weights import migrate_state_dict
    msd = migrate_state_dict(dict(sd, **{"joint_net.0.weight": np.zeros((J, H + P), np.float32),
                                        "joint_net.0.bias": np.zeros(J, np.float32)}))
    lens = rng.integers(fit_frames[0], fit_frames[1] + 1, size=fit_utts)
    feats, _ = planted_features(task, lens, seed + 1)
    x, lens = _batch(feats)
    f = transcription_f32(msd, x, lens)
    lab = _frame_labels(task, feats, lens)
    keep = lab >= 0
    X = f[keep].astype(np.float64)
    Y = np.zeros((X.shape[0], L - 1))
    lk = lab[keep]
    Y[np.arange(len(lk))[lk < BLANK], lk[lk < BLANK]] = 1.0
    Xa = np.concatenate([X, np.ones((X.shape[0], 1))], 1)
    A = Xa.T @ Xa + 1e-2 * np.eye(Xa.shape[1])
    Ws = np.linalg.solve(A, Xa.T @ Y)                    # [H+1, 28]
    # --- r_k: "last emitted label is k" read-out of the prediction output
    U_, N_ = 12, 400
    seqs = rng.integers(0, L - 1, size=(U_, N_))
    seqs[0] = -1
    g = prediction_f32(msd, seqs)
    Xg = np.concatenate([g.reshape(-1, P), np.ones((U_ * N_, 1))], 1).astype(np.float64)
    Yg = np.zeros((U_ * N_, L - 1))
    flat = seqs.reshape(-1)
    Yg[np.arange(len(flat))[flat >= 0], flat[flat >= 0]] = 1.0
    Wr = np.linalg.solve(Xg.T @ Xg + 1e-3 * np.eye(P + 1), Xg.T @ Yg)  # [P+1, 28]

    W1 = np.zeros((J, H + P), np.float64)
    b1 = np.zeros(J, np.float64)
    W1[: L - 1, :H] = margin * Ws[:H].T
    W1[: L - 1, H:] = -margin * Wr[:P].T
    b1[: L - 1] = margin * (Ws[H] - Wr[P])
    W1[L - 1:, :H] = rng.uniform(-1, 1, size=(J - L + 1, H)) / np.sqrt(H)   # random texture units
    W1[L - 1:, H:] = rng.uniform(-1, 1, size=(J - L + 1, P)) / np.sqrt(P)
    W2 = np.zeros((L, J), np.float64)
    W2[: L - 1, : L - 1] = np.eye(L - 1)
    W2[:, L - 1:] = rng.uniform(-1, 1, size=(L, J - L + 1)) * (0.05 * margin / np.sqrt(J))
    b2 = np.zeros(L, np.float64)
    b2[BLANK] = 0.5 * margin
    sd["joint_net.0.weight"] = W1.astype(np.float32)
    sd["joint_net.0.bias"] = b1.astype(np.float32)
    sd["joint_net.3.weight"] = W2.astype(np.float32)
    sd["joint_net.3.bias"] = b2.astype(np.float32)
    return sd, task
