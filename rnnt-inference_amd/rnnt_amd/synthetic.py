"""Synthetic RNN-T checkpoints, features and LibriSpeech-shaped lengths.

The trained checkpoint (reference ``run.sh:30``) and LibriSpeech are not available offline,
so every run uses random-init weights of the exact architecture, produced by a portable
counter-based PRNG (splitmix64) so any tool can regenerate them bit-exactly from a seed.

The checkpoint uses the ORIGINAL key format that ``migrate_state_dict``
(reference ``models/utils.py:60-81``) consumes.  Weight scales follow the recipe recorded in
SURVEY 8c (plain default-init weights give degenerate decodes): encoder LSTM weights
U(+-4/sqrt(H)), joint fc1 std 0.1, fc2 std 0.3 and a positive blank bias, tuned so greedy
decoding emits a LibriSpeech-like ~0.5 symbols per encoder frame and stays input-dependent.
"""
import math

import numpy as np

from .config import RNNTParam as R

DEFAULT_SEED = 0x524E4E54  # "RNNT"

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix_uniform(seed, n, lo=-1.0, hi=1.0):
    """n float32 uniforms in [lo, hi) from splitmix64(seed + i*golden) (24-bit mantissas)."""
    i = np.arange(1, n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(40)).astype(np.float64) * (1.0 / (1 << 24))  # [0,1), 24 bits exact
    return (lo + (hi - lo) * u).astype(np.float32)


def _tensor(seed, key_id, shape, scale):
    n = int(np.prod(shape))
    return (splitmix_uniform(seed * 1000003 + key_id * 7919, n) * np.float32(scale)).reshape(shape)


# recipe parameters (see module docstring); blank_bias sets the emission rate, anti_repeat
# the strength of the planted "label already emitted" suppression (see _plant_anti_repeat)
RECIPE = dict(enc=4.0 / 32.0, pred=2.0 / np.sqrt(320.0), embed=1.7, fc1=0.1 * np.sqrt(3.0),
              fc1_b=0.05, fc2=0.3 * np.sqrt(3.0), fc2_b=0.1, blank_bias=13.0, anti_repeat=2.0,
              fc1_pred_noise=0.2, fc1_pred_scale=1.0)


# A checkpoint whose joint is decided by the encoder frame alone (prediction half x0.3, no planted
# anti-repeat prior, blank bias 7): on some frames one non-blank label wins every time, so the
# frame emits max_symbols_per_step (30) symbols and the cap forces the advance
# (reference decoder.py:131-136, 153-167); other frames are blank.  tests/golden/make_golden.py
# asserts that the reference's greedy_decode_f32 hits the cap on it.
CAP_RECIPE = dict(anti_repeat=0.0, fc1_pred_scale=0.3, blank_bias=7.0)


def _plant_anti_repeat(sd, gamma, noise):
    """Fit the joint's prediction half W1p so that the prediction output after emitting label
    s pushes the joint hidden against label s's output row (G_s ~ -gamma * W2[s]).

    Purely random weights make greedy decoding degenerate (every frame emits the same label
    30 times); a trained transducer has learnt that an emitted label has consumed
    its acoustic evidence.  Planting that one prior gives LibriSpeech-like decodes (mostly
    blanks, ~0.47 symbols per encoder frame on dev-clean-shaped input -- LibriSpeech has ~0.45 --
    and all labels used).  Computed in float64 without
    BLAS-order sensitivity beyond 1e-16 and rounded once to float32, so every host regenerates
    the same weights (tests/golden stores a checkpoint hash to catch any drift)."""
    H, P = R.trans_hidden_size, R.pred_hidden_size
    sig = lambda v: 1.0 / (1.0 + np.exp(-v))  # noqa: E731
    emb = sd["prediction.embed.weight"].astype(np.float64)
    phis = []
    for s in range(R.num_labels - 1):
        x = emb[s]
        for l in range(R.pred_num_layers):
            pre = "prediction.dec_rnn.lstm."
            g = (sd[pre + f"weight_ih_l{l}"].astype(np.float64) * x[None, :]).sum(1) \
                + sd[pre + f"bias_ih_l{l}"].astype(np.float64) + sd[pre + f"bias_hh_l{l}"].astype(np.float64)
            i, f, gg, o = np.split(g, 4)
            c = sig(i) * np.tanh(gg)
            x = sig(o) * np.tanh(c)
        phis.append(x)
    phi = np.stack(phis, 1)                                   # [P, 28]
    gram = (phi[:, :, None] * phi[:, None, :]).sum(0)         # [28, 28]
    pinv = np.linalg.solve(gram + 1e-9 * np.eye(gram.shape[0]), phi.T)  # [28, P]
    u = sd["joint_net.3.weight"][: R.num_labels - 1].astype(np.float64).T  # [512, 28]
    w1p = -gamma * (u[:, :, None] * pinv[None, :, :]).sum(1)  # [512, P]: G_s ~ -gamma W2[s]
    w = sd["joint_net.0.weight"]
    w[:, H:] = (w1p + noise * w[:, H:].astype(np.float64)).astype(np.float32)


def make_checkpoint(seed=DEFAULT_SEED, recipe=None):
    """Random RNN-T state dict in the original checkpoint key format (numpy float32)."""
    rc = dict(RECIPE)
    if recipe:
        rc.update(recipe)
    H, P, J, L = R.trans_hidden_size, R.pred_hidden_size, R.joint_hidden_size, R.num_labels
    sd = {}
    kid = 0

    def add(key, shape, scale):
        nonlocal kid
        kid += 1
        sd[key] = _tensor(seed, kid, shape, scale)

    for stack, n_layers, in0 in (("pre_rnn", 2, R.trans_input_size), ("post_rnn", 3, 2 * H)):
        for l in range(n_layers):
            isz = in0 if l == 0 else H
            pre = f"encoder.{stack}.lstm."
            add(pre + f"weight_ih_l{l}", (4 * H, isz), rc["enc"])
            add(pre + f"weight_hh_l{l}", (4 * H, H), rc["enc"])
            add(pre + f"bias_ih_l{l}", (4 * H,), rc["enc"])
            add(pre + f"bias_hh_l{l}", (4 * H,), rc["enc"])
    add("prediction.embed.weight", (L - 1, P), rc["embed"])
    for l in range(2):
        pre = "prediction.dec_rnn.lstm."
        add(pre + f"weight_ih_l{l}", (4 * P, P), rc["pred"])
        add(pre + f"weight_hh_l{l}", (4 * P, P), rc["pred"])
        add(pre + f"bias_ih_l{l}", (4 * P,), rc["pred"])
        add(pre + f"bias_hh_l{l}", (4 * P,), rc["pred"])
    add("joint_net.0.weight", (J, H + P), rc["fc1"])
    add("joint_net.0.bias", (J,), rc["fc1_b"])
    add("joint_net.3.weight", (L, J), rc["fc2"])
    add("joint_net.3.bias", (L,), rc["fc2_b"])
    sd["joint_net.3.bias"][R.BLANK] += np.float32(rc["blank_bias"])
    if rc["anti_repeat"]:
        _plant_anti_repeat(sd, rc["anti_repeat"], rc["fc1_pred_noise"])
    if rc["fc1_pred_scale"] != 1.0:  # weaken (or strengthen) the prediction network's say in the joint
        sd["joint_net.0.weight"][:, H:] *= np.float32(rc["fc1_pred_scale"])
    return sd


def checkpoint_digest(sd):
    """sha256 over the checkpoint tensors (key-sorted) to detect cross-host drift."""
    import hashlib
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(np.ascontiguousarray(sd[k], np.float32).tobytes())
    return h.hexdigest()


def make_features(T, N, seed, channels=R.PADDED_INPUT_SIZE, lens=None):
    """Synthetic normalised log-mel features [T, N, channels] ~ N(0,1) on the 240 real
    channels (per-feature normalisation), zeros in the 16 pad channels and past lens[n]
    (the QSL's AssembleSamples layout, rnnt_qsl.cpp:150-188)."""
    rng = np.random.default_rng(seed)
    x = np.zeros((T, N, channels), dtype=np.float32)
    x[:, :, : R.trans_input_size] = rng.standard_normal((T, N, R.trans_input_size), dtype=np.float32)
    if lens is not None:
        for n, ln in enumerate(lens):
            x[int(ln):, n, :] = 0.0
    return x


def devclean_lengths(count, seed, max_frames=R.MAX_FEA_LEN, min_frames=47):
    """Feature lengths (30 ms frames) of a LibriSpeech-dev-clean-shaped QSL: log-normal
    durations (median 6.2 s, sigma 0.55) clipped to [1.4 s, 15 s], the <=15 s subset the
    MLPerf QSL uses (mlperf.conf:13, 2513 samples)."""
    rng = np.random.default_rng(seed)
    dur = np.exp(rng.normal(np.log(6.2), 0.55, size=count))
    frames = np.clip(np.round(dur / 0.03), min_frames, max_frames).astype(np.int32)
    return frames


def uniform_lengths(count, seed, lo=47, hi=R.MAX_FEA_LEN):
    rng = np.random.default_rng(seed)
    return rng.integers(lo, hi + 1, size=count).astype(np.int32)


def wav_lengths_for_frames(frames, seed):
    """Sample counts whose spliced feature length is exactly frames[i]:
    ceil((floor(L/160) + 1) / 3) = T  <=>  480 (T-1) <= L < 480 T  (features.py:212, :237)."""
    rng = np.random.default_rng(seed)
    f = np.asarray(frames, np.int64)
    return (480 * (f - 1) + rng.integers(0, 480, size=f.shape)).astype(np.int32)


def make_wavs(lengths, seed, device="cpu"):
    """Speech-shaped synthetic 16 kHz audio, one float32 torch tensor per length on `device`:
    voiced segments of 80-400 ms (f0 90-250 Hz with drift, 4 harmonics, random spectral tilt),
    unvoiced noise bursts and exact-zero pauses (which exercise the dither floor), under a
    per-segment amplitude envelope in roughly [-1, 1] like librosa's float loads."""
    import torch
    rng = np.random.default_rng(seed)
    out = []
    for L in np.asarray(lengths, np.int64):
        L = int(L)
        if L == 0:
            out.append(torch.zeros(0, dtype=torch.float32, device=device))
            continue
        bounds, t = [0], 0
        while t < L:
            t = min(L, t + int(rng.integers(1280, 6400)))
            bounds.append(t)
        nseg = len(bounds) - 1
        kind = rng.choice(3, size=nseg, p=[0.7, 0.2, 0.1])  # voiced / noise / silence
        seg_id = np.repeat(np.arange(nseg), np.diff(bounds))
        f0 = rng.uniform(90.0, 250.0, nseg)
        drift = rng.uniform(-0.5, 0.5, nseg)
        amp = np.exp(rng.uniform(np.log(0.01), np.log(0.5), nseg))
        tilt = rng.uniform(0.3, 0.9, nseg)
        g = torch.Generator().manual_seed(int(rng.integers(0, 2 ** 31)))
        noise = torch.randn(L, generator=g).to(device)
        sid = torch.from_numpy(seg_id).to(device)
        pos = torch.arange(L, device=device, dtype=torch.float64)
        start = torch.from_numpy(np.asarray(bounds[:-1], np.float64)).to(device)[sid]
        tt = (pos - start) / 16000.0
        f = torch.from_numpy(f0).to(device)[sid] * (1.0 + torch.from_numpy(drift).to(device)[sid] * tt)
        phase = 2.0 * math.pi * torch.cumsum(f / 16000.0, 0)
        til = torch.from_numpy(tilt).to(device)[sid]
        voiced = sum(til ** k * torch.sin(phase * (k + 1)) for k in range(4))
        k_t = torch.from_numpy(kind).to(device)[sid]
        sig = torch.where(k_t == 0, voiced + 0.05 * noise.double(), 0.6 * noise.double())
        sig = torch.where(k_t == 2, torch.zeros_like(sig), sig)
        sig = sig * torch.from_numpy(amp).to(device)[sid]
        out.append(sig.clamp(-1.0, 1.0).float())
    return out
