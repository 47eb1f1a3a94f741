"""CPU restatement (numpy, float64) of the reference's audio front end.

TEST INFRASTRUCTURE ONLY: imported by tests/ and bench.py's checks -- never by the product
package (rnnt_amd.featurizer runs the HIP kernels and has no CPU path).

Follows FilterbankFeatures.forward (reference datasets/parts/features.py:185-252) with the
configs/rnnt.toml [input_eval] geometry.  The torch stages (torch.stft :202-210, baddbmm :224-226,
log :229-230) are pinned by tests/test_featurizer_oracle.py against torch itself on the same
arguments.  The four plugin stages live in the absent intel_mlperf library, so their semantics are
restated from their readable counterparts and the call-site arguments ("parity unpinned"):
  * preemphasis(x, x_lens, coeff, pad_size=n_fft//2) (:196-199): y[0] = x[0],
    y[t] = x[t] - coeff x[t-1] for t < len; then torch.stft(center=True)'s reflect padding of
    pad_size on both sides -- per row, at the row's own length (periodic mirror for rows shorter
    than the pad);
  * power_spectrum(x, x_lens) (:215): |X|^2 for the row's first floor(len/hop)+1 frames;
  * frame_splicing(x, x_lens, 3) (:232-235): splice_frames (:80-93) -- spliced frame j holds
    frames 3j, 3j+1, 3j+2; frames past the row's length contribute zeros;
  * i_layernorm_pad(x, 1, 0, x_lens, eps=1e-12, unbiased=1, output_shape) (:239-250): per row and
    channel over the row's ceil(F/3) valid frames, (x - mean) / sqrt(var_unbiased + eps), var = 0
    for a single frame; zero in pad channels 240..255, past the length and in pad rows.
"""
import numpy as np

HOP, WIN, NFFT, NMEL, SPLICE, FEAT, FEAT_PAD = 160, 320, 512, 80, 3, 240, 256


def frames(wav_len):
    """STFT frames and spliced feature frames of a wav_len-sample row (features.py:212, :237)."""
    if wav_len <= 0:
        return 0, 0
    F = 1 + wav_len // HOP
    return F, -(-F // SPLICE)


def mirror_index(p, L):
    """torch reflect padding index, extended periodically (rows shorter than the pad)."""
    if L == 1:
        return np.zeros_like(p)
    period = 2 * (L - 1)
    m = np.mod(p, period)
    return np.where(m < L, m, period - m)


def preemphasis_padded(x, preemph=0.97, pad=NFFT // 2):
    x = np.asarray(x, np.float64)
    y = x.copy()
    y[1:] = x[1:] - preemph * x[:-1]
    idx = mirror_index(np.arange(-pad, len(x) + pad), len(x))
    return y[idx]


def power_spectrum(padded, n_frames, window):
    """|rfft(frame * window centred in n_fft)|^2 for frames f < n_frames (torch.stft center=False)."""
    w = np.zeros(NFFT)
    off = (NFFT - WIN) // 2
    w[off:off + WIN] = np.asarray(window, np.float64)
    idx = np.arange(n_frames)[:, None] * HOP + np.arange(NFFT)[None, :]
    spec = np.fft.rfft(padded[idx] * w[None, :], axis=1)
    return spec.real ** 2 + spec.imag ** 2  # [F][257]


def log_mel(power, fb, dither=1e-5, log_guard=1e-20):
    return np.log((power + dither * dither) @ np.asarray(fb, np.float64).T + log_guard)  # [F][80]


def splice(mel, T):
    F = mel.shape[0]
    out = np.zeros((T, FEAT))
    for q in range(SPLICE):
        src = np.arange(T) * SPLICE + q
        ok = src < F
        out[ok, q * NMEL:(q + 1) * NMEL] = mel[src[ok]]
    return out


def normalize(x, eps=1e-12):
    T = x.shape[0]
    mean = x.mean(axis=0)
    var = ((x - mean) ** 2).sum(axis=0) / (T - 1) if T > 1 else np.zeros(x.shape[1])
    return (x - mean) / np.sqrt(var + eps)


def featurize_row(x, window, fb, preemph=0.97, dither=1e-5, log_guard=1e-20, eps=1e-12):
    """One utterance -> normalised spliced features [T][240] (float64)."""
    F, T = frames(len(x))
    if T == 0:
        return np.zeros((0, FEAT))
    p = power_spectrum(preemphasis_padded(x, preemph), F, window)
    return normalize(splice(log_mel(p, fb, dither, log_guard), T), eps)


def featurize(wavs, window, fb, n_pad=None, T_out=None, **kw):
    """Rows -> (feats [T_out][n_pad][256] float64, lens [n_pad] int32): the engine input layout."""
    rows = [featurize_row(w, window, fb, **kw) for w in wavs]
    n_pad = n_pad or len(wavs)
    T_out = T_out or max([r.shape[0] for r in rows] + [1])
    out = np.zeros((T_out, n_pad, FEAT_PAD))
    lens = np.zeros(n_pad, np.int32)
    for n, r in enumerate(rows):
        out[:r.shape[0], n, :FEAT] = r
        lens[n] = r.shape[0]
    return out, lens
